// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of dinunet_implementations_amd.
// Written for wave64 + MFMA; no CUDA shims, no dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define DN_API extern "C" __attribute__((visibility("default")))

// Error codes returned by every launcher (0 = launched).
enum DnStatus { DN_OK = 0, DN_BAD_SHAPE = 1, DN_LAUNCH_FAILED = 2, DN_UNSUPPORTED = 3 };

// Transcendentals on the hardware units: v_exp_f32 (2^x) and v_rcp_f32 (1 ulp).  A plain
// `1.f / y` compiles to the ~10-instruction IEEE division sequence (v_div_scale/fmas/fixup),
// which made the LSTM gate phase VALU-bound at 2x the necessary instruction count.
__device__ __forceinline__ float dn_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float dn_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

constexpr float DN_LOG2E = 1.4426950408889634f;

// sigmoid(x) = 1 / (1 + 2^(-x log2 e)); saturates to 0 / 1 (rcp(inf) = 0)
__device__ __forceinline__ float dn_sigmoid(float x) { return dn_rcp(1.f + dn_exp2(-DN_LOG2E * x)); }

// tanh(x) = 1 - 2 / (2^(2x log2 e) + 1); saturates cleanly to +-1 for large |x|
__device__ __forceinline__ float dn_tanh(float x) {
  return 1.f - 2.f * dn_rcp(dn_exp2((2.f * DN_LOG2E) * x) + 1.f);
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Buffer-resource stores (gfx950 raw buffer ops, 32-bit per-lane byte offset, hardware range
// check): a lane whose offset is >= the descriptor's byte count is dropped by the hardware.  That
// masks a store WITHOUT a branch, so hipcc keeps counting vmcnt exactly across it (a divergent
// `if` around a store makes every later wait in the loop a conservative vmcnt(0)).
constexpr uint32_t DN_OOB = 0x80000000u;
// s_waitcnt immediate (gfx9 encoding) waiting for vmcnt(0) only: the builtin form is seen by
// hipcc's waitcnt bookkeeping (an asm wait is not)
constexpr int DN_VMCNT0 = 0x0F70;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dn_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void dn_store_f32x4(__amdgpu_buffer_rsrc_t r, uint32_t off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                         r, (int)off, 0, 0);
}

static inline int dn_launch_status() {
  return hipGetLastError() == hipSuccess ? DN_OK : DN_LAUNCH_FAILED;
}

// Poll limit of the in-kernel hand-off / barrier waits (head_step.hip, lowrank.hip): < 0 = each
// kernel's default (~0.1-0.2 s), else that many polls; 0 makes every wait give up at once -- the
// negative control of the runtime's hand-off check (runtime.health).  Set by dn_set_spin_limit.
extern int g_dn_spin_limit;
static inline int dn_spin_limit(int dflt) { return g_dn_spin_limit >= 0 ? g_dn_spin_limit : dflt; }

// Whole CUs left to concurrent kernels when a launch whose workgroups wait on each other is
// sized: at N > 1 sites RCCL's collective kernels (one workgroup per channel, <= 64 channels) can
// run beside a step's persistent launch on other streams.
constexpr int DN_RESERVE_CUS = 64;

// Can `blocks` workgroups of `fn` (threads, dynamic LDS) ALL be resident at once on the CUs left
// after `reserve_cus`?  The precondition of a persistent launch: a workgroup that never becomes
// resident would make its peers' spin waits time out.  (Cached per (fn, threads, lds).)
static inline bool dn_fits_resident(const void* fn, int blocks, int threads, size_t lds,
                                    int reserve_cus = DN_RESERVE_CUS) {
  static const void* c_fn = nullptr;
  static int c_threads = -1, c_per = 0, c_cus = 0;
  static size_t c_lds = 0;
  if (fn != c_fn || threads != c_threads || lds != c_lds) {
    int per = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, threads, lds) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    c_fn = fn, c_threads = threads, c_lds = lds, c_per = per, c_cus = cus;
  }
  return (long)c_per * (c_cus - reserve_cus) >= blocks;
}
