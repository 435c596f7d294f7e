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

__device__ __forceinline__ float dn_sigmoid(float x) { return 1.f / (1.f + __expf(-x)); }

// tanh via one exp + one rcp; saturates cleanly to +-1 for large |x|.
__device__ __forceinline__ float dn_tanh(float x) {
  float e = __expf(2.f * x);
  return 1.f - 2.f / (e + 1.f);
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

static inline int dn_launch_status() {
  return hipGetLastError() == hipSuccess ? DN_OK : DN_LAUNCH_FAILED;
}
