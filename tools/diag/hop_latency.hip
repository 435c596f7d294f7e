// Microbenchmark for the split-W_hh LSTM question (VERDICT r2 "next round" item 2): the
// round-trip latency of a per-time-step h hand-off between two workgroups on the SAME XCD (blocks
// b and b + 8 under round-robin placement; checked with HW_REG_XCC_ID) versus a workgroup
// barrier inside one CU.
//
// Each of two workgroups owns half of a 2 x 192-unit h vector (the ICA LSTM's per-direction
// state, 4 batch rows: 4 x 96 bf16 = 768 B per half).  Per step: write its half with write-through
// (sc1) 16-B stores, drain (s_waitcnt vmcnt(0)), publish the step number with one agent-scope
// store, poll the partner's step word with relaxed sc1 loads, then read the partner's half with
// sc1 loads (cdna_hip_programming §6 Guideline 16, first row of the sc1 table).  98 steps (S of
// the headline config); reports ns per step = one full exchange, the minimum the split recurrence
// would add on top of its (halved) MFMA phase.  The in-CU reference does the same exchange
// through LDS with one __syncthreads per step.
//
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/hop_latency tools/diag/hop_latency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

constexpr int STEPS = 98;
constexpr int HALF_BYTES = 768;     // 4 rows x 96 units x bf16
constexpr int SPIN = 1 << 22;

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

// grid = 16 blocks: blocks 0 and 8 exchange (same XCD); every other block exits.
__global__ void __launch_bounds__(256) pair_exchange(char* buf, unsigned* flags, unsigned long long* out,
                                                     unsigned* err, unsigned epoch_base) {
  const int b = blockIdx.x;
  if (b != 0 && b != 8) return;
  const int me = b == 0 ? 0 : 1, other = 1 - me;
  const int tid = threadIdx.x;
  auto rs = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 4 * HALF_BYTES, 0x00020000);
  u32x4 v = {(unsigned)tid, 1u, 2u, 3u};
  unsigned long long t0 = 0, t1 = 0;
  unsigned acc = 0;
  __syncthreads();
  if (tid == 0) t0 = __builtin_amdgcn_s_memrealtime();
  for (int s = 0; s < STEPS; ++s) {
    const unsigned ep = epoch_base + (unsigned)s + 1u;
    // publish my half: 48 lanes x 16 B = 768 B, write-through
    const int slot = (s & 1) * 2 + me;
    if (tid < HALF_BYTES / 16) __builtin_amdgcn_raw_buffer_store_b128(v, rs, slot * HALF_BYTES + 16 * tid, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_store((gu32*)(flags + 32 * me), ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int it = 0;
      while ((int)(__hip_atomic_load((gu32*)(flags + 32 * other), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - ep) < 0) {
        if (++it > SPIN) { *err = 1; break; }
      }
    }
    __syncthreads();
    const int oslot = (s & 1) * 2 + other;
    if (tid < HALF_BYTES / 16) {
      const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(rs, oslot * HALF_BYTES + 16 * tid, 0, 16);
      acc += w[0];
      v[1] = w[1] + 1u;
    }
  }
  __syncthreads();
  if (tid == 0) {
    t1 = __builtin_amdgcn_s_memrealtime();
    out[2 * me] = t1 - t0;
    out[2 * me + 1] = xcc_id();
  }
  if (acc == 0xdeadbeef) out[8] = acc;
}

// reference: the same per-step exchange between two wave groups of ONE workgroup through LDS
__global__ void __launch_bounds__(512) lds_exchange(unsigned long long* out) {
  __shared__ u32x4 img[2][2][HALF_BYTES / 16];
  const int tid = threadIdx.x, grp = tid >> 8, t = tid & 255;
  u32x4 v = {(unsigned)tid, 1u, 2u, 3u};
  unsigned acc = 0;
  unsigned long long t0 = 0;
  __syncthreads();
  if (tid == 0) t0 = __builtin_amdgcn_s_memrealtime();
  for (int s = 0; s < STEPS; ++s) {
    if (t < HALF_BYTES / 16) img[s & 1][grp][t] = v;
    __syncthreads();
    if (t < HALF_BYTES / 16) {
      const u32x4 w = img[s & 1][1 - grp][t];
      acc += w[0];
      v[1] = w[1] + 1u;
    }
  }
  __syncthreads();
  if (tid == 0) out[0] = __builtin_amdgcn_s_memrealtime() - t0;
  if (acc == 0xdeadbeef) out[1] = acc;
}

int main() {
  char* buf;
  unsigned* flags;
  unsigned* err;
  unsigned long long* out;
  hipMalloc(&buf, 4 * HALF_BYTES);
  hipMalloc(&flags, 4096);
  hipMalloc(&err, 4);
  hipMalloc(&out, 16 * sizeof(unsigned long long));
  hipMemset(flags, 0, 4096);
  hipMemset(err, 0, 4);
  const int reps = 20;
  double best = 1e30, sum = 0;
  unsigned long long h[16];
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(pair_exchange, dim3(16), dim3(256), 0, 0, buf, flags, out, err, (unsigned)(r * STEPS));
    hipDeviceSynchronize();
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    const double ns = (double)(h[0] > h[2] ? h[0] : h[2]) * 10.0 / STEPS;  // 100 MHz clock
    best = ns < best ? ns : best;
    sum += ns;
  }
  unsigned e = 0;
  hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
  printf("two-workgroup exchange (XCC %llu / %llu): %.0f ns per step best, %.0f mean (%d reps, timeout=%u)\n",
         h[1], h[3], best, sum / reps, reps, e);
  double lbest = 1e30;
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(lds_exchange, dim3(1), dim3(512), 0, 0, out);
    hipDeviceSynchronize();
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    const double ns = (double)h[0] * 10.0 / STEPS;
    lbest = ns < lbest ? ns : lbest;
  }
  printf("in-workgroup LDS exchange + barrier: %.0f ns per step best\n", lbest);
  return e != 0;
}
