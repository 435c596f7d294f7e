#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int KIND, int NACC>
__global__ void k(float* out, unsigned long long* cyc, int iters) {
  f32x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, (float)threadIdx.x};
  s16x4 a4 = {(short)threadIdx.x, 1, 2, 3}, b4 = {3, 2, 1, (short)threadIdx.x};
  bf16x8 a8, b8;
  for (int i = 0; i < 8; ++i) { a8[i] = (__bf16)(threadIdx.x * 0.01f + i); b8[i] = (__bf16)(i * 0.5f); }
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) {
      if constexpr (KIND == 0) acc[j] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a4, b4, acc[j], 0, 0, 0);
      else acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[j], 0, 0, 0);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int KIND, int NACC> void run(const char* name, int waves) {
  float* o; unsigned long long* c; hipMalloc(&o, 4 * 64 * waves * 4); hipMalloc(&c, 8 * 4);
  int iters = 1000;
  hipLaunchKernelGGL((k<KIND, NACC>), dim3(1), dim3(64 * waves), 0, 0, o, c, iters);
  hipLaunchKernelGGL((k<KIND, NACC>), dim3(1), dim3(64 * waves), 0, 0, o, c, iters);
  unsigned long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("%s waves=%d nacc=%d: %.2f cycles per MFMA per wave\n", name, waves, NACC, (double)h / (iters * NACC));
  hipFree(o); hipFree(c);
}
int main() {
  run<0, 1>("4x4x4_16b", 1); run<0, 4>("4x4x4_16b", 1); run<0, 8>("4x4x4_16b", 1);
  run<0, 4>("4x4x4_16b", 4); run<0, 4>("4x4x4_16b", 12);
  run<1, 1>("16x16x32", 1); run<1, 4>("16x16x32", 1); run<1, 4>("16x16x32", 4); run<1, 4>("16x16x32", 12);
  return 0;
}
