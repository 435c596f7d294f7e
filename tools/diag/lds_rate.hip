// ds_read_b128 issue cost on gfx950: full wave vs 16 active lanes (lane & 15 < 4), broadcast
// pattern as in the LSTM exchange tiles (lanes n read row n % 4).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ void k(float* out, unsigned long long* cyc, int iters) {
  __shared__ __attribute__((aligned(16))) float buf[16 * 1024];
  for (int i = threadIdx.x; i < 16 * 1024; i += blockDim.x) buf[i] = i * 0.5f;
  __syncthreads();
  const int lane = threadIdx.x & 63, q = lane >> 4, n = lane & 15;
  const int row = MODE == 2 ? n : (n & 3);
  f32x4 acc = {0, 0, 0, 0};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int off = (row * 224 + 32 * j + 8 * q + (it & 1) * 4) ;
      f32x4 v;
      if (MODE == 1) {
        if (n < 4) v = *reinterpret_cast<const f32x4*>(&buf[off]);
        else v = acc;
      } else {
        v = *reinterpret_cast<const f32x4*>(&buf[off]);
      }
      acc += v;
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int MODE> void run(const char* name, int waves) {
  float* o; unsigned long long* c;
  (void)hipMalloc(&o, 4 * 64 * waves); (void)hipMalloc(&c, 8);
  int iters = 200;
  hipLaunchKernelGGL((k<MODE>), dim3(1), dim3(64 * waves), 0, 0, o, c, iters);
  hipLaunchKernelGGL((k<MODE>), dim3(1), dim3(64 * waves), 0, 0, o, c, iters);
  unsigned long long h;
  (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("%-28s waves=%2d: %.2f cycles per ds_read_b128 per CU\n", name, waves, (double)h / (iters * 16 * waves));
  (void)hipFree(o); (void)hipFree(c);
}
int main() {
  for (int w : {1, 4, 12}) {
    run<0>("broadcast (n%4), full exec", w);
    run<1>("16 active lanes (n<4)", w);
    run<2>("distinct rows (n), full", w);
  }
  return 0;
}
