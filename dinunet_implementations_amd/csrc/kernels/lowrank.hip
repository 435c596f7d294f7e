// Batched modified Gram-Schmidt for the low-rank engines (rank-dAD P factors, PowerSGD P).
// One 256-thread workgroup per tall-skinny [n, r] fp32 matrix (r <= a few dozen); every matrix of
// a step is orthonormalised by ONE launch.  Columns are swept in order (MGS, same arithmetic order
// on every rank -> identical factors for identical inputs); dots reduce wave64 -> LDS.
#include "common.h"

namespace {

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

__global__ void __launch_bounds__(256)
mgs_batched_kernel(float* const* __restrict__ mats, const int* __restrict__ dims, float eps) {
  __shared__ float red[4];
  float* m = mats[blockIdx.x];
  const int n = dims[3 * blockIdx.x], r = dims[3 * blockIdx.x + 1], ld = dims[3 * blockIdx.x + 2];
  for (int j = 0; j < r; ++j) {
    for (int i = 0; i < j; ++i) {
      float d = 0.f;
      for (int k = threadIdx.x; k < n; k += blockDim.x) d += m[(long)k * ld + i] * m[(long)k * ld + j];
      d = block_sum(d, red);
      for (int k = threadIdx.x; k < n; k += blockDim.x) m[(long)k * ld + j] -= d * m[(long)k * ld + i];
      __syncthreads();
    }
    float s = 0.f;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      const float v = m[(long)k * ld + j];
      s += v * v;
    }
    s = block_sum(s, red);
    const float inv = 1.f / (sqrtf(s) + eps);
    for (int k = threadIdx.x; k < n; k += blockDim.x) m[(long)k * ld + j] *= inv;
    __syncthreads();
  }
}

}  // namespace

// mats: device array of float* ; dims: device int[count][3] = {rows, cols, ld}
DN_API int dn_mgs_batched(float* const* mats, const int* dims, void* unused, int count, int flags,
                          float eps, hipStream_t st) {
  if (count <= 0) return DN_OK;
  hipLaunchKernelGGL(mgs_batched_kernel, dim3(count), dim3(256), 0, st, mats, dims, eps);
  return dn_launch_status();
}
