// Loss heads: fused (log-)softmax + cross-entropy/NLL + argmax + input gradient, one launch.
//   ICA head (comps/icalstm/__init__.py:60-63): prob = softmax(z), loss = CE(z, y), pred = argmax
//   FS  head (comps/fs/__init__.py:54-57):      out = log_softmax(z), loss = NLL(out, y), pred
// Both share d loss / d z = (softmax(z) - onehot(y)) / B, computed in the same pass so the
// backward is a single scale.  One 256-thread workgroup; rows strided over waves, classes over
// lanes, wave64 shuffles for the row max / sum; loss reduced deterministically in LDS.
#include "common.h"

namespace {

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(256)
softmax_xent_kernel(const float* __restrict__ z, const long* __restrict__ y, int B, int C,
                    int log_out, float* __restrict__ out, float* __restrict__ dz,
                    float* __restrict__ loss, long* __restrict__ pred) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __shared__ float red[4];
  float lsum = 0.f;
  for (int r = wid; r < B; r += 4) {
    const float* zr = z + (long)r * C;
    float mx = -INFINITY;
    for (int c = lane; c < C; c += 64) mx = fmaxf(mx, zr[c]);
    mx = wave_max(mx);
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += __expf(zr[c] - mx);
    s = wave_sum(s);
    const float lse = mx + __logf(s);
    const long lab = y[r];
    // argmax (first max index, like torch.max)
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = lane; c < C; c += 64) {
      const float v = zr[c];
      if (v > bv || (v == bv && c < bi)) { bv = v; bi = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    for (int c = lane; c < C; c += 64) {
      const float lp = zr[c] - lse;
      const float p = __expf(lp);
      out[(long)r * C + c] = log_out ? lp : p;
      dz[(long)r * C + c] = (p - (c == lab ? 1.f : 0.f)) / (float)B;
    }
    if (lane == 0) {
      pred[r] = bi;
      lsum += (lab >= 0 && lab < C) ? (lse - zr[lab]) : 0.f;
    }
  }
  if (lane == 0) red[wid] = lsum;
  __syncthreads();
  if (threadIdx.x == 0) *loss = (red[0] + red[1] + red[2] + red[3]) / (float)B;
}

}  // namespace

DN_API int dn_softmax_xent(const float* z, const long* y, int B, int C, int log_out, float* out,
                           float* dz, float* loss, long* pred, hipStream_t st) {
  if (B <= 0 || C <= 0) return DN_BAD_SHAPE;
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(1), dim3(256), 0, st, z, y, B, C, log_out, out, dz,
                     loss, pred);
  return dn_launch_status();
}
