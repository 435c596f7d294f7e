// Fused optimizer kernels over ONE flat fp32 parameter buffer (all of a model's tensors are views
// into it), so a whole optimizer step is a single launch regardless of the parameter count.
#include "common.h"

namespace {

// torch.optim.Adam semantics (L2 weight decay, no amsgrad):
//   g += wd * p;  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2
//   p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
// grad_scale folds the dSGD mean (1/world) or loss scaling into the same pass.
__global__ void __launch_bounds__(256)
adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
            float* __restrict__ v, long n, float lr, float b1, float b2, float eps, float wd,
            float bc1, float inv_sqrt_bc2, float grad_scale, const int* __restrict__ tdev,
            double b1d, double b2d, int tofs, long long* __restrict__ cursor) {
  // the device-fed batch cursor (prologue.h) advances once per update; no workgroup of this
  // launch reads it
  if (cursor && blockIdx.x == 0 && threadIdx.x == 0) *cursor += 1;
  if (tdev) {  // graph-replayable form: the step number lives on the device (adam_bump_kernel);
               // double math as on the host, so both forms round to the same fp32 corrections
    const double t = (double)(*tdev + tofs);  // tofs 0: the step prologue advanced it
    bc1 = (float)(1.0 - pow(b1d, t));
    inv_sqrt_bc2 = (float)(1.0 / sqrt(1.0 - pow(b2d, t)));
  }
  const long n4 = n >> 2;
  const float step = lr / bc1;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float gr = gg[e] * grad_scale + wd * pp[e];
      mm[e] = b1 * mm[e] + (1.f - b1) * gr;
      vv[e] = b2 * vv[e] + (1.f - b2) * gr * gr;
      pp[e] -= step * mm[e] / (sqrtf(vv[e]) * inv_sqrt_bc2 + eps);
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
  }
  // scalar tail
  const long t = (n4 << 2) + blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) {
    float gr = g[t] * grad_scale + wd * p[t];
    m[t] = b1 * m[t] + (1.f - b1) * gr;
    v[t] = b2 * v[t] + (1.f - b2) * gr * gr;
    p[t] -= step * m[t] / (sqrtf(v[t]) * inv_sqrt_bc2 + eps);
  }
}

__global__ void adam_bump_kernel(int* __restrict__ tdev) { *tdev += 1; }

// plain SGD with momentum (torch.optim.SGD semantics, dampening 0, no nesterov)
__global__ void __launch_bounds__(256)
sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf, long n,
           float lr, float momentum, float wd, float grad_scale, int first) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float d = g[i] * grad_scale + wd * p[i];
    if (momentum != 0.f) {
      float b = first ? d : momentum * buf[i] + d;
      buf[i] = b;
      d = b;
    }
    p[i] -= lr * d;
  }
}

// out = in * scale, fp32 -> bf16 (grad payload compression for precision_bits = 16)
__global__ void cast_scale_bf16_kernel(const float* __restrict__ in, bf16* __restrict__ out, long n,
                                       float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (bf16)(in[i] * scale);
}

__global__ void cast_scale_f32_kernel(const bf16* __restrict__ in, float* __restrict__ out, long n,
                                      float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (float)in[i] * scale;
}

int grid_for(long n) {
  long b = (n + 255) / 256;
  return (int)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

}  // namespace

DN_API int dn_adam(float* p, const float* g, float* m, float* v, long n, float lr, float b1,
                   float b2, float eps, float wd, float bc1, float inv_sqrt_bc2, float grad_scale,
                   long long* cursor, hipStream_t st) {
  if (n <= 0) return DN_OK;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return DN_BAD_SHAPE;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, st, p, g, m, v, n, lr,
                     b1, b2, eps, wd, bc1, inv_sqrt_bc2, grad_scale, (const int*)nullptr, 0.0, 0.0, 1, cursor);
  return dn_launch_status();
}

// Adam whose step number t is read from (and then advanced in) device memory: capturable in a
// HIP graph and replayed every step with the right bias corrections.  *tdev = completed steps.
DN_API int dn_adam_dev(float* p, const float* g, float* m, float* v, long n, float lr, double b1,
                       double b2, float eps, float wd, float grad_scale, int* tdev, int prebumped,
                       long long* cursor, hipStream_t st) {
  if (n <= 0) return DN_OK;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return DN_BAD_SHAPE;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, st, p, g, m, v, n, lr,
                     (float)b1, (float)b2, eps, wd, 0.f, 0.f, grad_scale, (const int*)tdev, b1, b2, prebumped ? 0 : 1,
                     cursor);
  if (!prebumped) hipLaunchKernelGGL(adam_bump_kernel, dim3(1), dim3(1), 0, st, tdev);
  return dn_launch_status();
}

DN_API int dn_sgd(float* p, const float* g, float* buf, long n, float lr, float momentum, float wd,
                  float grad_scale, int first, hipStream_t st) {
  if (n <= 0) return DN_OK;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, g, buf, n, lr, momentum,
                     wd, grad_scale, first);
  return dn_launch_status();
}

DN_API int dn_cast_f32_bf16(const float* in, void* out, long n, float scale, hipStream_t st) {
  if (n <= 0) return DN_OK;
  hipLaunchKernelGGL(cast_scale_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, st, in, (bf16*)out, n,
                     scale);
  return dn_launch_status();
}

DN_API int dn_cast_bf16_f32(const void* in, float* out, long n, float scale, hipStream_t st) {
  if (n <= 0) return DN_OK;
  hipLaunchKernelGGL(cast_scale_f32_kernel, dim3(grid_for(n)), dim3(256), 0, st, (const bf16*)in,
                     out, n, scale);
  return dn_launch_status();
}
