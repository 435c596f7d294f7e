// LayerNorm over the last dimension (y = (x - mean) / sqrt(var + eps) * gamma + beta) for gfx950.
//
// The reference normalises with BatchNorm1d only; BASELINE.json's north
// star lists LayerNorm among the hand-written kernels, so it is an optional classifier norm here
// (config `norm_layer = "layer"`, models/ica.py / models/fs.py) with its own fused kernels:
//
//   forward   one wave per row: the lane's 16-B vectors of the row stay in VGPRs, two wave
//             reductions (mean, then the centred sum of squares -- no E[x^2] - mean^2
//             cancellation), one pass out; mean / rstd saved per row for the backward;
//   backward  one wave per row again: dx = rstd (g dy - mean(g dy) - xhat mean(g dy xhat)) from the
//             registers, and each workgroup accumulates d gamma = sum dy xhat, d beta = sum dy
//             over ITS rows (the rows of a workgroup: a grid-stride loop) into a partial row;
//   reduce    the workgroup partials summed in a fixed order (deterministic, no float atomics).
//
// Rows of up to 64 lanes x 4 x LN_KMAX = 2,048 elements (D % 4 == 0: 16-B vectors), fp32.
#include "common.h"

namespace {

constexpr int LN_KMAX = 8;    // 16-B vectors per lane: D <= 2048 (16 spilled in the backward)
constexpr int LN_WAVES = 4;   // rows in flight per workgroup

__device__ __forceinline__ float ln_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int K>
__global__ void __launch_bounds__(64 * LN_WAVES)
ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
              float* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out,
              int R, int D, float eps) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int D4 = D >> 2;
  for (int row = blockIdx.x * LN_WAVES + w; row < R; row += gridDim.x * LN_WAVES) {
    const f32x4* xr = reinterpret_cast<const f32x4*>(x + (long)row * D);
    f32x4 v[K];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = lane + 64 * k;
      v[k] = i < D4 ? xr[i] : f32x4{0.f, 0.f, 0.f, 0.f};
      s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
    }
    const float mu = ln_wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (lane + 64 * k < D4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = v[k][e] - mu;
          q += d * d;
        }
      }
    }
    const float rs = __builtin_amdgcn_rsqf(ln_wave_sum(q) / (float)D + eps);
    f32x4* yr = reinterpret_cast<f32x4*>(y + (long)row * D);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = lane + 64 * k;
      if (i < D4) {
        const f32x4 gg = g ? reinterpret_cast<const f32x4*>(g)[i] : f32x4{1.f, 1.f, 1.f, 1.f};
        const f32x4 bb = b ? reinterpret_cast<const f32x4*>(b)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (v[k][e] - mu) * rs * gg[e] + bb[e];
        yr[i] = o;
      }
    }
    if (lane == 0) {
      mean_out[row] = mu;
      rstd_out[row] = rs;
    }
  }
}

template <int K>
__global__ void __launch_bounds__(64 * LN_WAVES)
ln_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy, const float* __restrict__ g,
              const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
              float* __restrict__ dx, float* __restrict__ part, int R, int D) {
  // part: [gridDim.x][2][D] (d gamma, d beta partials of this workgroup's rows), or null
  __shared__ __attribute__((aligned(16))) float red[LN_WAVES][2][64 * 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int D4 = D >> 2;
  f32x4 pg[K], pb[K];
#pragma unroll
  for (int k = 0; k < K; ++k) pg[k] = pb[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int row = blockIdx.x * LN_WAVES + w; row < R; row += gridDim.x * LN_WAVES) {
    const f32x4* xr = reinterpret_cast<const f32x4*>(x + (long)row * D);
    const f32x4* dr = reinterpret_cast<const f32x4*>(dy + (long)row * D);
    const float mu = mean_in[row], rs = rstd_in[row];
    f32x4 xh[K], gd[K];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = lane + 64 * k;
      const bool ok = i < D4;
      const f32x4 xv = ok ? xr[i] : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 dv = ok ? dr[i] : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 gg = (ok && g) ? reinterpret_cast<const f32x4*>(g)[i] : f32x4{1.f, 1.f, 1.f, 1.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[k][e] = ok ? (xv[e] - mu) * rs : 0.f;
        gd[k][e] = ok ? gg[e] * dv[e] : 0.f;
        s1 += gd[k][e];
        s2 += gd[k][e] * xh[k][e];
        pg[k][e] += dv[e] * xh[k][e];
        pb[k][e] += dv[e];
      }
    }
    const float c1 = ln_wave_sum(s1) / (float)D, c2 = ln_wave_sum(s2) / (float)D;
    f32x4* xo = reinterpret_cast<f32x4*>(dx + (long)row * D);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = lane + 64 * k;
      if (i < D4) {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rs * (gd[k][e] - c1 - xh[k][e] * c2);
        xo[i] = o;
      }
    }
  }
  if (!part) return;
  // the 4 waves' column partials summed in wave order, one 256-column slab (k) at a time
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (64 * k * 4 >= D) break;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[w][0][4 * lane + e] = pg[k][e];
      red[w][1][4 * lane + e] = pb[k][e];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < 2 * 256; t += 64 * LN_WAVES) {
      const int which = t >> 8, col = 256 * k + (t & 255);
      if (col < D) {
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < LN_WAVES; ++q) v += red[q][which][t & 255];
        part[((long)blockIdx.x * 2 + which) * D + col] = v;
      }
    }
    __syncthreads();
  }
}

// d gamma / d beta = sum over the G workgroup partials in workgroup order (+ the existing value
// when acc != 0)
__global__ void __launch_bounds__(256)
ln_reduce_kernel(const float* __restrict__ part, int G, int D, float* __restrict__ dg,
                 float* __restrict__ db, int acc) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= 2 * D) return;
  const int which = t / D, col = t - which * D;
  float v = 0.f;
  for (int q = 0; q < G; ++q) v += part[((long)q * 2 + which) * D + col];
  float* out = which ? db : dg;
  if (out) out[col] = acc ? out[col] + v : v;
}

int ln_grid(int R) {
  const int g = (R + LN_WAVES - 1) / LN_WAVES;
  return g < 1024 ? (g > 0 ? g : 1) : 1024;
}

}  // namespace

#define DN_LN_DISPATCH(KERNEL, K, GRID, ST, ...)                                              \
  switch (K) {                                                                                \
    case 1: hipLaunchKernelGGL(KERNEL<1>, GRID, dim3(64 * LN_WAVES), 0, ST, __VA_ARGS__); break; \
    case 2: hipLaunchKernelGGL(KERNEL<2>, GRID, dim3(64 * LN_WAVES), 0, ST, __VA_ARGS__); break; \
    case 4: hipLaunchKernelGGL(KERNEL<4>, GRID, dim3(64 * LN_WAVES), 0, ST, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL(KERNEL<8>, GRID, dim3(64 * LN_WAVES), 0, ST, __VA_ARGS__); break; \
  }

static int ln_k(int D) {
  const int v = (D / 4 + 63) / 64;  // 16-B vectors per lane
  return v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : 8;
}

static bool ln_ok(const void* a, const void* b, int D) {
  return D > 0 && D % 4 == 0 && D <= 64 * 4 * LN_KMAX && ((((uintptr_t)a) | ((uintptr_t)b)) & 15) == 0;
}

// y, mean, rstd <- LayerNorm(x) over rows of D (gamma / beta may be null: no affine)
DN_API int dn_layernorm_fwd(const float* x, const float* g, const float* b, float* y, float* mean,
                            float* rstd, int R, int D, float eps, hipStream_t st) {
  if (R <= 0) return DN_OK;
  if (!ln_ok(x, y, D) || !mean || !rstd || (((uintptr_t)g | (uintptr_t)b) & 15))
    return DN_BAD_SHAPE;
  DN_LN_DISPATCH(ln_fwd_kernel, ln_k(D), dim3(ln_grid(R)), st, x, g, b, y, mean, rstd, R, D, eps);
  return dn_launch_status();
}

// workspace floats dn_layernorm_bwd needs for the d gamma / d beta partials
DN_API long dn_layernorm_ws(int R, int D) { return 2L * ln_grid(R) * D; }

// dx <- the input gradient; dg / db (each may be null) <- (acc ? += : =) the parameter
// gradients; ws: dn_layernorm_ws floats
DN_API int dn_layernorm_bwd(const float* x, const float* dy, const float* g, const float* mean,
                            const float* rstd, float* dx, float* dg, float* db, float* ws, int acc,
                            int R, int D, hipStream_t st) {
  if (R <= 0) return DN_OK;
  if (!ln_ok(x, dy, D) || !ln_ok(dx, dx, D) || (((uintptr_t)g) & 15)) return DN_BAD_SHAPE;
  const bool want = dg || db;
  if (want && !ws) return DN_BAD_SHAPE;
  const int G = ln_grid(R);
  DN_LN_DISPATCH(ln_bwd_kernel, ln_k(D), dim3(G), st, x, dy, g, mean, rstd, dx,
                 want ? ws : nullptr, R, D);
  if (want)
    hipLaunchKernelGGL(ln_reduce_kernel, dim3((2 * D + 255) / 256), dim3(256), 0, st, ws, G, D, dg,
                       db, acc);
  return dn_launch_status();
}
