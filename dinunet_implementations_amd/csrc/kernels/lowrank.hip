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

// optional per-matrix "still iterating" flag (rank-dAD power iteration), null elsewhere
struct PiLayerFlag {
  int* active;
};

constexpr int MGS_LDS = 12288;  // floats of a matrix kept in LDS (48 KB): n * r <= this

__global__ void __launch_bounds__(256)
mgs_batched_kernel(float* const* __restrict__ mats, const int* __restrict__ dims, float eps,
                   const PiLayerFlag* __restrict__ skip) {
  __shared__ float red[4];
  __shared__ float sm[MGS_LDS];
  if (skip && !*skip[blockIdx.x].active) return;  // converged power-iteration layer
  float* g = mats[blockIdx.x];
  const int n = dims[3 * blockIdx.x], r = dims[3 * blockIdx.x + 1], ld = dims[3 * blockIdx.x + 2];
  // the whole [n, r] matrix in LDS when it fits (the rank-dAD / PowerSGD factors do): every dot
  // product of the sweep then reads LDS instead of making an L2 round trip
  const bool in_lds = n * r <= MGS_LDS;
  float* m = in_lds ? sm : g;
  const int lm = in_lds ? r : ld;
  if (in_lds) {
    for (int i = threadIdx.x; i < n * r; i += blockDim.x) sm[i] = g[(long)(i / r) * ld + i % r];
    __syncthreads();
  }
  for (int j = 0; j < r; ++j) {
    for (int i = 0; i < j; ++i) {
      float d = 0.f;
      for (int k = threadIdx.x; k < n; k += blockDim.x) d += m[(long)k * lm + i] * m[(long)k * lm + j];
      d = block_sum(d, red);
      for (int k = threadIdx.x; k < n; k += blockDim.x) m[(long)k * lm + j] -= d * m[(long)k * lm + i];
      __syncthreads();
    }
    float s = 0.f;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      const float v = m[(long)k * lm + j];
      s += v * v;
    }
    s = block_sum(s, red);
    const float inv = 1.f / (sqrtf(s) + eps);
    for (int k = threadIdx.x; k < n; k += blockDim.x) m[(long)k * lm + j] *= inv;
    __syncthreads();
  }
  if (in_lds)
    for (int i = threadIdx.x; i < n * r; i += blockDim.x) g[(long)(i / r) * ld + i % r] = sm[i];
}

}  // namespace

// mats: device array of float* ; dims: device int[count][3] = {rows, cols, ld}
DN_API int dn_mgs_batched(float* const* mats, const int* dims, void* unused, int count, int flags,
                          float eps, hipStream_t st) {
  if (count <= 0) return DN_OK;
  hipLaunchKernelGGL(mgs_batched_kernel, dim3(count), dim3(256), 0, st, mats, dims, eps,
                     (const PiLayerFlag*)nullptr);
  return dn_launch_status();
}

// ---------------------------------------------------------------------------------------------
// rank-dAD power iteration in gradient space, every layer of the model per launch.
//
// For each large Linear l (gradient G_l [out, in] fp32, rank r <= 16) one iteration is
//   Pc = G Q                (dn_pi_gq:   one wave per row of G, coalesced along k, wave reduce)
//   Pc = orth(Pc)           (dn_mgs_batched)
//   Qc = G^T Pc             (dn_pi_gtp:  one wave per 64 columns of G, lane = column)
//   commit                  (dn_pi_commit: one workgroup per layer; while the layer is active
//                            P_send = Pc, Q_send = Q = Qc, then active &= ||Qc-Q||/||Qc|| >= tol)
// which is the structured dAD iteration P <- orth(Delta^T (A Q)), Q <- A^T (Delta P) with
// Delta^T A evaluated once (the fused kernels already accumulate G in the grad buffer).  The
// dad_tol early stop is the device-side `active` mask: no host sync, so a step graph captures
// the whole factorisation.  After the factor all-gather, dn_pi_reconstruct writes
// G = [P_1..P_W][Q_1..Q_W]^T / W for every layer in one launch.
namespace {

struct PiLayer {
  float* G;       // [out][in] (view of the flat gradient)
  float* Pc;      // [out][r] candidate P (orthonormalised in place)
  float* Q;       // [in][r] committed Q (warm start of the next step)
  float* Qc;      // [in][r] candidate Q
  float* Psend;   // [out][r] in the send buffer
  float* Qsend;   // [in][r]
  int* active;    // 1 while the layer iterates
  int out, in, r;
  int row0, col0;  // prefix offsets: first global row (gq) / first 64-column block (gtp)
};

constexpr int PI_MAXR = 16;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int find_layer(const int* starts, int n, int x) {
  int l = 0;
  while (l + 1 < n && x >= starts[l + 1]) ++l;
  return l;
}

// grid = ceil(total_rows / 4), block 256: wave -> one row of one layer's G
__global__ void __launch_bounds__(256)
pi_gq_kernel(const PiLayer* __restrict__ L, const int* __restrict__ row_starts, int n, int total_rows) {
  const int wrow = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wrow >= total_rows) return;
  const int l = find_layer(row_starts, n, wrow);
  const PiLayer& P = L[l];
  if (!*P.active) return;
  const int row = wrow - P.row0, r = P.r;
  float acc[PI_MAXR];
#pragma unroll
  for (int c = 0; c < PI_MAXR; ++c) acc[c] = 0.f;
  const float* g = P.G + (long)row * P.in;
#pragma unroll 4
  for (int k = lane; k < P.in; k += 64) {
    const float gv = g[k];
    const float* q = P.Q + (long)k * r;
#pragma unroll
    for (int c = 0; c < PI_MAXR; ++c)
      if (c < r) acc[c] += gv * q[c];
  }
#pragma unroll
  for (int c = 0; c < PI_MAXR; ++c) {
    if (c >= r) break;
    const float s = wave_sum(acc[c]);
    if (lane == 0) P.Pc[(long)row * r + c] = s;
  }
}

// grid = total 64-column blocks, block 256: lane -> one column k of one layer's G; the four
// waves split the rows, the P rows come from LDS, partial sums meet in LDS
constexpr int GTP_LDS = 12288;  // floats of P staged (out * r <= this; larger layers read L2)

__global__ void __launch_bounds__(1024)
pi_gtp_kernel(const PiLayer* __restrict__ L, const int* __restrict__ col_starts, int n) {
  __shared__ float ps[GTP_LDS];
  __shared__ float part[15][64 * PI_MAXR];
  const int l = find_layer(col_starts, n, blockIdx.x);
  const PiLayer& P = L[l];
  if (!*P.active) return;  // converged (dad_tol): this layer's iteration is a no-op
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = P.r;
  const int k = (blockIdx.x - P.col0) * 64 + lane;
  // rows [rb, re) of this split (blockIdx.y of gridDim.y): partial sums -> Qc + split * in * r
  const int nsp = gridDim.y, sp = blockIdx.y;
  const int rb = (int)((long)P.out * sp / nsp), re = (int)((long)P.out * (sp + 1) / nsp);
  const bool kv = k < P.in;
  const int kc = kv ? k : 0;
  const bool lds = (re - rb) * r <= GTP_LDS;
  if (lds) {
    for (int i = rb * r + threadIdx.x; i < re * r; i += 1024) ps[i - rb * r] = P.Pc[i];
    __syncthreads();
  }
  // (index LDS relative to rb explicitly: a pointer below ps, even one never dereferenced,
  // leaves the LDS aperture once converted to a flat address)
  float acc[PI_MAXR];
#pragma unroll
  for (int c = 0; c < PI_MAXR; ++c) acc[c] = 0.f;
#pragma unroll 8
  for (int row = rb + w; row < re; row += 16) {
    const float gv = P.G[(long)row * P.in + kc];
    if (lds) {
      const float* p = ps + (row - rb) * r;
#pragma unroll
      for (int c = 0; c < PI_MAXR; ++c)
        if (c < r) acc[c] += gv * p[c];
    } else {
      const float* p = P.Pc + (long)row * r;
#pragma unroll
      for (int c = 0; c < PI_MAXR; ++c)
        if (c < r) acc[c] += gv * p[c];
    }
  }
  if (w > 0) {
#pragma unroll
    for (int c = 0; c < PI_MAXR; ++c) part[w - 1][c * 64 + lane] = acc[c];
  }
  __syncthreads();
  if (w == 0 && kv) {
    float* qp = P.Qc + (long)sp * P.in * r;
#pragma unroll
    for (int c = 0; c < PI_MAXR; ++c) {
      if (c >= r) break;
      float v = acc[c];
      for (int t = 0; t < 15; ++t) v += part[t][c * 64 + lane];  // fixed order
      qp[(long)k * r + c] = v;
    }
  }
}

// grid = n layers, block 256
__global__ void __launch_bounds__(256)
pi_commit_kernel(const PiLayer* __restrict__ L, float tol, int nsplit) {
  __shared__ float red[2][4];
  const PiLayer& P = L[blockIdx.x];
  if (!*P.active) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nq = P.in * P.r, np = P.out * P.r;
  float dd = 0.f, qq = 0.f;
#pragma unroll 8
  for (int i = tid; i < nq; i += 256) {
    float a = P.Qc[i];  // row-split partials of G^T Pc, summed in a fixed order
    for (int s = 1; s < nsplit; ++s) a += P.Qc[(long)s * nq + i];
    P.Qc[i] = a;
    const float b = P.Q[i];
    dd += (a - b) * (a - b);
    qq += a * a;
  }
  dd = wave_sum(dd);
  qq = wave_sum(qq);
  if (lane == 0) { red[0][w] = dd; red[1][w] = qq; }
  __syncthreads();
  const float D = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  const float Qn = red[1][0] + red[1][1] + red[1][2] + red[1][3];
#pragma unroll 8
  for (int i = tid; i < np; i += 256) P.Psend[i] = P.Pc[i];
#pragma unroll 8
  for (int i = tid; i < nq; i += 256) {
    const float v = P.Qc[i];
    P.Q[i] = v;
    P.Qsend[i] = v;
  }
  if (tid == 0 && tol > 0.f && sqrtf(D) / (sqrtf(Qn) + 1e-8f) < tol) *P.active = 0;
}

struct PiRecon {
  float* G;
  const float* P;  // gathered [W][...] base of this layer's P in site 0's send buffer
  const float* Q;
  int out, in, r;
  long start;      // first output element (prefix over layers)
};

// one thread per output element of every layer: G[row][k] = sum_s sum_c P_s[row][c] Q_s[k][c] / W
__global__ void __launch_bounds__(256)
pi_reconstruct_kernel(const PiRecon* __restrict__ R, int n, long total, long stride, int W, float inv_w) {
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    int l = 0;
    while (l + 1 < n && e >= R[l + 1].start) ++l;
    const PiRecon& X = R[l];
    const long i = e - X.start;
    const int row = (int)(i / X.in), k = (int)(i - (long)row * X.in);
    float s = 0.f;
    for (int w = 0; w < W; ++w) {
      const float* p = X.P + (long)w * stride + (long)row * X.r;
      const float* q = X.Q + (long)w * stride + (long)k * X.r;
      for (int c = 0; c < X.r; ++c) s += p[c] * q[c];
    }
    X.G[i] = s * inv_w;
  }
}

constexpr int PI_SPLITS = 1;  // row splits of G^T P (Qc holds PI_SPLITS partials)

// Modified Gram-Schmidt of a [n, r] matrix by ONE wave with the matrix in registers (lane l holds
// rows l, l+64, ...): every dot product is a wave reduction (DPP / shuffles, no barriers).  The
// same column order and arithmetic as mgs_batched_kernel up to the reduction order.
constexpr int MGSW_RPL = 12;  // rows per lane: n <= 768

__global__ void __launch_bounds__(64)
mgs_wave_kernel(float* const* __restrict__ mats, const int* __restrict__ dims, float eps,
                const PiLayerFlag* __restrict__ skip) {
  if (skip && !*skip[blockIdx.x].active) return;
  float* g = mats[blockIdx.x];
  const int n = dims[3 * blockIdx.x], r = dims[3 * blockIdx.x + 1], ld = dims[3 * blockIdx.x + 2];
  const int lane = threadIdx.x;
  float m[MGSW_RPL][PI_MAXR];
#pragma unroll
  for (int i = 0; i < MGSW_RPL; ++i) {
    const int row = lane + 64 * i;
    const int rc = row < n ? row : n - 1;  // clamped, unconditional loads (no per-load branch)
#pragma unroll
    for (int c = 0; c < PI_MAXR; ++c) {
      const float v = g[(long)rc * ld + (c < r ? c : r - 1)];
      m[i][c] = (row < n && c < r) ? v : 0.f;
    }
  }
  // fully unrolled with compile-time indices (a `break` on the runtime r would leave m[][]
  // dynamically indexed -> scratch); columns >= r are zero and skipped by predicate
#pragma unroll
  for (int j = 0; j < PI_MAXR; ++j) {
    if (j < r) {
#pragma unroll
      for (int i = 0; i < j; ++i) {
        float d = 0.f;
#pragma unroll
        for (int t = 0; t < MGSW_RPL; ++t) d += m[t][i] * m[t][j];
        d = wave_sum(d);
#pragma unroll
        for (int t = 0; t < MGSW_RPL; ++t) m[t][j] -= d * m[t][i];
      }
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < MGSW_RPL; ++t) s += m[t][j] * m[t][j];
      const float inv = 1.f / (sqrtf(wave_sum(s)) + eps);
#pragma unroll
      for (int t = 0; t < MGSW_RPL; ++t) m[t][j] *= inv;
    }
  }
#pragma unroll
  for (int i = 0; i < MGSW_RPL; ++i) {
    const int row = lane + 64 * i;
    if (row < n) {
#pragma unroll
      for (int c = 0; c < PI_MAXR; ++c)
        if (c < r) g[(long)row * ld + c] = m[i][c];
    }
  }
}

__global__ void pi_reset_kernel(const PiLayer* __restrict__ L, int n) {
  if ((int)threadIdx.x < n) *L[threadIdx.x].active = 1;
}

}  // namespace

DN_API long dn_pi_layer_size() { return (long)sizeof(PiLayer); }
DN_API long dn_pi_recon_size() { return (long)sizeof(PiRecon); }

DN_API int dn_pi_splits() { return PI_SPLITS; }

// One power iteration over every layer of the table (device arrays prepared once by the engine).
//   layers: PiLayer[n]; row_starts / col_starts: int[n] prefix tables; pc_ptrs / pc_dims: the
//   dn_mgs_batched tables of the Pc matrices; active: int[n] (each layer's PiLayer::active).
// Layers whose power iteration has converged (dad_tol) skip their work inside every launch.
DN_API int dn_pi_iterate(const void* layers, const int* row_starts, const int* col_starts, int n,
                         int total_rows, int total_colblocks, float* const* pc_ptrs,
                         const int* pc_dims, const void* active_ptrs, int max_rows, float tol,
                         int first, hipStream_t st) {
  if (n <= 0) return DN_OK;
  if (n > 256) return DN_BAD_SHAPE;
  const PiLayer* L = (const PiLayer*)layers;
  if (first) hipLaunchKernelGGL(pi_reset_kernel, dim3(1), dim3(256), 0, st, L, n);
  hipLaunchKernelGGL(pi_gq_kernel, dim3((total_rows + 3) / 4), dim3(256), 0, st, L, row_starts, n,
                     total_rows);
  if (max_rows <= 64 * MGSW_RPL)
    hipLaunchKernelGGL(mgs_wave_kernel, dim3(n), dim3(64), 0, st, pc_ptrs, pc_dims, 1e-8f,
                       (const PiLayerFlag*)active_ptrs);
  else
    hipLaunchKernelGGL(mgs_batched_kernel, dim3(n), dim3(256), 0, st, pc_ptrs, pc_dims, 1e-8f,
                       (const PiLayerFlag*)active_ptrs);
  hipLaunchKernelGGL(pi_gtp_kernel, dim3(total_colblocks, PI_SPLITS), dim3(1024), 0, st, L,
                     col_starts, n);
  hipLaunchKernelGGL(pi_commit_kernel, dim3(n), dim3(256), 0, st, L, tol, PI_SPLITS);
  return dn_launch_status();
}

// G_l = sum over W sites of P_s Q_s^T / W for every layer; `stride` = send-buffer length.
DN_API int dn_pi_reconstruct(const void* recon, int n, long total, long stride, int W,
                             hipStream_t st) {
  if (n <= 0 || total <= 0) return DN_OK;
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pi_reconstruct_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const PiRecon*)recon, n, total, stride, W, 1.f / (float)W);
  return dn_launch_status();
}
