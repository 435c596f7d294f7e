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
// Low-rank factorisation of every large Linear's gradient G [out, in], all layers per launch.
// One power iteration (rank-dAD) or one PowerSGD round is three short launches:
//
//   lr_gq      P = G Q           16 rows per block, f32 MFMA 16x16x4 over K (4 waves split K),
//                                Q staged in LDS.  PowerSGD: M = G + err is formed in the same
//                                pass and written back.
//   lr_orth    Pn = CholQR2(P)   one workgroup per layer: Gram P^T P by f32 MFMA, Cholesky by one
//                                wave in registers (lane = row of the r x r Gram, shuffles),
//                                R^{-1} by back substitution, P R^{-1} by f32 MFMA; twice
//                                (CholeskyQR2).  A pivot that vanishes (rank(P) < r) drops its
//                                column.
//   lr_gtp     Q = G^T Pn        16 columns per block over all rows, f32 MFMA, Pn in LDS; the
//                                block commits its Q slice to Qsend with the change norms the
//                                next lr_gq turns into the dad_tol decision (`active` flag)
//
// Qsend is the committed Q: the next iteration's input and the next step's warm start.  The
// `active` flag (device memory) stops a converged layer without a host sync.
namespace {

constexpr int LR_MAXR = 16;
constexpr int LR_PLDS = 16384;  // floats of P staged by lr_orth (out * r)

struct LrLayer {
  float* G;        // [out][in] gradient view (PowerSGD: becomes M = G + err)
  float* err;      // PowerSGD error feedback [out][in]; null for rank-dAD
  float* P;        // [out][r] raw G Q
  float* Psend;    // [out][r] orthonormal P (output)
  float* Qsend;    // [in][r]  committed Q: input of every iteration, output, warm start
  float* norms;    // [n3][2] per-block ||Q - Q_prev||^2, ||Q||^2 of the last lr_gtp
  int* active;     // power iteration still running
  int out, in, r;
  int b1, n1;      // lr_gq: first block, blocks (16 rows each)
  int b3, n3;      // lr_gtp: first block, blocks (16 columns each)
};

constexpr int LR_QLDS = 16384;  // floats of Q staged by lr_gq (in * r)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// grid = sum of n1, block 256: 16 rows of one layer per block.  At it > 0 the layer's dad_tol
// decision is taken here from the last commit's per-block norms (every block of the layer sums
// them in the same order: one decision everywhere); block 0 records it for the later launches.
__global__ void __launch_bounds__(256)
lr_gq_kernel(const LrLayer* __restrict__ Ls, int nl, int it, float tol) {
  __shared__ float qs[LR_QLDS];
  __shared__ float red[4 * 256];
  int l = 0;
  while (l + 1 < nl && (int)blockIdx.x >= Ls[l + 1].b1) ++l;
  const LrLayer& X = Ls[l];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = X.r, in = X.in;
  const bool lead = blockIdx.x == (unsigned)X.b1 && tid == 0;
  if (it == 0) {
    if (lead) *X.active = 1;
  } else {
    if (!*X.active) return;  // stopped at an earlier iteration
    if (tol > 0.f) {
      float D = 0.f, Qn = 0.f;
      for (int b = 0; b < X.n3; ++b) { D += X.norms[2 * b]; Qn += X.norms[2 * b + 1]; }
      if (sqrtf(D) / (sqrtf(Qn) + 1e-8f) < tol) {
        if (lead) *X.active = 0;
        return;
      }
    }
  }
  const int nq = in * r;
  const bool lds = nq <= LR_QLDS;
  if (lds) {
    if ((nq & 3) == 0) {
      const f32x4* src = reinterpret_cast<const f32x4*>(X.Qsend);
#pragma unroll 4
      for (int i = tid; i < nq / 4; i += 256) reinterpret_cast<f32x4*>(qs)[i] = src[i];
    } else {
      for (int i = tid; i < nq; i += 256) qs[i] = X.Qsend[i];
    }
  }
  __syncthreads();
  const float* q = lds ? qs : X.Qsend;
  // P[16 rows] = G[16 rows][:] Q on the matrix cores (f32 16x16x4): lane l feeds
  // A[l & 15][k] = G[row0 + (l & 15)][k0 + k] and B[k][l & 15] = Q[k0 + k][l & 15], k = l >> 4;
  // the 4 waves take interleaved 4-column chunks of K and meet in LDS
  const int row0 = 16 * (blockIdx.x - X.b1);
  const int c = lane & 15, kr = lane >> 4;
  const int row = row0 + c;
  const bool rv = row < X.out;
  const float* grow = X.G + (long)(rv ? row : row0) * in;
  float* gw = X.G + (long)(rv ? row : row0) * in;
  const float* erow = X.err ? X.err + (long)(rv ? row : row0) * in : nullptr;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k0 = 4 * w; k0 < in; k0 += 16) {
    const int k = k0 + kr;
    const bool kv = k < in;
    float av = (rv && kv) ? grow[k] : 0.f;
    if (erow && rv && kv) {  // PowerSGD: M = G + error feedback, kept in the gradient buffer
      av += erow[k];
      gw[k] = av;
    }
    const float bv = (kv && c < r) ? q[k * r + c] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w * 256 + (4 * kr + j) * 16 + c] = acc[j];  // [w][i][c]
  __syncthreads();
  {
    const int i = tid >> 4, cc = tid & 15, e = i * 16 + cc;
    if (row0 + i < X.out && cc < r)
      X.P[(long)(row0 + i) * r + cc] = red[e] + red[256 + e] + red[512 + e] + red[768 + e];
  }
}

// P [n, r] in LDS <- P R^{-1}, R^T R = P^T P.  256 threads.
__device__ __forceinline__ void cholqr_lds(float* p, int n, int r, float* part, float* R,
                                           unsigned* deadp) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // Gram P^T P on the matrix cores (f32 in, exact f32 FMA chain): for 16x16x4, lane l holds
  // A[l & 15][k = l >> 4] = P[row k][col l & 15] and B[k = l >> 4][l & 15] -- the same value,
  // so one LDS read feeds both operands; each wave takes every 4th block of 4 rows
  {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int c = lane & 15, kr = lane >> 4;
    for (int rb = 4 * w; rb < n; rb += 16) {
      const int row = rb + kr;
      const float v = (row < n && c < r) ? p[row * r + c] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v, v, acc, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) part[w * 256 + (4 * kr + j) * 16 + c] = acc[j];  // [w][i][c]
  }
  __syncthreads();
  if (w == 0) {
    // wave 0: lane i < r holds row i of the Gram (fixed-order combine of the 4 partials)
    float a[LR_MAXR];
#pragma unroll
    for (int jj = 0; jj < LR_MAXR; ++jj) {
      const int e = (lane & 15) * 16 + jj;
      a[jj] = (lane < r && jj < r) ? part[e] + part[256 + e] + part[512 + e] + part[768 + e] : 0.f;
    }
    float dmax = 0.f;
#pragma unroll
    for (int jj = 0; jj < LR_MAXR; ++jj) dmax = fmaxf(dmax, __shfl(a[jj], jj, 64));
    const float thr = fmaxf(1e-9f * dmax, 1e-30f);
    unsigned dead = 0;
    // right-looking Cholesky, upper R (R^T R = A): row k of R lives in lane k
#pragma unroll
    for (int k = 0; k < LR_MAXR; ++k) {
      if (k < r) {
        const float akk = __shfl(a[k], k, 64);
        const bool dk = akk <= thr;  // vanished pivot: drop column k
        const float inv = dk ? 0.f : 1.f / sqrtf(akk);
        if (dk) dead |= 1u << k;
        if (lane == k) {
#pragma unroll
          for (int jj = 0; jj < LR_MAXR; ++jj)
            a[jj] = jj == k ? (dk ? 1.f : akk * inv) : (jj > k ? a[jj] * inv : 0.f);
        }
        float rk[LR_MAXR];
#pragma unroll
        for (int jj = 0; jj < LR_MAXR; ++jj) rk[jj] = __shfl(a[jj], k, 64);  // row k of R
        float rki = 0.f;
#pragma unroll
        for (int jj = 0; jj < LR_MAXR; ++jj) rki = lane == jj ? rk[jj] : rki;
        if (lane > k && lane < r) {
#pragma unroll
          for (int jj = 0; jj < LR_MAXR; ++jj)
            if (jj > k) a[jj] -= rki * rk[jj];
        }
      }
    }
    if (lane < r) {
#pragma unroll
      for (int jj = 0; jj < LR_MAXR; ++jj) R[lane * LR_MAXR + jj] = a[jj];
    }
    // R^{-1} (upper): lane j < r back-substitutes column j (compile-time indices, predicated);
    // a dropped column j stays zero
    float col[LR_MAXR];
#pragma unroll
    for (int i = LR_MAXR - 1; i >= 0; --i) {
      float v = 0.f;
      if (i <= lane && lane < r) {
        v = i == lane ? 1.f : 0.f;
#pragma unroll
        for (int k = i + 1; k < LR_MAXR; ++k)
          if (k <= lane) v -= R[i * LR_MAXR + k] * col[k];
        v /= R[i * LR_MAXR + i];
      }
      col[i] = (dead >> lane & 1u) ? 0.f : v;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): R reads done before it is overwritten
    if (lane < LR_MAXR) {
#pragma unroll
      for (int i = 0; i < LR_MAXR; ++i) R[i * LR_MAXR + lane] = lane < r ? col[i] : 0.f;
    }
    if (lane == 0) *deadp = dead;
  }
  __syncthreads();
  // P <- P R^{-1} on the matrix cores: 16-row blocks, K = 16 in four 16x16x4 steps; lane l
  // feeds A[l & 15][k = l >> 4] = P[row][4 s + k] and B[k][l & 15] = R^{-1}[4 s + k][l & 15]
  {
    const int c = lane & 15, kr = lane >> 4;
    for (int b0 = 16 * w; b0 < n; b0 += 64) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int row = b0 + c;
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int k = 4 * st + kr;
        const float av = (row < n && k < r) ? p[row * r + k] : 0.f;
        const float bv = R[k * LR_MAXR + c];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int orow = b0 + 4 * kr + j;
        if (orow < n && c < r) p[orow * r + c] = acc[j];
      }
    }
  }
  __syncthreads();
}

// grid = nl, block 256
__global__ void __launch_bounds__(256)
lr_orth_kernel(const LrLayer* __restrict__ Ls, int it) {
  __shared__ float ps[LR_PLDS];
  __shared__ float part[4 * 256];
  __shared__ float R[LR_MAXR * LR_MAXR];
  __shared__ unsigned dead;
  const LrLayer& X = Ls[blockIdx.x];
  if (it > 0 && !*X.active) return;
  const int tid = threadIdx.x, n = X.out, r = X.r;
  if (((n * r) & 3) == 0) {  // 16-B loads, several in flight (a scalar loop here is latency-bound)
    const f32x4* src = reinterpret_cast<const f32x4*>(X.P);
#pragma unroll 8
    for (int i = tid; i < n * r / 4; i += 256) reinterpret_cast<f32x4*>(ps)[i] = src[i];
  } else {
    for (int i = tid; i < n * r; i += 256) ps[i] = X.P[i];
  }
  __syncthreads();
  cholqr_lds(ps, n, r, part, R, &dead);  // Cholesky QR ...
  cholqr_lds(ps, n, r, part, R, &dead);  // ... twice (CholeskyQR2)
  for (int i = tid; i < n * r; i += 256) X.Psend[i] = ps[i];
}

// grid = sum of n3, block 256: 16 columns of one layer per block, all rows.  Q[16 cols] =
// G[:, 16 cols]^T Pn on the matrix cores: lane l feeds A[l & 15][k] = G[r0 + k][16 cb + (l & 15)]
// (coalesced along the row) and B[k][l & 15] = Pn[r0 + k][l & 15], k = l >> 4; the 4 waves
// take interleaved 4-row chunks and meet in LDS.  The commit rides here: the new Q slice
// replaces Qsend, and the block's ||Q - Q_prev||^2, ||Q||^2 go to `norms` for the next lr_gq.
__global__ void __launch_bounds__(256)
lr_gtp_kernel(const LrLayer* __restrict__ Ls, int nl, int it) {
  __shared__ float ps[LR_PLDS];
  __shared__ float red[4 * 256];
  __shared__ float nrm[2][4];
  int l = 0;
  while (l + 1 < nl && (int)blockIdx.x >= Ls[l + 1].b3) ++l;
  const LrLayer& X = Ls[l];
  if (it > 0 && !*X.active) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = X.r, n = X.out;
  const int cb = blockIdx.x - X.b3;
  if (((n * r) & 3) == 0) {
    const f32x4* src = reinterpret_cast<const f32x4*>(X.Psend);
#pragma unroll 8
    for (int i = tid; i < n * r / 4; i += 256) reinterpret_cast<f32x4*>(ps)[i] = src[i];
  } else {
    for (int i = tid; i < n * r; i += 256) ps[i] = X.Psend[i];
  }
  __syncthreads();
  const int c = lane & 15, kr = lane >> 4;
  const int col = 16 * cb + c;
  const bool cv = col < X.in;
  const float* gcol = X.G + (cv ? col : 16 * cb);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int r0 = 4 * w; r0 < n; r0 += 16) {
    const int row = r0 + kr;
    const bool rv = row < n;
    const float av = (rv && cv) ? gcol[(long)row * X.in] : 0.f;
    const float bv = (rv && c < r) ? ps[row * r + c] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w * 256 + (4 * kr + j) * 16 + c] = acc[j];  // [w][k][c]
  __syncthreads();
  const int i = tid >> 4, cc = tid & 15, e = i * 16 + cc, k = 16 * cb + i;
  float dd = 0.f, qq = 0.f;
  if (k < X.in && cc < r) {
    const float v = red[e] + red[256 + e] + red[512 + e] + red[768 + e];
    const float old = X.Qsend[(long)k * r + cc];
    dd = (v - old) * (v - old);
    qq = v * v;
    X.Qsend[(long)k * r + cc] = v;
  }
  dd = wave_sum(dd);
  qq = wave_sum(qq);
  if (lane == 0) { nrm[0][w] = dd; nrm[1][w] = qq; }
  __syncthreads();
  if (tid == 0) {
    X.norms[2 * cb] = nrm[0][0] + nrm[0][1] + nrm[0][2] + nrm[0][3];
    X.norms[2 * cb + 1] = nrm[1][0] + nrm[1][1] + nrm[1][2] + nrm[1][3];
  }
}

// PowerSGD: G <- P Q^T (the compressed update), err <- M - P Q^T (M = G + err from lr_gq)
__global__ void __launch_bounds__(256)
lr_recon_ef_kernel(const LrLayer* __restrict__ Ls, const long* __restrict__ starts, int nl,
                   long total) {
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    int l = 0;
    while (l + 1 < nl && e >= starts[l + 1]) ++l;
    const LrLayer& X = Ls[l];
    const long i = e - starts[l];
    const int row = (int)(i / X.in), k = (int)(i - (long)row * X.in);
    float s = 0.f;
    for (int c = 0; c < X.r; ++c) s += X.Psend[(long)row * X.r + c] * X.Qsend[(long)k * X.r + c];
    const float m = X.G[i];
    X.G[i] = s;
    if (X.err) X.err[i] = m - s;
  }
}

struct PiRecon {
  float* G;
  const float* P;  // gathered [W][...] base of this layer's P in site 0's send buffer
  const float* Q;
  int out, in, r;
  long start;      // first output element (prefix over layers)
};

// rank-dAD: one thread per output element of every layer:
// G[row][k] = sum_s sum_c P_s[row][c] Q_s[k][c] / W
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

}  // namespace

DN_API long dn_lr_layer_size() { return (long)sizeof(LrLayer); }
DN_API long dn_pi_recon_size() { return (long)sizeof(PiRecon); }
DN_API int dn_lr_limits(int* maxr, int* plds, int* qlds) {
  *maxr = LR_MAXR;
  *plds = LR_PLDS;
  *qlds = LR_QLDS;
  return DN_OK;
}

// One power iteration / PowerSGD half-round over every layer of the table.
//   stage 0: lr_gq (P = G Q; it == 0 re-activates every layer, it > 0 applies dad_tol first)
//   stage 1: lr_orth + lr_gtp (Pn = CholQR2(P); Q = G^T Pn committed to Qsend)
//   (stages 2 / 3: lr_orth / lr_gtp alone, for tools/lowrank_bench.py)
DN_API int dn_lr_stage(const void* layers, int nl, int blocks1, int blocks3, int stage, int it,
                       float tol, hipStream_t st) {
  if (nl <= 0) return DN_OK;
  if (nl > 256) return DN_BAD_SHAPE;
  const LrLayer* L = (const LrLayer*)layers;
  if (stage == 0)
    hipLaunchKernelGGL(lr_gq_kernel, dim3(blocks1), dim3(256), 0, st, L, nl, it, tol);
  if (stage == 1 || stage == 2) hipLaunchKernelGGL(lr_orth_kernel, dim3(nl), dim3(256), 0, st, L, it);
  if (stage == 1 || stage == 3)
    hipLaunchKernelGGL(lr_gtp_kernel, dim3(blocks3), dim3(256), 0, st, L, nl, it);
  return dn_launch_status();
}

// PowerSGD reconstruction + error feedback over every layer (starts: device long[nl] prefix)
DN_API int dn_lr_recon_ef(const void* layers, const long* starts, int nl, long total,
                          hipStream_t st) {
  if (nl <= 0 || total <= 0) return DN_OK;
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(lr_recon_ef_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const LrLayer*)layers, starts, nl, total);
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
