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
// One power iteration (rank-dAD) or one PowerSGD round is TWO short launches:
//
//   lr_gq      P = G Q           16 rows per block, f32 MFMA 16x16x4 over K (4 waves split K),
//                                Q staged in LDS.  PowerSGD: M = G + err is formed in the same
//                                pass and written back.  (PowerSGD all-reduces P here.)
//   lr_gtp     Pn = P R^{-1}, Q = G^T Pn
//                                16 columns per block over all rows.  Every block forms the Gram
//                                P^T P of the LDS-staged P in fp64 (a few us of redundant work
//                                instead of a serial per-layer launch), factors R^T R = P^T P
//                                (fp64 Cholesky by one wave, lane = row; a vanishing pivot drops
//                                its column) and inverts R in fp64 -- the same bits in every
//                                block -- then forms Pn in LDS by f32 MFMA and Q by f32 MFMA.  Column
//                                block 0 writes Pn (Psend).  The block commits its Q slice to
//                                Qsend with the change norms the next lr_gq turns into the
//                                dad_tol decision (`active` flag).
//
// Cholesky QR with an fp64 Gram and fp64 factor: the orthogonality loss of plain CholQR is the
// Gram's rounding times cond(P)^2, which fp64 keeps far below fp32 resolution for the condition
// numbers of these factors; the fp32 product P R^{-1} then leaves ~eps32 * cond(P).  This replaced
// a per-layer CholeskyQR2 workgroup in fp32 (two serial one-wave factorisations per iteration,
// 38 us per launch for the 768-row LSTM gradients, `tools/lowrank_bench.py`).
// Qsend is the committed Q: the next iteration's input and the next step's warm start.  The
// `active` flag (device memory) stops a converged layer without a host sync.
namespace {

constexpr int LR_MAXR = 16;
constexpr int LR_PLDS = 16384;  // floats of P staged by lr_gtp (out * r)

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
typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double shfl_d(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __shfl((int)(b & 0xffffffffLL), src, 64);
  const int hi = __shfl((int)(b >> 32), src, 64);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
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
      // every wave reduces the per-block norms the same way (lane-strided partials, butterfly):
      // one bit-identical decision in every wave and block, no serial L2 round-trip chain
      float D = 0.f, Qn = 0.f;
      for (int b = lane; b < X.n3; b += 64) { D += X.norms[2 * b]; Qn += X.norms[2 * b + 1]; }
      D = wave_sum(D);
      Qn = wave_sum(Qn);
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
  // 16 chunks per round: all their G loads are issued before the first MFMA (a K loop with a
  // few loads in flight was latency-bound: ~1 us per round trip)
  constexpr int U = 16;
  for (int kb = 4 * w; kb < in; kb += 16 * U) {
    float av[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = kb + 16 * u + kr;
      av[u] = (rv && k < in) ? grow[k] : 0.f;
    }
    if (erow) {  // PowerSGD: M = G + error feedback, kept in the gradient buffer
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = kb + 16 * u + kr;
        if (rv && k < in) {
          av[u] += erow[k];
          gw[k] = av[u];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = kb + 16 * u + kr;
      const float bv = (k < in && c < r) ? q[k * r + c] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv, acc, 0, 0, 0);
    }
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

// grid = sum of n3, block 256: 16 columns of one layer per block, all rows.  Q[16 cols] =
// G[:, 16 cols]^T Pn on the matrix cores: lane l feeds A[l & 15][k] = G[r0 + k][16 cb + (l & 15)]
// (coalesced along the row) and B[k][l & 15] = Pn[r0 + k][l & 15], k = l >> 4; the 4 waves
// take interleaved 4-row chunks and meet in LDS.  The commit rides here: the new Q slice
// replaces Qsend, and the block's ||Q - Q_prev||^2, ||Q||^2 go to `norms` for the next lr_gq.
__global__ void __launch_bounds__(256)
lr_gtp_kernel(const LrLayer* __restrict__ Ls, int nl, int it) {
  __shared__ float ps[LR_PLDS];
  __shared__ float red[4 * 256];
  __shared__ double gm[256];
  __shared__ double gpart[4 * 256];
  __shared__ double rdiag[LR_MAXR];
  __shared__ float Ri[LR_MAXR * LR_MAXR];
  __shared__ float nrm[2][4];
  int l = 0;
  while (l + 1 < nl && (int)blockIdx.x >= Ls[l + 1].b3) ++l;
  const LrLayer& X = Ls[l];
  if (it > 0 && !*X.active) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = X.r, n = X.out;
  const int cb = blockIdx.x - X.b3;
  const int c = lane & 15, kr = lane >> 4;
  if (((n * r) & 3) == 0) {
    const f32x4* src = reinterpret_cast<const f32x4*>(X.P);
#pragma unroll 8
    for (int i = tid; i < n * r / 4; i += 256) reinterpret_cast<f32x4*>(ps)[i] = src[i];
  } else {
    for (int i = tid; i < n * r; i += 256) ps[i] = X.P[i];
  }
  __syncthreads();
  {  // Gram P^T P on the fp64 matrix cores (fp32 values, exact products): for 16x16x4 f64 lane l
     // holds A[l & 15][k = l >> 4] = P[row k][col l & 15] and B[k][l & 15] -- the same value
     // (C: row (l >> 4) + 4 reg, col l & 15 -- the f64 map, not the f32 one);
     // wave w takes every 4th block of 4 rows, the four partials meet in LDS in a fixed order
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    const int c = lane & 15, kr = lane >> 4;
    for (int rb = 4 * w; rb < n; rb += 16) {
      const int row = rb + kr;
      const double v = (row < n && c < r) ? (double)ps[row * r + c] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, acc, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) gpart[w * 256 + (kr + 4 * j) * 16 + c] = acc[j];  // f64 C map
  }
  __syncthreads();
  gm[tid] = (gpart[tid] + gpart[256 + tid]) + (gpart[512 + tid] + gpart[768 + tid]);
  __syncthreads();
  if (w == 0) {
    // wave 0: lane i < r holds row i of the Gram; right-looking Cholesky, upper R (R^T R = A),
    // row k of R in lane k; then R^{-1} by back substitution, lane j = column j
    double a[LR_MAXR];
#pragma unroll
    for (int jj = 0; jj < LR_MAXR; ++jj) a[jj] = (lane < r && jj < r) ? gm[(lane & 15) * 16 + jj] : 0.0;
    double dmax = 0.0;
#pragma unroll
    for (int jj = 0; jj < LR_MAXR; ++jj) dmax = fmax(dmax, jj < r ? gm[jj * 17] : 0.0);
    const double thr = fmax(1e-13 * dmax, 1e-280);
    unsigned dead = 0;
#pragma unroll
    for (int k = 0; k < LR_MAXR; ++k) {
      if (k < r) {
        const double akk = shfl_d(a[k], k);
        const bool dk = akk <= thr;  // vanished pivot: drop column k
        const double inv = dk ? 0.0 : 1.0 / sqrt(akk);
        if (dk) dead |= 1u << k;
        if (lane == k) {
#pragma unroll
          for (int jj = 0; jj < LR_MAXR; ++jj)
            a[jj] = jj == k ? (dk ? 1.0 : akk * inv) : (jj > k ? a[jj] * inv : 0.0);
          rdiag[k] = inv;
        }
        double rk[LR_MAXR];
#pragma unroll
        for (int jj = 0; jj < LR_MAXR; ++jj) rk[jj] = (jj > k && jj < r) ? shfl_d(a[jj], k) : 0.0;
        double rki = 0.0;
#pragma unroll
        for (int jj = 0; jj < LR_MAXR; ++jj) rki = lane == jj ? rk[jj] : rki;
        if (lane > k && lane < r) {
#pragma unroll
          for (int jj = 0; jj < LR_MAXR; ++jj)
            if (jj > k) a[jj] -= rki * rk[jj];
        }
      }
    }
    // R row-major through LDS (gm is free now: every lane has read its Gram row)
    if (lane < r) {
#pragma unroll
      for (int jj = 0; jj < LR_MAXR; ++jj) gm[lane * LR_MAXR + jj] = a[jj];
    }

    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    double col[LR_MAXR];
#pragma unroll
    for (int i = LR_MAXR - 1; i >= 0; --i) {
      double v = 0.0;
      if (i < r && i <= lane && lane < r) {
        v = i == lane ? 1.0 : 0.0;
#pragma unroll
        for (int k = i + 1; k < LR_MAXR; ++k)
          if (k <= lane) v -= gm[i * LR_MAXR + k] * col[k];
        v *= rdiag[i];  // 1 / R_ii (0 for a dropped column)
      }
      col[i] = (dead >> lane & 1u) ? 0.0 : v;
    }
    if (lane < LR_MAXR) {
#pragma unroll
      for (int i = 0; i < LR_MAXR; ++i) Ri[i * LR_MAXR + lane] = lane < r ? (float)col[i] : 0.f;
    }
  }
  __syncthreads();
  // Pn = P R^{-1} in place, f32 MFMA: 16-row blocks, K = 16 in four 16x16x4 steps; lane l feeds
  // A[l & 15][k = l >> 4] = P[row][4 s + k] and B[k][l & 15] = R^{-1}[4 s + k][l & 15]
  for (int b0 = 16 * w; b0 < n; b0 += 64) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int row = b0 + c;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int k = 4 * st + kr;
      const float av = (row < n && k < r) ? ps[row * r + k] : 0.f;
      const float bv = Ri[k * LR_MAXR + c];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
    // a block's 16 rows are read only by the wave that rewrites them
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int orow = b0 + 4 * kr + j;
      if (orow < n && c < r) ps[orow * r + c] = acc[j];
    }
  }
  __syncthreads();
  if (cb == 0) {
    if (((n * r) & 3) == 0) {
      f32x4* dst = reinterpret_cast<f32x4*>(X.Psend);
      for (int i = tid; i < n * r / 4; i += 256) dst[i] = reinterpret_cast<const f32x4*>(ps)[i];
    } else {
      for (int i = tid; i < n * r; i += 256) X.Psend[i] = ps[i];
    }
  }
  const int col = 16 * cb + c;
  const bool cv = col < X.in;
  const float* gcol = X.G + (cv ? col : 16 * cb);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr int U = 16;  // as in lr_gq: a round's G loads all in flight before its MFMAs
  for (int rb = 4 * w; rb < n; rb += 16 * U) {
    float av[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = rb + 16 * u + kr;
      av[u] = (row < n && cv) ? gcol[(long)row * X.in] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = rb + 16 * u + kr;
      const float bv = (row < n && c < r) ? ps[row * r + c] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv, acc, 0, 0, 0);
    }
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

// rank-dAD: G = sum over the W sites of P_s Q_s^T / W for every layer, one 16 x 16 output tile
// per wave on the f32 matrix cores (16x16x4, K = r in chunks of 4 per site: lane l feeds
// A[l & 15][k] = P_s[r0 + (l & 15)][c + k] and B[k][l & 15] = Q_s[k0 + (l & 15)][c + k],
// k = l >> 4).  The tile list is every layer's tiles in order; the per-thread-element loop it
// replaced was latency-bound (17 us for the ICA layers).
__global__ void __launch_bounds__(256)
pi_reconstruct_kernel(const PiRecon* __restrict__ R, int n, long total, long stride, int W, float inv_w) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c16 = lane & 15, kq = lane >> 4;
  long ntiles = 0;
  for (int l = 0; l < n; ++l) ntiles += (long)((R[l].out + 15) / 16) * ((R[l].in + 15) / 16);
  for (long tile = blockIdx.x * 4L + w; tile < ntiles; tile += (long)gridDim.x * 4) {
    int l = 0;
    long t0 = 0;
    for (;; ++l) {
      const long nt = (long)((R[l].out + 15) / 16) * ((R[l].in + 15) / 16);
      if (tile < t0 + nt || l + 1 == n) break;
      t0 += nt;
    }
    const PiRecon& X = R[l];
    const int tn = (X.in + 15) / 16;
    const int ti = (int)(tile - t0);
    const int r0 = 16 * (ti / tn), k0 = 16 * (ti % tn);
    const int prow = r0 + c16, qrow = k0 + c16;
    const bool pv = prow < X.out, qv = qrow < X.in;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < W; ++s) {
      const float* p = X.P + (long)s * stride + (long)(pv ? prow : 0) * X.r;
      const float* q = X.Q + (long)s * stride + (long)(qv ? qrow : 0) * X.r;
      for (int c = 0; c < X.r; c += 4) {
        const int cc = c + kq;
        const float av = (pv && cc < X.r) ? p[cc] : 0.f;
        const float bv = (qv && cc < X.r) ? q[cc] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = r0 + 4 * kq + j, col = k0 + c16;
      if (row < X.out && col < X.in) X.G[(long)row * X.in + col] = acc[j] * inv_w;
    }
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
//   stage 1: lr_gtp (Pn = P R^{-1} from the fp64 Gram; Q = G^T Pn committed to Qsend)
DN_API int dn_lr_stage(const void* layers, int nl, int blocks1, int blocks3, int stage, int it,
                       float tol, hipStream_t st) {
  if (nl <= 0) return DN_OK;
  if (nl > 256) return DN_BAD_SHAPE;
  const LrLayer* L = (const LrLayer*)layers;
  if (stage == 0)
    hipLaunchKernelGGL(lr_gq_kernel, dim3(blocks1), dim3(256), 0, st, L, nl, it, tol);
  if (stage == 1) hipLaunchKernelGGL(lr_gtp_kernel, dim3(blocks3), dim3(256), 0, st, L, nl, it);
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
  long blocks = (total / 256 + 3) / 4;  // ~one 16 x 16 tile per wave
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pi_reconstruct_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const PiRecon*)recon, n, total, stride, W, 1.f / (float)W);
  return dn_launch_status();
}
