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
  int* iters;      // iterations run (cumulative, counted by lr_gq; rank-dAD dad_tol reporting)
  int out, in, r;
  int b1, n1;      // lr_gq: first block, blocks (16 rows each)
  int b3, n3;      // lr_gtp: first block, blocks (16 columns each)
};

// LR_STAMPS (diagnostic builds only): lr_gtp phase timestamps (s_memtime) of the last column
// block of every layer, [layer][8], via dn_lr_set_stamps
#ifdef LR_STAMPS
__device__ unsigned long long* lr_stamp_buf;
#define LR_STAMP(i) do { if (threadIdx.x == 0 && lr_stamp_buf && bid == X.b3 + X.n3 - 1) { \
  unsigned long long v_; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v_) :: "memory"); \
  lr_stamp_buf[(long)l * 8 + (i)] = v_; } } while (0)
#else
#define LR_STAMP(i) do { } while (0)
#endif
constexpr int LR_QLDS = 16384;  // floats of Q staged by lr_gq (in * r)
// Layer lookup by kernel argument: first block (lr_gq: b1, lr_gtp: b3) or first tile (recon) of
// each of <= LR_KMAX layers of one launch (the host cuts a larger table into launches of
// LR_KMAX layers).  A search through the device table was a chain of dependent scalar loads, one
// L2 round trip per layer before any block could start its real loads.
constexpr int LR_KMAX = 16;
struct LrIndex {
  int n;                // layers of this launch
  int first[LR_KMAX];   // absolute first block / first tile of layer j
};
// unrolled selects (a runtime index into the by-value argument would copy it to scratch)
__device__ __forceinline__ int lr_layer_of(int v, const LrIndex& ix, int* first = nullptr) {
  int l = 0, f = ix.first[0];
#pragma unroll
  for (int j = 1; j < LR_KMAX; ++j) {
    const bool in = j < ix.n && v >= ix.first[j];
    l = in ? j : l;
    f = in ? ix.first[j] : f;
  }
  if (first) *first = f;
  return l;
}
typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float rlane(float v, int k) {  // k: compile-time lane index
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
__device__ __forceinline__ double shfl_d(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __shfl((int)(b & 0xffffffffLL), src, 64);
  const int hi = __shfl((int)(b >> 32), src, 64);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

typedef const __attribute__((address_space(1))) float gfloat;  // global loads, not flat
typedef const __attribute__((address_space(1))) f32x4 gfloat4;

// LDS staging of a small fp32 matrix through registers: every thread issues all of its (clamped)
// loads up front, the caller issues its own long loads, then the stores wait only for these.
constexpr int LR_STV = 16;  // f32x4 per thread: 256 * 16 * 4 = 16384 floats
__device__ __forceinline__ void stage_load(f32x4 (&v)[LR_STV], const float* src, int nf, int tid) {
  const int n4 = nf >> 2;
#pragma unroll
  for (int j = 0; j < LR_STV; ++j) {
    const int i = tid + 256 * j;
    if (j * 256 < n4) v[j] = ((gfloat4*)src)[i < n4 ? i : n4 - 1];  // uniform: no loads past the end
  }
}
__device__ __forceinline__ void stage_store(const f32x4 (&v)[LR_STV], float* dst, int nf, int tid) {
  const int n4 = nf >> 2;
#pragma unroll
  for (int j = 0; j < LR_STV; ++j) {
    const int i = tid + 256 * j;
    if (j * 256 < n4 && i < n4) reinterpret_cast<f32x4*>(dst)[i] = v[j];
  }
}

// lr_gq body for one layer kind: VEC = 16-byte row runs (in % 4 == 0, every ICA layer), ERR =
// PowerSGD error feedback (M = G + err formed on the fly and written back to the gradient buffer),
// QL = Q staged in LDS (in * r <= LR_QLDS; a generic pointer would make every B read a flat load)
template <bool VEC, bool ERR, bool QL>
__device__ __forceinline__ void gq_main(const LrLayer& X, float* qs, float* red, int tid, int w,
                                        int bid) {
  const int lane = tid & 63, r = X.r, in = X.in;
  const int nq = in * r;
  constexpr bool lds = QL;
  const bool qvec = lds && (nq & 3) == 0;
  f32x4 qv[LR_STV];
  if (qvec) stage_load(qv, X.Qsend, nq, tid);
  const int row0 = 16 * (bid - X.b1);
  const int c = lane & 15, kr = lane >> 4;
  const int row = row0 + c;
  const bool rv = row < X.out;
  const long roff = (long)(rv ? row : row0) * in;
  typedef __attribute__((address_space(1))) float wfloat;
  typedef __attribute__((address_space(1))) f32x4 wfloat4;
  wfloat* gw = (wfloat*)(X.G + roff);  // global stores: a flat store also counts in lgkmcnt
  gfloat* grow = (gfloat*)(X.G + roff);
  gfloat* erow = (gfloat*)(X.err + (ERR ? roff : 0));
  constexpr int U = 8;
  const int nch = (in + 15) >> 4;
  // chunk j of this wave = global chunk w + 4 j; its lane run starts at column 16 ch + 4 kr.
  // issue: every load of U chunks (G and, for PowerSGD, err) goes out before any is used; fix:
  // M = G + err, written back, and the out-of-range zeroing.  (With the add and the write-back
  // inside the load loop hipcc waited for each chunk's loads before issuing the next chunk's:
  // one L2 round trip per chunk, 13.7 us for the ICA layers.)
  auto issue = [&](f32x4 (&v)[U], f32x4 (&e)[U], int j0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k0 = 16 * (w + 4 * (j0 + u)) + 4 * kr;
      if (VEC) {
        const int kk = (rv && k0 < in) ? k0 : 0;
        v[u] = ((gfloat4*)grow)[kk >> 2];
        if (ERR) e[u] = ((gfloat4*)erow)[kk >> 2];
      } else {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int k = k0 + s2, kk = (rv && k < in) ? k : 0;
          v[u][s2] = grow[kk];
          if (ERR) e[u][s2] = erow[kk];
        }
      }
    }
  };
  auto fix = [&](f32x4 (&v)[U], const f32x4 (&e)[U], int j0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k0 = 16 * (w + 4 * (j0 + u)) + 4 * kr;
      if (VEC) {
        const bool ok = rv && k0 < in;
        if (ERR) {
          v[u] += e[u];
          if (ok) ((wfloat4*)gw)[k0 >> 2] = v[u];
        }
        v[u] *= ok ? 1.f : 0.f;  // a multiply, not a select: keeps the load unconditional
      } else {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int k = k0 + s2;
          const bool ok = rv && k < in;
          if (ERR) {
            v[u][s2] += e[u][s2];
            if (ok) gw[k] = v[u][s2];
          }
          v[u][s2] *= ok ? 1.f : 0.f;
        }
      }
    }
  };
  const float cmask = c < r ? 1.f : 0.f;
  const int cc = c < r ? c : 0;
  auto mma = [&](const f32x4 (&v)[U], int j0, f32x4& acc) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k0 = 16 * (w + 4 * (j0 + u)) + 4 * kr;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int k = k0 + s2;
        // columns past `in` meet a zero A entry; the clamp keeps the read in bounds
        const int qi = (k < in ? k : 0) * r + cc;
        const float bq = (QL ? qs[qi] : ((gfloat*)X.Qsend)[qi]) * cmask;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[u][s2], bq, acc, 0, 0, 0);
      }
    }
  };
  const int nj = (nch - w + 3) >> 2;  // this wave's chunk count (scalar)
  f32x4 g0[U], g1[U], e0[U], e1[U];
  issue(g0, e0, 0);
  if (U < nj) issue(g1, e1, U);
  if (qvec) {
    stage_store(qv, qs, nq, tid);
  } else if (lds) {
    for (int i = tid; i < nq; i += 256) qs[i] = X.Qsend[i];
  }
  __syncthreads();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < nj; j += 2 * U) {
    fix(g0, e0, j);
    mma(g0, j, acc);
    if (j + 2 * U < nj) issue(g0, e0, j + 2 * U);
    if (j + U >= nj) break;
    fix(g1, e1, j + U);
    mma(g1, j + U, acc);
    if (j + 3 * U < nj) issue(g1, e1, j + 3 * U);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w * 256 + (4 * kr + j) * 16 + c] = acc[j];  // [w][i][c]
  __syncthreads();
  {
    const int i = tid >> 4, c2 = tid & 15, e = i * 16 + c2;
    if (row0 + i < X.out && c2 < r)
      X.P[(long)(row0 + i) * r + c2] = red[e] + red[256 + e] + red[512 + e] + red[768 + e];
  }
}

// grid = sum of n1, block 256: 16 rows of one layer per block.  At it > 0 the layer's dad_tol
// decision is taken here from the last commit's per-block norms (every block of the layer sums
// them in the same order: one decision everywhere); block 0 records it for the later launches.
// P[16 rows] = G[16 rows][:] Q on the matrix cores (f32 16x16x4): the K axis is cut in 16-column
// chunks, wave w taking chunks w, w + 4, ...; in a chunk lane l loads the 16-byte run
// G[row0 + (l & 15)][16 ch + 4 (l >> 4) .. + 3] and MFMA step s uses its element s with
// B[k][l & 15] = Q[16 ch + 4 (l >> 4) + s][l & 15].  Two rounds of U chunks are in flight at
// once, issued before Q is staged: one HBM round trip for a 1000-column layer instead of four.
__global__ void __launch_bounds__(256)
lr_gq_kernel(const LrLayer* __restrict__ Ls, LrIndex ix, int it, float tol) {
  __shared__ float qs[LR_QLDS];
  __shared__ float red[4 * 256];
  const int bid = (int)blockIdx.x + ix.first[0];
  const LrLayer& X = Ls[lr_layer_of(bid, ix)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: uniform loops, no exec masks
  const bool lead = bid == X.b1 && tid == 0;
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
  if (lead) *X.iters += 1;  // one writer per layer (its first block's thread 0)
  const bool vec = (X.in & 3) == 0, ql = X.in * X.r <= LR_QLDS;  // uniform per layer
#define LR_GQ(V, E) (ql ? gq_main<V, E, true>(X, qs, red, tid, w, bid) : gq_main<V, E, false>(X, qs, red, tid, w, bid))
  if (X.err) {
    if (vec) LR_GQ(true, true); else LR_GQ(false, true);
  } else {
    if (vec) LR_GQ(true, false); else LR_GQ(false, false);
  }
#undef LR_GQ
}

// Scaled Cholesky of the fp64 Gram gm (the lr_gtp_kernel factorisation), wave 0, unrolled to the
// rank bound R >= r (R x R steps instead of LR_MAXR x LR_MAXR): Rh / Sv as lp_solve reads them.
// ALLW: every wave of the workgroup runs it (the same values: a benign LDS race) with branch-free
// stores -- lanes >= LR_MAXR write the pad past Rh's LR_MAXR^2 entries / Sv's LR_MAXR, so the
// factorisation shares a basic block with the caller's MFMAs and can issue under them
template <int R, bool ALLW = false>
__device__ __forceinline__ void lp_chol(const double* gm, float* Rh, float* Sv, int r, int lane) {
  // the diagonal by broadcast LDS reads in every lane (no cross-lane max / readlane rounds); the
  // scaling D^{-1/2} only preconditions the factorisation (R = R_s D^{1/2} whatever positive D
  // is used, and lp_solve applies the same Sv), so the hardware fp64 rsq serves
  double dg[R];
#pragma unroll
  for (int i = 0; i < R; ++i) dg[i] = i < r ? gm[i * 17] : 0.0;
  double dmax = 0.0;
#pragma unroll
  for (int i = 0; i < R; ++i) dmax = fmax(dmax, dg[i]);
  const double floor_d = fmax(1e-13 * dmax, 1e-280);
  float sv[R];
  unsigned dead = 0;
#pragma unroll
  for (int jj = 0; jj < R; ++jj) {
    const bool lj = jj < r && dg[jj] > floor_d;
    sv[jj] = lj ? (float)__builtin_amdgcn_rsq(dg[jj]) : 0.f;
    dead |= (jj < r && !lj) ? 1u << jj : 0u;
  }
  const double di = lane < r ? gm[(lane & 15) * 17] : 0.0;
  const bool live = lane < r && di > floor_d;
  const double si = live ? __builtin_amdgcn_rsq(di) : 0.0;
  float av[R];
#pragma unroll
  for (int jj = 0; jj < R; ++jj)
    av[jj] = (lane < r && jj < r) ? (float)(gm[(lane & 15) * 16 + jj] * si) * sv[jj] : 0.f;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const float akk = rlane(av[k], k);
    const bool dk = ((dead >> k) & 1u) || akk <= 1e-6f;
    const float inv = dk ? 0.f : __builtin_amdgcn_rsqf(akk);
    dead |= dk ? 1u << k : 0u;
    const float rki = av[k] * inv;
    const float rv = lane > k ? rki : (lane == k ? inv : 0.f);
    if constexpr (ALLW)
      Rh[lane < LR_MAXR ? k * LR_MAXR + lane : LR_MAXR * LR_MAXR + lane - LR_MAXR] = rv;
    else if (lane < LR_MAXR)
      Rh[k * LR_MAXR + lane] = rv;
    const float sk = rki * inv;
#pragma unroll
    for (int jj = k + 1; jj < R; ++jj) av[jj] = __builtin_fmaf(-sk, rlane(av[jj], k), av[jj]);
  }
  if constexpr (ALLW)
    Sv[lane] = lane < R ? (float)si : 0.f;
  else if (lane < LR_MAXR)
    Sv[lane] = lane < R ? (float)si : 0.f;
}

// Forward substitution x <- x D^{-1/2} R_s^{-1} for one row held in registers, bounded by R
// (entries >= R of x stay untouched: zero on entry, never read): Rh[k][m] = R_s[k][m] above the
// diagonal, Rh[k][k] = 1 / R_s[k][k] (0 for a dropped column), zeros below; Sv = D^{-1/2}.
// Uniform LDS reads (broadcast); right-looking so the chain per step is one FMA.
template <int R>
__device__ __forceinline__ void lp_solve(float (&x)[LR_MAXR], const float* Rh, const float* Sv) {
#pragma unroll
  for (int jj = 0; jj < R; ++jj) x[jj] *= Sv[jj];
#pragma unroll
  for (int jj = 0; jj < R; ++jj) {
    float rw[LR_MAXR];
#pragma unroll
    for (int q4 = 0; q4 < (R + 3) / 4; ++q4) {  // (entries >= R read, never used)
      const f32x4 v = reinterpret_cast<const f32x4*>(Rh + jj * LR_MAXR)[q4];
      rw[4 * q4] = v[0]; rw[4 * q4 + 1] = v[1]; rw[4 * q4 + 2] = v[2]; rw[4 * q4 + 3] = v[3];
    }
    x[jj] *= rw[jj];
#pragma unroll
    for (int mm = jj + 1; mm < R; ++mm) x[mm] = __builtin_fmaf(-x[jj], rw[mm], x[mm]);
  }
}

// grid = sum of n3, block 256: 16 columns of one layer per block, all rows.  Q[16 cols] =
// G[:, 16 cols]^T Pn with Pn = P R^{-1} is computed as (G^T P) R^{-1}: the G^T P product does not
// wait for the factorisation, so its column loads are issued at the top of the kernel and land
// while P is staged and the Gram formed; R^{-1} is then applied to the 16 x r result by forward
// substitution (no explicit inverse, no n-row apply pass).  Column block 0 alone forms Pn (Psend)
// by the same substitution over P's rows.  G^T P on the matrix cores: lane l feeds
// A[l & 15][k] = G[r0 + k][16 cb + (l & 15)] (coalesced along the row) and B[k][l & 15] =
// P[r0 + k][l & 15], k = l >> 4; the 4 waves take interleaved 4-row chunks and meet in LDS.  The
// commit rides here: the new Q slice replaces Qsend, and the block's ||Q - Q_prev||^2, ||Q||^2
// go to `norms` for the next lr_gq.
template <int R>  // rank bound: r <= R in {4, 8, 16} for every layer of the launch
__global__ void __launch_bounds__(256)
lr_gtp_kernel(const LrLayer* __restrict__ Ls, LrIndex ix, int it) {
  __shared__ __attribute__((aligned(16))) float ps[LR_PLDS];
  __shared__ float red[4 * 256];
  __shared__ double gm[256];
  __shared__ double gpart[4 * 256];
  __shared__ __attribute__((aligned(16))) float Rh[LR_MAXR * LR_MAXR];
  __shared__ float Sv[LR_MAXR];
  const int bid = (int)blockIdx.x + ix.first[0];
  const int l = lr_layer_of(bid, ix);
  const LrLayer& X = Ls[l];
  if (it > 0 && !*X.active) return;
  LR_STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, r = X.r, n = X.out;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: uniform loops, no exec masks
  const int cb = bid - X.b3;
  const int c = lane & 15, kr = lane >> 4;
  const int col = 16 * cb + c;
  const bool cv = col < X.in;
  gfloat* gcol = (gfloat*)(X.G + (cv ? col : 16 * cb));
  // P's loads go out first (registers, then LDS): in-order vmcnt lets the LDS staging wait for
  // them alone while the G column loads behind them are still in flight, so the Gram below runs
  // under the G loads instead of after them
  const int n4 = (n * r) >> 2;
  const bool pvec = ((n * r) & 3) == 0;
  f32x4 pv[LR_STV];
  if (pvec) {
#pragma unroll
    for (int j = 0; j < LR_STV; ++j) {
      const int i = tid + 256 * j;
      if (j * 256 < n4) pv[j] = ((gfloat4*)X.P)[i < n4 ? i : n4 - 1];  // uniform: none past P's end
    }
  }
  // the first two rounds of this wave's G^T P column loads: in flight from here on (double
  // buffered below -- a load-then-MFMA loop exposed one HBM round trip per round)
  constexpr int U = 16;
  float g0[U], g1[U];
  auto load = [&](float (&v)[U], int rb) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = rb + 16 * u + kr;
      // clamped load, zeroed by a multiply: with a select hipcc sinks the load into an
      // exec-mask branch (and the LDS reads below each into a serialised lgkmcnt(0) wait)
      v[u] = gcol[(long)(row < n ? row : 0) * X.in] * ((row < n && cv) ? 1.f : 0.f);
    }
  };
  const float cmask = c < r ? 1.f : 0.f;
  auto mma = [&](const float (&v)[U], int rb, f32x4& acc) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = rb + 16 * u + kr;
      // rows past n meet a zero A entry; columns past r give H columns the solve ignores
      const float pw = ps[(row < n ? row : 0) * r + (c < r ? c : 0)] * cmask;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[u], pw, acc, 0, 0, 0);
    }
  };
  const int rb0 = 4 * w;
  load(g0, rb0);
  if (rb0 + 16 * U < n) load(g1, rb0 + 16 * U);
  if (pvec) {
#pragma unroll
    for (int j = 0; j < LR_STV; ++j) {
      const int i = tid + 256 * j;
      if (j * 256 < n4 && i < n4) reinterpret_cast<f32x4*>(ps)[i] = pv[j];
    }
  } else {
    for (int i = tid; i < n * r; i += 256) ps[i] = X.P[i];
  }
  __syncthreads();
  LR_STAMP(1);
  // Gram P^T P on the fp64 matrix cores (fp32 values, exact products), NG = 16 / RG row groups
  // packed side by side in the 16 columns (RG = 4 for r <= 4, 8 for r <= 8, else 16): lane l
  // holds A[i][k] = P[row(g, k)][c'] with i = l & 15 = g RG + c', k = l >> 4, row(g, k) = base +
  // 4 g + k, and B[k][i] the same value, so C's diagonal RG x RG block g is the Gram of group g's
  // rows -- one MFMA covers 4 NG rows.  (C map of 16x16x4 f64: row (l >> 4) + 4 reg, col l & 15.)
  // Wave w takes every 4th block of 4 NG rows; the partials of the waves and groups are added in
  // a fixed order.  The loop is uniform (scalar wave id and trip count) with unconditional clamped
  // LDS reads: a divergent loop made hipcc shuttle the accumulators between AGPRs and VGPRs every
  // iteration (19k cycles for 768 rows)
  constexpr int RG = R <= 4 ? 4 : R <= 8 ? 8 : 16, NG = 16 / RG, RB = 4 * NG;
  {
    const int gi = c / RG, cc = c % RG;
    const float vmask = cc < r ? 1.f : 0.f;
    const int ccl = cc < r ? cc : 0;
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    const int iters = (n - RB * w + 4 * RB - 1) / (4 * RB);  // scalar trip count
    int it2 = 0;
    for (; it2 + 4 <= iters; it2 += 4) {  // four MFMAs' reads in flight per round
      float x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = RB * w + 4 * RB * (it2 + j) + 4 * gi + kr;
        x[j] = ps[(row < n ? row : 0) * r + ccl] * (row < n ? vmask : 0.f);  // clamped reads
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64((double)x[j], (double)x[j], acc, 0, 0, 0);
    }
    for (; it2 < iters; ++it2) {
      const int row = RB * w + 4 * RB * it2 + 4 * gi + kr;
      const float x = ps[(row < n ? row : 0) * r + ccl] * (row < n ? vmask : 0.f);
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64((double)x, (double)x, acc, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) gpart[w * 256 + (kr + 4 * j) * 16 + c] = acc[j];
  }
  LR_STAMP(2);
  {  // H = G[:, 16 cols]^T P, rounds of 16 chunks, two buffers in flight
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int rb = rb0; rb < n; rb += 32 * U) {
      mma(g0, rb, acc);
      if (rb + 32 * U < n) load(g0, rb + 32 * U);
      if (rb + 16 * U >= n) break;
      mma(g1, rb + 16 * U, acc);
      if (rb + 48 * U < n) load(g1, rb + 48 * U);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) red[w * 256 + (4 * kr + j) * 16 + c] = acc[j];  // [w][k][c]
  }
  __syncthreads();
  LR_STAMP(3);
  {
    const int i = tid >> 4, j = tid & 15;
    double v = 0.0;
    if (i < RG && j < RG) {
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int e = (g * RG + i) * 16 + g * RG + j;
        v += (gpart[e] + gpart[256 + e]) + (gpart[512 + e] + gpart[768 + e]);
      }
    }
    gm[tid] = v;
  }
  red[tid] = red[tid] + red[256 + tid] + red[512 + tid] + red[768 + tid];  // H[k][c], own entry
  __syncthreads();
  LR_STAMP(4);
  if (w == 0) {
    // wave 0, lane i < r = row i.  Jacobi scaling in fp64: A_s = D^{-1/2} A D^{-1/2} has a unit
    // diagonal (P's columns are ~sigma_i u_i: the scaling removes nearly all of cond(A)), so the
    // Cholesky R_s^T R_s = A_s runs in fp32 on the hardware rsq / FMA units, and
    // R^{-1} = D^{-1/2} R_s^{-1} is applied by substitution (lp_chol / lp_solve, R x R steps).
    // A column whose norm vanished (d_i <= 1e-13 max d) or that is numerically dependent
    // (pivot <= 1e-6 after scaling) is dropped: its Pn and Q columns are zero.
    lp_chol<R>(gm, Rh, Sv, r, lane);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    LR_STAMP(5);
    // Q rows: lane i < 16 takes column 16 cb + i of G: q = H[i][:] D^{-1/2} R_s^{-1}
    const int k = 16 * cb + lane;
    float dd = 0.f, qq = 0.f;
    if (lane < 16) {
      const bool kv = k < X.in;
      float* qrow = X.Qsend + (long)(kv ? k : 0) * r;
      float old[R];  // the last commit, loaded before the solve (all at once, clamped)
#pragma unroll
      for (int j = 0; j < R; ++j) old[j] = ((gfloat*)qrow)[j < r ? j : 0];
      float x[LR_MAXR];
#pragma unroll
      for (int j = 0; j < LR_MAXR; ++j) x[j] = 0.f;
#pragma unroll
      for (int q4 = 0; q4 < (R + 3) / 4; ++q4) {
        const f32x4 v = reinterpret_cast<const f32x4*>(red + lane * 16)[q4];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[4 * q4 + e] = 4 * q4 + e < R ? v[e] : 0.f;
      }
      lp_solve<R>(x, Rh, Sv);
      if (kv) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
          if (j < r) {
            dd += (x[j] - old[j]) * (x[j] - old[j]);
            qq += x[j] * x[j];
            qrow[j] = x[j];
          }
        }
      }
    }
    dd = wave_sum(dd);
    qq = wave_sum(qq);
    LR_STAMP(6);
    if (lane == 0) {
      X.norms[2 * cb] = dd;
      X.norms[2 * cb + 1] = qq;
    }
    LR_STAMP(7);
  }
  if (cb == 0) {  // Psend = P D^{-1/2} R_s^{-1}, one row per thread
    __syncthreads();
    for (int row = tid; row < n; row += 256) {
      float x[LR_MAXR];
#pragma unroll
      for (int j = 0; j < LR_MAXR; ++j) x[j] = (j < R && j < r) ? ps[row * r + j] : 0.f;
      lp_solve<R>(x, Rh, Sv);
      float* prow = X.Psend + (long)row * r;
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (j < r) prow[j] = x[j];
    }
  }
}

// PowerSGD: G <- P Q^T (the compressed update), err <- M - P Q^T (M = G + err from lr_gq), one
// 16 x 16 output tile per wave on the f32 matrix cores (16x16x4, K = r in chunks of 4; operand
// lanes as in pi_reconstruct_kernel below).  The tile list is every layer's tiles in order.  The
// per-thread-element loop it replaced (layer search, 64-bit division and r dependent loads per
// element) was latency-bound: 14.6 us for the ICA layers.
__global__ void __launch_bounds__(256)
lr_recon_ef_kernel(const LrLayer* __restrict__ Ls, LrIndex ix, int ntiles) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kq = lane >> 4;
  for (int tile = blockIdx.x * 4 + w; tile < ntiles; tile += gridDim.x * 4) {
    int t0;
    const LrLayer& X = Ls[lr_layer_of(tile, ix, &t0)];
    const int tn = (X.in + 15) / 16;
    const int ti = tile - t0;
    const int r0 = 16 * (ti / tn), k0 = 16 * (ti % tn);
    const int prow = r0 + c16, qrow = k0 + c16;
    const bool pv = prow < X.out, qv = qrow < X.in;
    const float* p = X.Psend + (long)(pv ? prow : 0) * X.r;
    const float* q = X.Qsend + (long)(qv ? qrow : 0) * X.r;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < X.r; c += 4) {
      const int cc = c + kq;
      const float av = (pv && cc < X.r) ? p[cc] : 0.f;
      const float bv = (qv && cc < X.r) ? q[cc] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
    const int col = k0 + c16;
    float m[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = r0 + 4 * kq + j;
      m[j] = (row < X.out && col < X.in) ? X.G[(long)row * X.in + col] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = r0 + 4 * kq + j;
      if (row < X.out && col < X.in) {
        const long i = (long)row * X.in + col;
        X.G[i] = acc[j];
        if (X.err) X.err[i] = m[j] - acc[j];
      }
    }
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
// k = l >> 4).  The tile list is every layer's tiles in order; a tile's layer comes from the
// host-made tile prefix and layer records in the kernel arguments (no device table), and every
// factor load of a site issues before its MFMAs (r <= 16: four k chunks; a loop of load ->
// MFMA per chunk was one memory round trip each).
constexpr int PR_MAXL = 16;
struct PrIndex {
  long tstart[PR_MAXL + 1];  // first tile of each layer; tstart[n] = all tiles
  int n;
  PiRecon L[PR_MAXL];        // the layer records themselves (kernel arguments: no table load)
};

__global__ void __launch_bounds__(256)
pi_reconstruct_kernel(PrIndex ix, long stride, int W, float inv_w) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kq = lane >> 4;
  const long ntiles = ix.tstart[ix.n];
  for (long tile = blockIdx.x * 4L + w; tile < ntiles; tile += (long)gridDim.x * 4) {
    int l = 0;
#pragma unroll
    for (int j = 1; j < PR_MAXL; ++j) l += (j < ix.n && tile >= ix.tstart[j]) ? 1 : 0;
    const PiRecon& X = ix.L[l];
    const int r = X.r;
    const int tn = (X.in + 15) / 16;
    const int ti = (int)(tile - ix.tstart[l]);
    const int r0 = 16 * (ti / tn), k0 = 16 * (ti % tn);
    const int prow = r0 + c16, qrow = k0 + c16;
    const bool pv = prow < X.out, qv = qrow < X.in;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < W; ++s) {
      const float* p = X.P + (long)s * stride + (long)(pv ? prow : 0) * r;
      const float* q = X.Q + (long)s * stride + (long)(qv ? qrow : 0) * r;
      float av[4], bv[4];
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) {  // clamped loads, selected: all eight in flight at once
        const int cc = 4 * c4 + kq, ci = cc < r ? cc : r - 1;
        const float a = p[ci], b = q[ci];
        av[c4] = (pv && cc < r) ? a : 0.f;
        bv[c4] = (qv && cc < r) ? b : 0.f;
      }
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4)
        if (4 * c4 < r) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[c4], bv[c4], acc, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = r0 + 4 * kq + j, col = k0 + c16;
      if (row < X.out && col < X.in) X.G[(long)row * X.in + col] = acc[j] * inv_w;
    }
  }
}


// ---------------------------------------------------------------------------------------------
// rank-dAD power iteration, ALL iterations of ALL layers in ONE launch.
// Layer l is owned by J_l member workgroups (blocks 8 j + l: one layer's members share an XCD
// when the dispatcher deals blocks round-robin over the 8 XCDs -- for speed only, the hand-offs
// below are valid at any placement).  Member j keeps two slices of G in REGISTERS for the whole
// launch: rows [16 rb_per j, ..) x all columns (P = G Q) and all rows x columns [16 cb_per j, ..)
// (H = G^T P).  One iteration = two phases and two per-layer barriers:
//   A  P[my rows] = G[my rows] Q (Q staged in LDS from Qsend), published with sc1 stores, plus my
//      rows' partial Gram P^T P (fp64), published likewise;            -> barrier
//   B  Gram = sum of the J partials (fixed order), scaled Cholesky (wave 0, as lr_gtp), P staged
//      in LDS, H = G[:, my cols]^T P, Q[my cols] = H R^{-1} -> Qsend + change norms, Psend for my
//      rows = P R^{-1};                                                  -> barrier
// The dad_tol decision of iteration it > 0 is taken by every member from all members' norms (same
// order: one decision).  Hand-off form (MI355X_MICROARCH.md visibility table, first row): every
// byte a peer reads is stored sc1 and drained by every storing wave, one lane adds to the layer's
// arrival counter (agent-scope atomic) and polls it with sc1 loads (bounded: a timeout sets the
// error word instead of hanging), the other waves follow through a workgroup barrier, and every
// load of peer data is an sc1 buffer load.  The arrival counters count up within a launch and
// the last member to finish resets them, so every launch starts from zero.
constexpr int LP_MAXL = 8;    // layers per launch
constexpr int LP_MAXJ = 32;   // members per layer
constexpr int LP_GV = 16;     // G slice registers per lane and slice (f32x4): 64 floats / thread
constexpr int LP_RB = 4;      // row blocks per member (the phase-A reduction buffer)
constexpr int LP_LDS = 16384; // floats staged (max(in, out) * r)
constexpr int LP_SPIN = 1 << 20;  // ~0.1 s of polling before a barrier gives up

struct LpLayer {
  LrLayer X;
  int J, rb_per, cb_per;  // members, 16-row / 16-column blocks per member (powers of 2, <= 4)
  double* gram;   // [J][256] partial Grams
  float* norms;   // [J][2]
};
struct LpArgs {
  LpLayer L[LP_MAXL];
  int nl, iters;
  float tol;
  unsigned* sync;  // [LP_MAXL][64] (arrivals at 0, done at 32) + error word at [LP_MAXL * 64]
  unsigned long long* stamps;  // diagnostics (null): member 0 of layer l, [l][1 + 8 it + k]
  int spin;                    // poll limit of a barrier wait (dn_spin_limit)
};
#define LP_STAMP(k) do { if (a.stamps && j == 0 && threadIdx.x == 0) \
  a.stamps[l * 64 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t lp_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
typedef __attribute__((ext_vector_type(4))) unsigned lp_u32x4;
typedef __attribute__((address_space(1))) unsigned lp_gu32;
__device__ __forceinline__ void lp_st4(__amdgpu_buffer_rsrc_t r, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(lp_u32x4, v), r, off, 0, 16);
}
__device__ __forceinline__ void lp_st1(__amdgpu_buffer_rsrc_t r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 16);
}
__device__ __forceinline__ f32x4 lp_ld4(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}
__device__ __forceinline__ float lp_ld1(__amdgpu_buffer_rsrc_t r, int off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 16));
}

// LDS-only workgroup barrier: orders the waves and their LDS traffic without waiting for
// outstanding global stores (a __syncthreads is also a device-scope fence: each phase ending in
// global stores -- Psend, published payloads -- then waited a memory round trip); lp_barrier
// drains explicitly where peers need the stores
__device__ __forceinline__ void lp_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// every storing wave drains, one lane arrives and polls, the workgroup follows
__device__ __forceinline__ void lp_barrier(unsigned* sync, int l, unsigned target, unsigned code,
                                           int spin) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lp_sync();
  if (threadIdx.x == 0) {
    lp_gu32* c = (lp_gu32*)(sync + l * 64);
    __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int it = 0;
    for (; it < spin; ++it) {
      const unsigned v = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)(v - target) >= 0) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (it >= spin)
      __hip_atomic_store((lp_gu32*)(sync + LP_MAXL * 64), code, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  lp_sync();
}

// stage nf floats of a peer-written buffer into LDS (16-B sc1 loads; nf % 4 == 0), 8 loads per
// thread in flight per round (a load-store loop made every 16 B a serial memory round trip)
__device__ __forceinline__ void lp_stage(float* dst, __amdgpu_buffer_rsrc_t src, int nf, int tid) {
  const int n4 = nf >> 2;
  for (int i0 = 0; i0 < n4; i0 += 8 * 256) {
    f32x4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = i0 + q * 256 + tid;
      v[q] = lp_ld4(src, 16 * (i < n4 ? i : 0));
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = i0 + q * 256 + tid;
      if (i < n4) reinterpret_cast<f32x4*>(dst)[i] = v[q];
    }
  }
}

// publish rows [r0, r1) of an [., r] matrix held in LDS rows 0.. (lds row stride r) with sc1
// stores: 16-B where the flat range allows, 4-B at the ragged end
__device__ __forceinline__ void lp_publish(__amdgpu_buffer_rsrc_t dst, const float* src, int r0,
                                           int r1, int r, int tid) {
  const int e0 = r0 * r, e1 = r1 * r;  // e0 % 4 == 0 (r0 a multiple of 16)
  const int q1 = e1 & ~3;
  for (int e = e0 + 4 * tid; e < q1; e += 1024)
    lp_st4(dst, 4 * e, *reinterpret_cast<const f32x4*>(src + (e - e0)));
  for (int e = q1 + tid; e < e1; e += 256) lp_st1(dst, 4 * e, src[e - e0]);
}


// LP_BF16X3 (default 1): the G Q and G^T P products of the power iteration on bf16 matrix cores
// with each fp32 operand split into hi + lo bf16 parts (hi*hi + hi*lo + lo*hi, fp32 accumulation:
// ~1e-5 relative per product, far below the rank-r truncation the factors exist for): three
// 16x16x32 MFMAs per 32-deep chunk instead of eight dependent 16x16x4 f32 ones.  0: fp32 MFMAs.
#ifndef LP_BF16X3
#define LP_BF16X3 1
#endif
__device__ __forceinline__ void lp_split8(const float* v, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bf16 h = (bf16)v[e];
    hi[e] = h;
    lo[e] = (bf16)(v[e] - (float)h);
  }
}
__device__ __forceinline__ f32x4 lp_mfma3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                          const bf16x8& bl, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);  // small terms first
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
}

// every 64-B line of the (1+ KB) argument block requested in one round at entry: the layer's
// fields are then scalar-cache hits instead of a chain of dependent argument loads
__device__ __forceinline__ void lp_warm_kernargs() {
  constexpr int LINES = (int)((sizeof(LpArgs) + 63) / 64);
  typedef const __attribute__((address_space(4))) unsigned cu32;
  cu32* kp = (cu32*)__builtin_amdgcn_kernarg_segment_ptr();
  unsigned acc = 0;
#pragma unroll
  for (int i = 0; i < LINES; ++i) acc += kp[16 * i];
  asm volatile("" ::"s"(acc));
}

// R: rank bound, r <= R in {4, 8, 10, 12, 16} for every layer of the launch.  EX: every layer's
// rank IS R (the default: one rank for all layers), so r is a compile-time constant and every
// `e < r` below folds away -- with a run-time r the per-entry predicates were hoisted out of the
// iteration loop and spilled (hundreds of SGPRs parked in VGPR lanes, reloaded per use).
template <int R, bool EX>
__global__ void __launch_bounds__(256)
lr_persist_kernel(LpArgs a) {
  __shared__ __attribute__((aligned(16))) float stg[LP_LDS];        // Q (phase A) / P (phase B)
  __shared__ __attribute__((aligned(16))) float red[4 * 256];
  __shared__ __attribute__((aligned(16))) float mine[LP_RB * 16 * LR_MAXR];  // my P / H rows
  __shared__ float qold[LP_RB * 16 * LR_MAXR];  // my Q rows of the last commit
  __shared__ double gpart[4 * 256];
  __shared__ double gm[256];
  __shared__ __attribute__((aligned(16))) float Rh[LR_MAXR * LR_MAXR + 64 - LR_MAXR];
  __shared__ float Sv[64];
  __shared__ float dq[2 * 4];
  lp_warm_kernargs();
  const int l = blockIdx.x & (LP_MAXL - 1), j = blockIdx.x / LP_MAXL;
  if (l >= a.nl || j >= a.L[l].J) return;
  LP_STAMP(60);  // entry (the span before stamp 0: argument loads, G load issue)
  const LpLayer& Y = a.L[l];
  const LrLayer& X = Y.X;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, kr = lane >> 4;
  const int n = X.out, m = X.in, r = EX ? R : X.r, J = Y.J;
  const int cc = c < r ? c : 0;
  const float cmask = c < r ? 1.f : 0.f;
  // my row slice (phase A): row blocks [rb0, rb1), chunks (rb, ch) dealt to waves w, w+4, ...
  const int nrb = (n + 15) >> 4, nch = (m + 15) >> 4, ncb = nch;
  const int rb0 = min(nrb, j * Y.rb_per), rb1 = min(nrb, rb0 + Y.rb_per);
  const int cb0 = min(ncb, j * Y.cb_per), cb1 = min(ncb, cb0 + Y.cb_per);
  // wave -> block maps, no divisions in the loops: phase A gives each row block WA = 4 / rb_per
  // waves, which split its column chunks (wave slot i = chunk chw + WA i); phase B likewise gives
  // each column block WB waves splitting the row chunks.  Every slot runs (zero operands past the
  // edge): straight-line MFMA code the compiler can schedule
  const int WA = 4 / Y.rb_per, rbw = w / WA, chw = w % WA;
  const int WB = 4 / Y.cb_per, cbw = w / WB, rlw = w % WB;
  gfloat* G = (gfloat*)X.G;
#if LP_BF16X3
  // 32-deep chunks: lane (c, kr) holds G[row c][32 q + 8 kr .. + 7] (phase A, q = chw + WA i)
  // and G[32 q + 8 kr .. + 7][col c] (phase B, q = rlw + WB i), split into bf16 hi / lo
  constexpr int NQ = LP_GV / 2;
  bf16x8 gah[NQ], gal[NQ], gbh[NQ], gbl[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int row = 16 * (rb0 + rbw) + c;
    float v[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // m % 4 == 0: a 4-run never straddles m
      const int k0 = 32 * (chw + WA * i) + 8 * kr + 4 * h;
      const bool ok = rb0 + rbw < rb1 && row < n && k0 < m;
      const f32x4 t = ((gfloat4*)(G + (long)(ok ? row : 0) * m))[(ok ? k0 : 0) >> 2] * (ok ? 1.f : 0.f);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * h + e] = t[e];
    }
    lp_split8(v, gah[i], gal[i]);
  }
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int col = 16 * (cb0 + cbw) + c;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int row = 32 * (rlw + WB * i) + 8 * kr + e;
      const bool ok = cb0 + cbw < cb1 && row < n && col < m;
      v[e] = G[(ok ? (long)row * m + col : 0)] * (ok ? 1.f : 0.f);
    }
    lp_split8(v, gbh[i], gbl[i]);
  }
#else
  f32x4 ga[LP_GV], gb[LP_GV];
#pragma unroll
  for (int i = 0; i < LP_GV; ++i) {
    const int row = 16 * (rb0 + rbw) + c, k0 = 16 * (chw + WA * i) + 4 * kr;
    const bool ok = rb0 + rbw < rb1 && row < n && k0 < m;  // m % 4 == 0: runs never straddle m
    ga[i] = ((gfloat4*)(G + (long)(ok ? row : 0) * m))[(ok ? k0 : 0) >> 2] * (ok ? 1.f : 0.f);
  }
#pragma unroll
  for (int i = 0; i < LP_GV; ++i) {
    const int col = 16 * (cb0 + cbw) + c;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int row = 16 * (rlw + WB * i) + 4 * s2 + kr;
      const bool ok = cb0 + cbw < cb1 && row < n && col < m;
      gb[i][s2] = G[(ok ? (long)row * m + col : 0)] * (ok ? 1.f : 0.f);
    }
  }
#endif
  LP_STAMP(0);
  const __amdgpu_buffer_rsrc_t rP = lp_rsrc(X.P), rQ = lp_rsrc(X.Qsend);
  const __amdgpu_buffer_rsrc_t rG = lp_rsrc(Y.gram), rN = lp_rsrc(Y.norms);
  unsigned bar = 0;
  int it = 0;
  for (;; ++it) {
    if (j == 0 && tid == 0) *X.iters += 1;
    // ---- phase A: P[my rows] = G[my rows] Q ----
    const int sb = 1 + 10 * (it < 5 ? it : 5);
    LP_STAMP(sb);
    lp_stage(stg, rQ, (m * r + 3) & ~3, tid);
    lp_sync();
    const int ncol = min(m, 16 * cb1) - 16 * cb0;
    for (int e = tid; e < ncol * r; e += 256) qold[e] = stg[16 * cb0 * r + e];  // my Q rows now
    {
#if LP_BF16X3
      f32x4 acc2[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};  // two chains
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        float bq[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = 32 * (chw + WA * i) + 8 * kr + e;
          bq[e] = stg[(k < m ? k : 0) * r + cc] * cmask;  // k >= m meets a zero A entry
        }
        bf16x8 bh, bl;
        lp_split8(bq, bh, bl);
        acc2[i & 1] = lp_mfma3(gah[i], gal[i], bh, bl, acc2[i & 1]);
      }
      const f32x4 acc = acc2[0] + acc2[1];
#else
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < LP_GV; ++i) {
        float bq[4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int k = 16 * (chw + WA * i) + 4 * kr + s2;
          bq[s2] = stg[(k < m ? k : 0) * r + cc] * cmask;  // k >= m meets a zero A entry
        }
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[i][s2], bq[s2], acc, 0, 0, 0);
      }
#endif
#pragma unroll
      for (int e = 0; e < 4; ++e) red[w * 256 + (4 * kr + e) * 16 + c] = acc[e];
    }
    lp_sync();
    LP_STAMP(sb + 1);
    const int nr = min(n, 16 * rb1) - 16 * rb0;  // my rows
    for (int e = tid; e < (rb1 - rb0) * 256; e += 256) {
      const int rb = e >> 8, i = (e >> 4) & 15, c2 = e & 15;
      const int rr = 16 * rb + i;
      if (rr < nr && c2 < r) {  // the WA waves of row block rb, in wave order
        float v = 0.f;
        for (int q = 0; q < WA; ++q) v += red[(rb * WA + q) * 256 + i * 16 + c2];
        mine[rr * r + c2] = v;
      }
    }
    lp_sync();
    lp_publish(rP, mine, 16 * rb0, 16 * rb0 + nr, r, tid);
    {  // my rows' partial Gram on the fp64 matrix cores (fp32 values, exact products): wave w
       // takes my rows 16 w .. 16 w + 15 (<= 64 rows), lane l feeds A[l & 15][k] = B[k][l & 15] =
       // P[row k][col l & 15]; the four wave partials are added in a fixed order
      f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int rr = 16 * w + 4 * s2 + kr;
        const double v = (rr < nr && c < r) ? (double)mine[(rr < nr ? rr : 0) * r + cc] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, acc, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) gpart[w * 256 + (kr + 4 * e) * 16 + c] = acc[e];  // f64 C map
    }
    lp_sync();
    gm[tid] = (gpart[tid] + gpart[256 + tid]) + (gpart[512 + tid] + gpart[768 + tid]);
    lp_sync();
    if (tid < 128) {
      const double2 v = {gm[2 * tid], gm[2 * tid + 1]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(lp_u32x4, v), rG,
                                             (j * 256 + 2 * tid) * 8, 0, 16);
    }
    LP_STAMP(sb + 2);
    lp_barrier(a.sync, l, (++bar) * (unsigned)J, 0x100u + (unsigned)l, a.spin);
    LP_STAMP(sb + 3);
    // ---- phase B: Gram, Cholesky, H = G[:, my cols]^T P, Q[my cols], Psend[my rows] ----
    // One round of loads for both inputs of the phase: the J partial Grams (rows < r only; thread
    // t takes double2 entry t & 127 of members [h Jh, h Jh + Jh), h = t >> 7) first, then this
    // thread's share of P.  The Gram sums wait only for the Gram loads (in-order vmcnt), so wave
    // 0's Cholesky runs while the P loads are still in flight; P reaches LDS after it.  (Loading
    // the Grams, then staging P, then factorising was two round trips plus the Cholesky in series.)
    const int Jh = (J + 1) >> 1, gh = tid >> 7, gp = tid & 127;
    const bool gload = gp < 8 * r;  // double2 entries of Gram rows 0 .. r-1
    constexpr int GV = 8, PV = 8;   // registers for 16 members and 8192 floats of P; the rest
                                    // (larger tables) is loaded after, in series
    double2 gv[GV];
#pragma unroll
    for (int q = 0; q < GV; ++q) {
      // unconditional, clamped: a per-load branch (or a `break`) made hipcc wait for every load
      // at the join, or keep gv in LDS
      const int mb = gh * Jh + q;
      gv[q] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
          rG, (((gload && q < Jh && mb < J) ? mb : 0) * 256 + 2 * gp) * 8, 0, 16));
    }
    __builtin_amdgcn_sched_barrier(0);  // keep every Gram load ahead of the P loads
    const int pn4 = (n * r + 3) >> 2;
    f32x4 pv[PV];
#pragma unroll
    for (int q = 0; q < PV; ++q) {
      const int i = q * 256 + tid;
      pv[q] = lp_ld4(rP, 16 * (i < pn4 ? i : 0));
    }
    {
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int q = 0; q < GV; ++q)
        if (q < Jh && gh * Jh + q < J) { s0 += gv[q].x; s1 += gv[q].y; }
      for (int q = GV; q < Jh; ++q) {  // J > 2 GV members
        const int mb = gh * Jh + q;
        if (mb < J) {
          const double2 v = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
              rG, ((gload ? mb : 0) * 256 + 2 * gp) * 8, 0, 16));
          s0 += v.x;
          s1 += v.y;
        }
      }
      gpart[gh * 256 + 2 * gp] = s0;
      gpart[gh * 256 + 2 * gp + 1] = s1;
    }
    lp_sync();
    gm[tid] = (tid < 16 * r) ? gpart[tid] + gpart[256 + tid] : 0.0;
    lp_sync();
    LP_STAMP(sb + 4);
    // R = 16: wave 0 factorises ahead of the P staging (every wave's copy beside the MFMAs would
    // spill at that bound)
    if constexpr (R > 12) {
      if (w == 0) lp_chol<R>(gm, Rh, Sv, r, lane);
    }
#pragma unroll
    for (int q = 0; q < PV; ++q) {
      const int i = q * 256 + tid;
      if (q * 256 < pn4 && i < pn4) reinterpret_cast<f32x4*>(stg)[i] = pv[q];
    }
    if (pn4 > PV * 256)  // larger P: the rest in series
      lp_stage(stg + 4 * PV * 256, lp_rsrc(X.P + 4 * PV * 256), 4 * (pn4 - PV * 256), tid);
    lp_sync();  // P staged
    LP_STAMP(sb + 8);
    {  // H = G[:, my cols]^T P on the matrix cores (the WB waves of a column block meet in red),
       // with the scaled Cholesky of the Gram (every wave, identical values) in the same block:
       // its readlane / VALU chain issues between the MFMAs instead of ahead of them in wave 0
      if constexpr (R <= 12) lp_chol<R, true>(gm, Rh, Sv, r, lane);
#if LP_BF16X3
      f32x4 acc2[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        float pv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int row = 32 * (rlw + WB * i) + 8 * kr + e;
          pv[e] = stg[(row < n ? row : 0) * r + cc] * cmask;
        }
        bf16x8 ph, pl;
        lp_split8(pv, ph, pl);
        acc2[i & 1] = lp_mfma3(gbh[i], gbl[i], ph, pl, acc2[i & 1]);
      }
      const f32x4 acc = acc2[0] + acc2[1];
#else
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < LP_GV; ++i) {
        float pv[4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int row = 16 * (rlw + WB * i) + 4 * s2 + kr;
          pv[s2] = stg[(row < n ? row : 0) * r + cc] * cmask;
        }
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(gb[i][s2], pv[s2], acc, 0, 0, 0);
      }
#endif
#pragma unroll
      for (int e = 0; e < 4; ++e) red[w * 256 + (4 * kr + e) * 16 + c] = acc[e];
    }
    lp_sync();  // red complete, Rh / Sv visible
    LP_STAMP(sb + 5);
    // the WB wave partials of each column block summed by all threads (one element each, wave
    // order), in place into the block's first slot: the solve lanes then read finished sums
    // (a per-lane reduction loop made each of its 16 entries a chain of WB dependent LDS reads)
    for (int e = tid; e < (cb1 - cb0) * 256; e += 256) {
      const int cb = e >> 8, o = e & 255;
      float v = 0.f;
      for (int q = 0; q < WB; ++q) v += red[(cb * WB + q) * 256 + o];
      red[cb * WB * 256 + o] = v;
    }
    lp_sync();
    LP_STAMP(sb + 9);
    float dd = 0.f, qq = 0.f;
    if (tid < ncol) {  // wave 0: one Q row per lane, H[col][:] D^{-1/2} R_s^{-1}
      const int cb = tid >> 4, i = tid & 15;
      // unconditional clamped loads + selects, R (not LR_MAXR) entries: an `e < r ? load : 0`
      // per entry compiled to a branch and a separate LDS wait each (predicates spilled to VGPR
      // lanes), ~2 us of the phase
      float old[LR_MAXR], x[LR_MAXR];
#pragma unroll
      for (int e = 0; e < LR_MAXR; ++e) old[e] = x[e] = 0.f;
#pragma unroll
      for (int e = 0; e < R; ++e) {
        const float o = qold[tid * r + (e < r ? e : r - 1)];
        const float h = red[cb * WB * 256 + i * 16 + e];
        old[e] = e < r ? o : 0.f;
        x[e] = e < r ? h : 0.f;
      }
      lp_solve<R>(x, Rh, Sv);
#pragma unroll
      for (int e = 0; e < R; ++e) {
        const float d = e < r ? x[e] - old[e] : 0.f, q = e < r ? x[e] : 0.f;
        dd += d * d;
        qq += q * q;
      }
#pragma unroll
      for (int e = 0; e < R; ++e)
        if (e < r) mine[tid * r + e] = x[e];
    }
    dd = wave_sum(dd);
    qq = wave_sum(qq);
    if (lane == 0) { dq[2 * w] = dd; dq[2 * w + 1] = qq; }
    lp_sync();
    lp_publish(rQ, mine, 16 * cb0, 16 * cb0 + ncol, r, tid);
    if (tid == 0) {
      lp_st1(rN, 8 * j, (dq[0] + dq[2]) + (dq[4] + dq[6]));
      lp_st1(rN, 8 * j + 4, (dq[1] + dq[3]) + (dq[5] + dq[7]));
    }
    LP_STAMP(sb + 6);
    lp_barrier(a.sync, l, (++bar) * (unsigned)J, 0x200u + (unsigned)l, a.spin);
    LP_STAMP(sb + 7);
    // stop after this commit?  dad_tol: lane b of every wave loads member b's norms (one round
    // trip) and the butterfly sums them the same way in every wave of every member: one decision
    bool stop = it + 1 >= a.iters;
    if (!stop && a.tol > 0.f) {
      float D = lane < J ? lp_ld1(rN, 8 * lane) : 0.f;
      float Qn = lane < J ? lp_ld1(rN, 8 * lane + 4) : 0.f;
      D = wave_sum(D);
      Qn = wave_sum(Qn);
      stop = sqrtf(D) / (sqrtf(Qn) + 1e-8f) < a.tol;
    }
    if (stop) {
      // Psend for my rows from the last iteration's P (still staged) and factor, once per launch
      const int nr = min(n, 16 * rb1) - 16 * rb0;
      if (tid < nr) {
        float x[LR_MAXR];
        const int row = 16 * rb0 + tid;
#pragma unroll
        for (int e = 0; e < LR_MAXR; ++e) x[e] = 0.f;
#pragma unroll
        for (int e = 0; e < R; ++e) {
          const float v = stg[row * r + (e < r ? e : r - 1)];
          x[e] = e < r ? v : 0.f;
        }
        lp_solve<R>(x, Rh, Sv);
#pragma unroll
        for (int e = 0; e < R; ++e)
          if (e < r) X.Psend[(long)row * r + e] = x[e];
      }
      break;
    }
  }
  // the last member out resets the layer's counters for the next launch (every member has
  // passed every poll of this launch when it arrives here)
  if (tid == 0) {
    lp_gu32* d = (lp_gu32*)(a.sync + l * 64 + 32);
    const unsigned prev = __hip_atomic_fetch_add(d, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (unsigned)J - 1u) {
      __hip_atomic_store((lp_gu32*)(a.sync + l * 64), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(d, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  LP_STAMP(61);  // exit of member 0 (Psend stored)
}

}  // namespace

#ifdef LR_STAMPS
DN_API int dn_lr_set_stamps(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(lr_stamp_buf), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
#endif
DN_API long dn_lr_layer_size() { return (long)sizeof(LrLayer); }
DN_API long dn_pi_recon_size() { return (long)sizeof(PiRecon); }
DN_API int dn_lr_limits(int* maxr, int* plds, int* qlds) {
  *maxr = LR_MAXR;
  *plds = LR_PLDS;
  *qlds = LR_QLDS;
  return DN_OK;
}

// One power iteration / PowerSGD half-round over every layer of the table (`layers`: the device
// table; `host`: the same table in host memory, read for the launch index).  Launches of at most
// LR_KMAX layers each (one launch for every ICA model).
//   stage 0: lr_gq (P = G Q; it == 0 re-activates every layer, it > 0 applies dad_tol first)
//   stage 1: lr_gtp (Pn = P R^{-1} from the fp64 Gram; Q = G^T Pn committed to Qsend)
DN_API int dn_lr_stage(const void* layers, const void* host, int nl, int stage, int it, float tol,
                       hipStream_t st) {
  if (nl <= 0) return DN_OK;
  if (nl > 256 || !host || (stage != 0 && stage != 1)) return DN_BAD_SHAPE;
  const LrLayer* L = (const LrLayer*)layers;
  const LrLayer* H = (const LrLayer*)host;
  for (int c0 = 0; c0 < nl; c0 += LR_KMAX) {
    LrIndex ix{};
    ix.n = nl - c0 < LR_KMAX ? nl - c0 : LR_KMAX;
    for (int j = 0; j < ix.n; ++j) ix.first[j] = stage == 0 ? H[c0 + j].b1 : H[c0 + j].b3;
    const LrLayer& E = H[c0 + ix.n - 1];
    const int blocks = (stage == 0 ? E.b1 + E.n1 : E.b3 + E.n3) - ix.first[0];
    if (blocks <= 0) continue;
    if (stage == 0)
      hipLaunchKernelGGL(lr_gq_kernel, dim3(blocks), dim3(256), 0, st, L + c0, ix, it, tol);
    else {
      int rm = 1;
      for (int j = 0; j < ix.n; ++j) rm = H[c0 + j].r > rm ? H[c0 + j].r : rm;
      if (rm <= 4)
        hipLaunchKernelGGL(lr_gtp_kernel<4>, dim3(blocks), dim3(256), 0, st, L + c0, ix, it);
      else if (rm <= 8)
        hipLaunchKernelGGL(lr_gtp_kernel<8>, dim3(blocks), dim3(256), 0, st, L + c0, ix, it);
      else
        hipLaunchKernelGGL(lr_gtp_kernel<16>, dim3(blocks), dim3(256), 0, st, L + c0, ix, it);
    }
  }
  return dn_launch_status();
}

// PowerSGD reconstruction + error feedback over every layer (`host`: the table in host memory)
DN_API int dn_lr_recon_ef(const void* layers, const void* host, int nl, hipStream_t st) {
  if (nl <= 0) return DN_OK;
  if (nl > 256 || !host) return DN_BAD_SHAPE;
  const LrLayer* L = (const LrLayer*)layers;
  const LrLayer* H = (const LrLayer*)host;
  for (int c0 = 0; c0 < nl; c0 += LR_KMAX) {
    LrIndex ix{};
    ix.n = nl - c0 < LR_KMAX ? nl - c0 : LR_KMAX;
    long t = 0;
    for (int j = 0; j < ix.n; ++j) {
      ix.first[j] = (int)t;
      t += (long)((H[c0 + j].out + 15) / 16) * ((H[c0 + j].in + 15) / 16);
    }
    if (t <= 0) continue;
    if (t > (1L << 30)) return DN_BAD_SHAPE;
    long blocks = (t + 3) / 4;  // one 16 x 16 tile per wave
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(lr_recon_ef_kernel, dim3((unsigned)blocks), dim3(256), 0, st, L + c0, ix,
                       (int)t);
  }
  return dn_launch_status();
}

// G_l = sum over W sites of P_s Q_s^T / W for every layer; `stride` = send-buffer length;
// `recon` the device table, `host` the same table in host memory (read for the tile prefix).
DN_API int dn_pi_reconstruct(const void* recon, const void* host, int n, long total, long stride,
                             int W, hipStream_t st) {
  if (n <= 0 || total <= 0) return DN_OK;
  if (n > PR_MAXL || !host) return DN_BAD_SHAPE;
  const PiRecon* H = (const PiRecon*)host;
  PrIndex ix{};
  ix.n = n;
  long t = 0;
  for (int l = 0; l < n; ++l) {
    if (H[l].r < 1 || H[l].r > 16) return DN_BAD_SHAPE;
    ix.L[l] = H[l];
    ix.tstart[l] = t;
    t += (long)((H[l].out + 15) / 16) * ((H[l].in + 15) / 16);
  }
  ix.tstart[n] = t;
  for (int l = n + 1; l <= PR_MAXL; ++l) ix.tstart[l] = t;
  long blocks = (t + 3) / 4;  // one 16 x 16 tile per wave
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  (void)recon;  // (the device copy of the table: kept in the interface, the records ride in ix)
  hipLaunchKernelGGL(pi_reconstruct_kernel, dim3((unsigned)blocks), dim3(256), 0, st, ix, stride,
                     W, 1.f / (float)W);
  return dn_launch_status();
}

// Members per layer for the persistent launch: the fewest J <= LP_MAXJ whose two register slices
// fit (row-block and column-block chunks per wave <= LP_GV); 0 when a layer cannot take it.
static int lp_plan(int out, int in, int r, int& J, int& rbp, int& cbp) {
  if (in % 4 || r < 1 || r > LR_MAXR || (long)in * r > LP_LDS || (long)out * r > LP_LDS) return 0;
  const int nrb = (out + 15) / 16, ncb = (in + 15) / 16;
  auto p2 = [](int v) { return v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : 8; };
  for (J = 1; J <= LP_MAXJ; ++J) {
    rbp = p2((nrb + J - 1) / J);
    cbp = p2((ncb + J - 1) / J);
    // per wave: one row (column) block and at most LP_GV of its chunks
    if (rbp <= LP_RB && cbp <= LP_RB && ncb <= LP_GV * (4 / rbp) && nrb <= LP_GV * (4 / cbp))
      return 1;
  }
  return 0;
}

// ALL `iters` power iterations of every layer of a host-side LrLayer table in one launch
// (lr_persist_kernel); DN_UNSUPPORTED when the table does not fit it (the caller then runs
// dn_lr_stage).  gram: >= nl * LP_MAXJ * 256 doubles; norms: >= nl * LP_MAXJ * 2 floats; sync:
// (LP_MAXL * 64 + 1) zeroed unsigned words, owned by this table (counters reset by each launch).
static unsigned long long* g_lp_stamps = nullptr;
DN_API int dn_lr_persist_set_stamps(void* p) {
  g_lp_stamps = (unsigned long long*)p;
  return DN_OK;
}

DN_API int dn_lr_persist(const void* host_layers, int nl, int iters, float tol, double* gram,
                         float* norms, unsigned* sync, hipStream_t st) {
  if (nl <= 0) return DN_OK;
  if (nl > LP_MAXL || iters < 1 || !gram || !norms || !sync) return DN_UNSUPPORTED;
  LpArgs a{};
  a.nl = nl;
  a.iters = iters;
  a.tol = tol;
  a.sync = sync;
  a.stamps = g_lp_stamps;
  int jmax = 1;
  const LrLayer* hl = reinterpret_cast<const LrLayer*>(host_layers);
  for (int l = 0; l < nl; ++l) {
    LpLayer& Y = a.L[l];
    Y.X = hl[l];
    if (Y.X.err) return DN_UNSUPPORTED;  // PowerSGD keeps the staged kernels
    if (!lp_plan(Y.X.out, Y.X.in, Y.X.r, Y.J, Y.rb_per, Y.cb_per)) return DN_UNSUPPORTED;
    Y.gram = gram + (long)l * LP_MAXJ * 256;
    Y.norms = norms + (long)l * LP_MAXJ * 2;
    jmax = Y.J > jmax ? Y.J : jmax;
  }
  a.spin = dn_spin_limit(LP_SPIN);
  // members of a layer meet at barriers: every workgroup must be resident at once (else the
  // staged kernels, DN_UNSUPPORTED)
  int rmax = 1, rmin = 1 << 30;
  for (int l = 0; l < nl; ++l) {
    rmax = a.L[l].X.r > rmax ? a.L[l].X.r : rmax;
    rmin = a.L[l].X.r < rmin ? a.L[l].X.r : rmin;
  }
  const int rb = rmax <= 4 ? 4 : rmax <= 8 ? 8 : rmax <= 10 ? 10 : rmax <= 12 ? 12 : 16;
  const bool ex = rmin == rmax && rmax == rb;
  const void* kfn = nullptr;
  void (*kl)(LpArgs) = nullptr;
#define LP_PICK(RB_)                                                              \
  if (rb == RB_) kl = ex ? lr_persist_kernel<RB_, true> : lr_persist_kernel<RB_, false>;
  LP_PICK(4) LP_PICK(8) LP_PICK(10) LP_PICK(12) LP_PICK(16)
#undef LP_PICK
  kfn = reinterpret_cast<const void*>(kl);
  if (!dn_fits_resident(kfn, LP_MAXL * jmax, 256, 0))
    return DN_UNSUPPORTED;
  hipLaunchKernelGGL(kl, dim3(LP_MAXL * jmax), dim3(256), 0, st, a);
  return dn_launch_status();
}

DN_API long dn_lr_persist_words() { return LP_MAXL * 64 + 1; }
DN_API long dn_lr_persist_maxj() { return LP_MAXJ; }
