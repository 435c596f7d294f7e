// General bf16-MFMA GEMM for gfx950 with fused epilogues.
//
//   C[M,N] = alpha * op(A)[M,K] . op(B)[K,N]  (+ bias[N]) (ReLU) (+ beta * C)
//
// * op(A): A stored [M][lda] (k contiguous) or, with TA, [K][lda] (m contiguous); same for B
//   (TB: [N][ldb] k contiguous, else [K][ldb] n contiguous).  Operands may be fp32 or bf16: fp32
//   is rounded to bf16 while staging, so an fp32 activation never needs a separate cast kernel.
// * Tiles are staged global -> VGPR -> LDS (k-contiguous, +16 B row pad: the 16-lane groups of
//   ds_read_b128 hit distinct bank quads), double-buffered with the next tile's global loads in
//   flight during the current tile's MFMAs (16x16x32 bf16, fp32 accumulators).
// * Small/skinny problems (the ICA shapes: M = B*S = 3136, N <= 1536) use 64x64 tiles to put
//   >= 200 workgroups on the 256 CUs; long-K weight-gradient GEMMs (K = B*S) split K across
//   workgroups into fp32 slabs reduced by a second, deterministic kernel (no float atomics, so
//   every site computes bit-identical gradients for identical inputs).
// * Epilogue: bias add, ReLU, accumulate (beta), fp32 or bf16 store, optional row permutation
//   (used to emit LSTM gate-permuted rows straight into the reference [i|f|o|g] layout).
#include "common.h"

namespace {

template <typename T> __device__ __forceinline__ bf16 to_bf(T v) { return (bf16)v; }

template <int BM, int BN, bool TA, bool TB, typename TAe, typename TBe>
struct GemmTile {
  static constexpr int BK = 32;
  static constexpr int LDK = BK + 8;
  static constexpr int NT = 256;
  static constexpr int WM = BM / 2, WN = BN / 2;   // 2x2 waves
  static constexpr int FM = WM / 16, FN = WN / 16;  // 16x16 frags per wave
  static constexpr int A_ELEMS = BM * BK / NT;      // elements each thread stages per tile
  static constexpr int B_ELEMS = BN * BK / NT;
};

// Stage one operand tile (rows x BK, logical [row][k]) into registers as bf16.
// KCONTIG: element (r,k) at base[r*ld + k] (vector along k); else at base[k*ld + r] (along r).
template <int ROWS, bool KCONTIG, typename TE>
__device__ __forceinline__ void stage_load(const TE* __restrict__ base, long ld, int row0, int k0,
                                           int nrows, int K, int tid, bf16 (&reg)[ROWS * 32 / 256]) {
  constexpr int PER = ROWS * 32 / 256;  // 8 or 16
  if constexpr (KCONTIG) {
    // thread -> (row, 8-wide k chunk); PER/8 chunks per thread
#pragma unroll
    for (int c = 0; c < PER / 8; ++c) {
      const int idx = tid + c * 256;
      const int r = idx >> 2, kk = (idx & 3) * 8;
      const int gr = row0 + r, gk = k0 + kk;
      const TE* p = base + (long)gr * ld + gk;
      if (gr < nrows && gk + 8 <= K && ((((uintptr_t)p) & (sizeof(TE) * 8 - 1)) == 0)) {
        if constexpr (sizeof(TE) == 2) {
          bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
          for (int e = 0; e < 8; ++e) reg[c * 8 + e] = v[e];
        } else {
          f32x4 v0 = *reinterpret_cast<const f32x4*>(p);
          f32x4 v1 = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) { reg[c * 8 + e] = (bf16)v0[e]; reg[c * 8 + 4 + e] = (bf16)v1[e]; }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          reg[c * 8 + e] = (gr < nrows && gk + e < K) ? to_bf(p[e]) : (bf16)0.f;
      }
    }
  } else {
    // thread -> (k, 8-wide row chunk)
    constexpr int RCH = ROWS / 8;  // row chunks per k
#pragma unroll
    for (int c = 0; c < PER / 8; ++c) {
      const int idx = tid + c * 256;
      const int kk = idx / RCH, r = (idx % RCH) * 8;
      const int gk = k0 + kk, gr = row0 + r;
      const TE* p = base + (long)gk * ld + gr;
      if (gk < K && gr + 8 <= nrows && ((((uintptr_t)p) & (sizeof(TE) * 8 - 1)) == 0)) {
        if constexpr (sizeof(TE) == 2) {
          bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
          for (int e = 0; e < 8; ++e) reg[c * 8 + e] = v[e];
        } else {
          f32x4 v0 = *reinterpret_cast<const f32x4*>(p);
          f32x4 v1 = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) { reg[c * 8 + e] = (bf16)v0[e]; reg[c * 8 + 4 + e] = (bf16)v1[e]; }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          reg[c * 8 + e] = (gk < K && gr + e < nrows) ? to_bf(p[e]) : (bf16)0.f;
      }
    }
  }
}

template <int ROWS, bool KCONTIG>
__device__ __forceinline__ void stage_store(bf16 (*lds)[40], int tid, const bf16 (&reg)[ROWS * 32 / 256]) {
  constexpr int PER = ROWS * 32 / 256;
  if constexpr (KCONTIG) {
#pragma unroll
    for (int c = 0; c < PER / 8; ++c) {
      const int idx = tid + c * 256;
      const int r = idx >> 2, kk = (idx & 3) * 8;
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = reg[c * 8 + e];
      *reinterpret_cast<bf16x8*>(&lds[r][kk]) = v;
    }
  } else {
    constexpr int RCH = ROWS / 8;
#pragma unroll
    for (int c = 0; c < PER / 8; ++c) {
      const int idx = tid + c * 256;
      const int kk = idx / RCH, r = (idx % RCH) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) lds[r + e][kk] = reg[c * 8 + e];
    }
  }
}

struct Epi {
  const float* bias;   // [N] or null
  const int* row_map;  // output row remap (C row = row_map[m]) or null
  float alpha, beta;
  int relu;
  int out_bf16;
};

template <int BM, int BN, bool TA, bool TB, typename TAe, typename TBe>
__global__ void __launch_bounds__(256)
gemm_kernel(const TAe* __restrict__ A, long lda, const TBe* __restrict__ B, long ldb,
            void* __restrict__ C, long ldc, int M, int N, int K, int kchunk,
            float* __restrict__ slab, Epi epi) {
  typedef GemmTile<BM, BN, TA, TB, TAe, TBe> T;
  __shared__ __attribute__((aligned(16))) bf16 As[2][BM][T::LDK];
  __shared__ __attribute__((aligned(16))) bf16 Bs[2][BN][T::LDK];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (N + BN - 1) / BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);

  bf16 ra[T::A_ELEMS], rb[T::B_ELEMS];
  f32x4 acc[T::FM][T::FN];
#pragma unroll
  for (int i = 0; i < T::FM; ++i)
#pragma unroll
    for (int j = 0; j < T::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + T::BK - 1) / T::BK;
  if (nk > 0) {
    stage_load<BM, !TA, TAe>(A, lda, row0, kbeg, M, kend, tid, ra);
    stage_load<BN, TB, TBe>(B, ldb, col0, kbeg, N, kend, tid, rb);
    stage_store<BM, !TA>(As[0], tid, ra);
    stage_store<BN, TB>(Bs[0], tid, rb);
  }
  __syncthreads();
  for (int it = 0; it < nk; ++it) {
    const int cur = it & 1;
    const bool more = it + 1 < nk;
    if (more) {  // next tile's global loads fly under this tile's MFMAs
      const int k0 = kbeg + (it + 1) * T::BK;
      stage_load<BM, !TA, TAe>(A, lda, row0, k0, M, kend, tid, ra);
      stage_load<BN, TB, TBe>(B, ldb, col0, k0, N, kend, tid, rb);
    }
    bf16x8 af[T::FM], bfr[T::FN];
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(&As[cur][wm * T::WM + 16 * i + (lane & 15)][8 * (lane >> 4)]);
#pragma unroll
    for (int j = 0; j < T::FN; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][wn * T::WN + 16 * j + (lane & 15)][8 * (lane >> 4)]);
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
#pragma unroll
      for (int j = 0; j < T::FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    if (more) {
      stage_store<BM, !TA>(As[cur ^ 1], tid, ra);
      stage_store<BN, TB>(Bs[cur ^ 1], tid, rb);
    }
    __syncthreads();
  }

  // epilogue
  const bool split = slab != nullptr;
#pragma unroll
  for (int i = 0; i < T::FM; ++i)
#pragma unroll
    for (int j = 0; j < T::FN; ++j) {
      const int col = col0 + wn * T::WN + 16 * j + (lane & 15);
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * T::WM + 16 * i + 4 * (lane >> 4) + r;
        if (row >= M) continue;
        float v = acc[i][j][r];
        if (split) {
          slab[((long)blockIdx.z * M + row) * N + col] = v;
          continue;
        }
        v *= epi.alpha;
        if (epi.bias) v += epi.bias[col];
        if (epi.relu) v = fmaxf(v, 0.f);
        const long orow = epi.row_map ? epi.row_map[row] : row;
        if (orow < 0) continue;  // dropped row (e.g. zero-padded LSTM units)
        if (epi.out_bf16) {
          bf16* cp = reinterpret_cast<bf16*>(C) + orow * ldc + col;
          if (epi.beta != 0.f) v += epi.beta * (float)*cp;
          *cp = (bf16)v;
        } else {
          float* cp = reinterpret_cast<float*>(C) + orow * ldc + col;
          if (epi.beta != 0.f) v += epi.beta * *cp;
          *cp = v;
        }
      }
    }
}

// deterministic split-K combine + epilogue
__global__ void gemm_splitk_reduce(const float* __restrict__ slab, int splits, int M, int N,
                                   void* __restrict__ C, long ldc, Epi epi) {
  const long total = (long)M * N;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += slab[(long)s * total + idx];
    const int row = (int)(idx / N), col = (int)(idx % N);
    v *= epi.alpha;
    if (epi.bias) v += epi.bias[col];
    if (epi.relu) v = fmaxf(v, 0.f);
    const long orow = epi.row_map ? epi.row_map[row] : row;
    if (orow < 0) continue;
    if (epi.out_bf16) {
      bf16* cp = reinterpret_cast<bf16*>(C) + orow * ldc + col;
      if (epi.beta != 0.f) v += epi.beta * (float)*cp;
      *cp = (bf16)v;
    } else {
      float* cp = reinterpret_cast<float*>(C) + orow * ldc + col;
      if (epi.beta != 0.f) v += epi.beta * *cp;
      *cp = v;
    }
  }
}

template <int BM, int BN, bool TA, bool TB, typename TAe, typename TBe>
int launch(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N,
           int K, int splits, float* slab, Epi epi, hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int kchunk = K;
  if (splits > 1) {
    kchunk = (K + splits - 1) / splits;
    kchunk = (kchunk + 31) / 32 * 32;
    splits = (K + kchunk - 1) / kchunk;
  }
  dim3 grid(tiles, 1, splits);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, TA, TB, TAe, TBe>), grid, dim3(256), 0, st,
                     (const TAe*)A, lda, (const TBe*)B, ldb, C, ldc, M, N, K, kchunk,
                     splits > 1 ? slab : nullptr, epi);
  if (splits > 1) {
    const long total = (long)M * N;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, st, slab, splits, M, N, C,
                       ldc, epi);
  }
  return dn_launch_status();
}

template <int BM, int BN, typename TAe, typename TBe>
int dispatch_t(int ta, int tb, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
               int M, int N, int K, int splits, float* slab, Epi epi, hipStream_t st) {
  if (!ta && !tb) return launch<BM, BN, false, false, TAe, TBe>(A, lda, B, ldb, C, ldc, M, N, K, splits, slab, epi, st);
  if (!ta && tb) return launch<BM, BN, false, true, TAe, TBe>(A, lda, B, ldb, C, ldc, M, N, K, splits, slab, epi, st);
  if (ta && !tb) return launch<BM, BN, true, false, TAe, TBe>(A, lda, B, ldb, C, ldc, M, N, K, splits, slab, epi, st);
  return launch<BM, BN, true, true, TAe, TBe>(A, lda, B, ldb, C, ldc, M, N, K, splits, slab, epi, st);
}

template <int BM, int BN>
int dispatch_tile(int a_bf16, int b_bf16, int ta, int tb, const void* A, long lda, const void* B,
                  long ldb, void* C, long ldc, int M, int N, int K, int splits, float* slab, Epi epi,
                  hipStream_t st) {
  if (a_bf16 && b_bf16) return dispatch_t<BM, BN, bf16, bf16>(ta, tb, A, lda, B, ldb, C, ldc, M, N, K, splits, slab, epi, st);
  if (a_bf16 && !b_bf16) return dispatch_t<BM, BN, bf16, float>(ta, tb, A, lda, B, ldb, C, ldc, M, N, K, splits, slab, epi, st);
  if (!a_bf16 && b_bf16) return dispatch_t<BM, BN, float, bf16>(ta, tb, A, lda, B, ldb, C, ldc, M, N, K, splits, slab, epi, st);
  return dispatch_t<BM, BN, float, float>(ta, tb, A, lda, B, ldb, C, ldc, M, N, K, splits, slab, epi, st);
}

}  // namespace

// Returns the fp32 slab elements the caller must provide for a split-K launch (0 if none).
DN_API long dn_gemm_workspace(int M, int N, int K, int splits) {
  return splits > 1 ? (long)splits * M * N : 0;
}

// tile: 0 -> 64x64, 1 -> 128x128
DN_API int dn_gemm(const void* A, int a_bf16, int ta, long lda, const void* B, int b_bf16, int tb,
                   long ldb, void* C, int c_bf16, long ldc, int M, int N, int K, float alpha,
                   float beta, const float* bias, int relu, const int* row_map, int tile,
                   int splits, float* slab, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return DN_BAD_SHAPE;
  if (splits > 1 && !slab) return DN_BAD_SHAPE;
  Epi epi{bias, row_map, alpha, beta, relu, c_bf16};
  if (tile == 1)
    return dispatch_tile<128, 128>(a_bf16, b_bf16, ta, tb, A, lda, B, ldb, C, ldc, M, N, K, splits, slab, epi, st);
  return dispatch_tile<64, 64>(a_bf16, b_bf16, ta, tb, A, lda, B, ldb, C, ldc, M, N, K, splits, slab, epi, st);
}
