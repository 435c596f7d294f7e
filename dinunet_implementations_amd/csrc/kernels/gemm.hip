// General bf16-MFMA GEMM for gfx950 with fused epilogues.
//
//   C[M,N] = alpha * op(A)[M,K] . op(B)[K,N]  (+ bias[N]) (ReLU) (+ beta * C)
//
// * op(A): A stored [M][lda] (k contiguous) or, with TA, [K][lda] (m contiguous); same for B
//   (TB: [N][ldb] k contiguous, else [K][ldb] n contiguous).  Operands may be fp32 or bf16: fp32
//   is rounded to bf16 while staging, so an fp32 activation never needs a separate cast kernel.
// * Tiles are staged global -> VGPR (16 B vectors along the contiguous axis) -> LDS in the
//   operand's own layout, double-buffered with the next tile's global loads in flight during the
//   current tile's MFMAs (16x16x32 bf16, fp32 accumulators).  k-major operands are turned into
//   MFMA fragments by the CDNA4 LDS transpose read (ds_read_b64_tr_b16), so no layout costs a
//   register shuffle.
// * Small/skinny problems (the ICA shapes: M = B*S = 3136, N <= 1536) use 64x64 tiles to put
//   >= 200 workgroups on the 256 CUs; long-K weight-gradient GEMMs (K = B*S) split K across
//   workgroups into fp32 slabs, combined in a fixed split order (no float atomics, so every site
//   computes bit-identical gradients for identical inputs) either inside the launch by each
//   tile's last-arriving split (GemmGroup::cnt) or by a second reduce kernel.
// * Epilogue: bias add, ReLU, accumulate (beta), fp32 or bf16 store, optional row permutation
//   (used to emit LSTM gate-permuted rows straight into the reference [i|f|o|g] layout).
#include "common.h"

namespace {

template <typename T> __device__ __forceinline__ bf16 to_bf(T v) { return (bf16)v; }

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// LDS images, by the operand's memory layout:
//  k-contiguous (A with !TA, B with TB): [rows][64 + 8] bf16; a fragment = one ds_read_b128.
//  k-major      (A with TA,  B with !TB): [64 k][cols + 16] bf16, filled with 16 B vectors
//    along cols; a fragment = two ds_read_b64_tr_b16 (4 k each, hardware transpose).  The row
//    stride is 8 * odd banks and k-rows are stored with bit 2 flipped in odd 8-row groups, so
//    each 32-lane half touches 8 distinct rows mod 8 -> conflict-free transposed reads.
template <int ROWS, bool KCONTIG> struct Img {
  static constexpr int R = KCONTIG ? ROWS : 64;          // image rows
  static constexpr int C = KCONTIG ? 64 + 8 : ROWS + 16; // image row length (elements)
  static constexpr int ELEMS = R * C;
};

template <int BM, int BN, bool TA, bool TB>
struct GemmTile {
  static constexpr int BK = 64;
  static constexpr int NT = 256;
  static constexpr int WM = BM / 2, WN = BN / 2;   // 2x2 waves
  static constexpr int FM = WM / 16, FN = WN / 16;  // 16x16 frags per wave
  static constexpr int A_ELEMS = BM * BK / NT;      // elements each thread stages per tile
  static constexpr int B_ELEMS = BN * BK / NT;
  typedef Img<BM, !TA> IA;
  typedef Img<BN, TB> IB;
};

// Stage one operand tile (ROWS x 64 logical [row][k]) into registers as bf16, 8 elements per
// 16 B vector (fp32 sources are rounded while staging).
//  KCONTIG: element (r,k) at base[r*ld + k]; chunk -> (row, 8 consecutive k)
//  else   : element (r,k) at base[k*ld + r]; chunk -> (k, 8 consecutive rows)
template <int ROWS, bool KCONTIG, typename TE>
__device__ __forceinline__ void stage_load(const TE* __restrict__ base, long ld, int row0, int k0,
                                           int nrows, int K, int tid, bf16 (&reg)[ROWS * 64 / 256]) {
  constexpr int PER = ROWS * 64 / 256;  // 16 or 32
  constexpr int CPR = KCONTIG ? 8 : ROWS / 8;  // chunks per image row
#pragma unroll
  for (int c = 0; c < PER / 8; ++c) {
    const int idx = tid + c * 256;
    const int ir = idx / CPR, ic = (idx % CPR) * 8;
    const int gr = KCONTIG ? row0 + ir : row0 + ic;  // logical row of the chunk's first element
    const int gk = KCONTIG ? k0 + ic : k0 + ir;
    const TE* p = KCONTIG ? base + (long)gr * ld + gk : base + (long)gk * ld + gr;
    const bool full = KCONTIG ? (gr < nrows && gk + 8 <= K) : (gk < K && gr + 8 <= nrows);
    if (full && ((((uintptr_t)p) & (sizeof(TE) * 8 - 1)) == 0)) {
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
      for (int e = 0; e < 8; ++e) {
        const bool ok = KCONTIG ? (gr < nrows && gk + e < K) : (gk < K && gr + e < nrows);
        reg[c * 8 + e] = ok ? to_bf(p[e]) : (bf16)0.f;
      }
    }
  }
}

// Branch-free variant for the common aligned case (host-checked, GemmGroup::vec): the
// contiguous axis (k when KCONTIG, rows otherwise) has extent and leading dimension divisible by
// 8 and 16-B aligned bases, so a chunk is entirely in range or entirely out.  Out-of-range chunks
// load a clamped in-range address and are zeroed by a select.  The RAW vectors stay in registers
// until the LDS store after the MFMAs (rounding / zeroing happens there), so the next tile's
// loads issue back to back and their latency hides under the current tile's MFMAs -- the
// branchy variant makes the compiler drain vmcnt after every chunk.
template <typename TE> struct Chunk;
template <> struct Chunk<bf16> { bf16x8 v; };
template <> struct Chunk<float> { f32x4 lo, hi; };

template <int ROWS, bool KCONTIG, typename TE>
struct VecStager {
  static constexpr int CH = ROWS * 64 / 256 / 8;  // 16-B chunks per thread per tile
  static constexpr int CPR = KCONTIG ? 8 : ROWS / 8;
  Chunk<TE> c[CH];
  bool ok[CH];
  __device__ __forceinline__ void load(const TE* __restrict__ base, long ld, int row0, int k0,
                                       int nrows, int K, int tid) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int idx = tid + i * 256;
      const int ir = idx / CPR, ic = (idx % CPR) * 8;
      const int gr = KCONTIG ? row0 + ir : row0 + ic;
      const int gk = KCONTIG ? k0 + ic : k0 + ir;
      ok[i] = gr < nrows && gk < K;
      const int grc = min(gr, nrows - (KCONTIG ? 1 : 8));
      const int gkc = min(gk, K - (KCONTIG ? 8 : 1));
      const TE* p = KCONTIG ? base + (long)grc * ld + gkc : base + (long)gkc * ld + grc;
      if constexpr (sizeof(TE) == 2) {
        c[i].v = *reinterpret_cast<const bf16x8*>(p);
      } else {
        c[i].lo = *reinterpret_cast<const f32x4*>(p);
        c[i].hi = *reinterpret_cast<const f32x4*>(p + 4);
      }
    }
  }
  __device__ __forceinline__ void store(bf16* __restrict__ img, int tid) const {
    constexpr int C = Img<ROWS, KCONTIG>::C;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int idx = tid + i * 256;
      const int ir = idx / CPR, ic = (idx % CPR) * 8;
      bf16x8 v;
      if constexpr (sizeof(TE) == 2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ok[i] ? c[i].v[e] : (bf16)0.f;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = (bf16)(ok[i] ? c[i].lo[e] : 0.f);
          v[4 + e] = (bf16)(ok[i] ? c[i].hi[e] : 0.f);
        }
      }
      const int r = KCONTIG ? ir : (ir ^ ((ir >> 1) & 4));  // see stage_store
      *reinterpret_cast<bf16x8*>(img + r * C + ic) = v;
    }
  }
};

template <int ROWS, bool KCONTIG>
__device__ __forceinline__ void stage_store(bf16* __restrict__ img, int tid, const bf16 (&reg)[ROWS * 64 / 256]);

// the general (ragged / unaligned) stager: converts while loading
template <int ROWS, bool KCONTIG, typename TE>
struct GenStager {
  bf16 reg[ROWS * 64 / 256];
  __device__ __forceinline__ void load(const TE* __restrict__ base, long ld, int row0, int k0,
                                       int nrows, int K, int tid) {
    stage_load<ROWS, KCONTIG, TE>(base, ld, row0, k0, nrows, K, tid, reg);
  }
  __device__ __forceinline__ void store(bf16* __restrict__ img, int tid) const {
    stage_store<ROWS, KCONTIG>(img, tid, reg);
  }
};

template <bool VEC, int ROWS, bool KCONTIG, typename TE> struct StagerSel { typedef GenStager<ROWS, KCONTIG, TE> type; };
template <int ROWS, bool KCONTIG, typename TE> struct StagerSel<true, ROWS, KCONTIG, TE> { typedef VecStager<ROWS, KCONTIG, TE> type; };

template <int ROWS, bool KCONTIG>
__device__ __forceinline__ void stage_store(bf16* __restrict__ img, int tid, const bf16 (&reg)[ROWS * 64 / 256]) {
  constexpr int PER = ROWS * 64 / 256;
  constexpr int CPR = KCONTIG ? 8 : ROWS / 8;
  constexpr int C = Img<ROWS, KCONTIG>::C;
#pragma unroll
  for (int c = 0; c < PER / 8; ++c) {
    const int idx = tid + c * 256;
    const int ir = idx / CPR, ic = (idx % CPR) * 8;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = reg[c * 8 + e];
    // k-major images store k-row k at row k ^ 4*((k>>3)&1): the two 16-lane groups of each
    // 32-lane half then read rows 8 apart mod 8 -> distinct banks (row stride = 8*odd banks)
    const int r = KCONTIG ? ir : (ir ^ ((ir >> 1) & 4));
    *reinterpret_cast<bf16x8*>(img + r * C + ic) = v;
  }
}

// 16x32 MFMA operand fragment (16 rows starting at r0, k = 32*ks .. +31) from an image
template <int ROWS, bool KCONTIG>
__device__ __forceinline__ bf16x8 frag(const bf16* __restrict__ img, int r0, int ks, int lane) {
  constexpr int C = Img<ROWS, KCONTIG>::C;
  if constexpr (KCONTIG) {
    return *reinterpret_cast<const bf16x8*>(img + (r0 + (lane & 15)) * C + 32 * ks + 8 * (lane >> 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int kb = 32 * ks + 8 * g + q;
    const int h0 = (g & 1) ? 4 : 0;  // image row of k is k ^ 4*((k>>3)&1), see stage_store
    const bf16* a0 = img + (kb + h0) * C + r0 + 4 * p;
    const bf16* a1 = img + (kb + (4 - h0)) * C + r0 + 4 * p;
    s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
    s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

struct Epi {
  const float* bias;   // [N] or null
  const int* row_map;  // output row remap (C row = row_map[m]) or null
  float alpha, beta;
  int relu;
  int out_bf16;
  int ncol;  // > 0: only output columns < ncol are stored (e.g. a ones-operand column sum)
  const bf16* mask;  // optional [M][ldm] bf16: outputs where mask <= 0 are zeroed (ReLU backward)
  long ldm;
  void* C2;  // optional second output (same ldc, its own beta accumulate): the LSTM's b_ih and
             // b_hh gradients are the same column sum of the gate gradient, formed once
  // >= 0: result column `xcol` is the column sum of op(A) (the LDS-DMA kernel reads a virtual
  // column of ones as B's column xcol, B holding xcol real columns) and goes to the vectors X1
  // (and X2) [row_map(m)] instead of C: a bias gradient riding in the spare columns of a weight
  // gradient's last tile column, so A is not streamed a second time for it.  The problem's N is
  // xcol + 4 (16-B slab rows for the split-K reduce); columns past xcol are zeros, never stored
  int xcol;
  float* X1;
  float* X2;
};

constexpr int GMAX = 12;  // problems per grouped launch (kernarg: ~1.6 KB)

// Rows of one operand gathered from a dataset resident in HBM instead of a batch copy (the
// device-fed step at large batch): logical row r of the operand is dataset row
// subj[r / gs] * gs + r % gs of gx (row stride = the operand's ld) -- the ICA batch of B
// subjects x S windows, read in place through the step's subject indices (prologue.h sd).  The
// LDS-DMA kernels only: A's rows (k-contiguous A) or B's k rows (k-major B); gs >= 64.
struct RowGather {
  const bf16* gx;            // null: no gather
  const long long* subj;     // [rows / gs + 1] dataset subject indices
  int gs;                    // rows per subject
  int op;                    // 1: operand A, 2: operand B
  int r0;                    // A rows: the problem's row 0 is logical row r0 (a row-range view)
};

// One GEMM problem of a (possibly grouped) launch.
struct GemmProb {
  const void* A;
  const void* B;
  void* C;
  float* slab;  // split-K partials [splits][M][N] (null: no split)
  long lda, ldb, ldc;
  int M, N, K, kchunk;
  Epi epi;
  RowGather rg;
};

// A launch: problems sharing layouts / element types / tile shape.  blockIdx.x enumerates the
// output tiles of problem 0, then problem 1, ...; blockIdx.z is the K split.
struct GemmGroup {
  GemmProb p[GMAX];
  int tile_start[GMAX + 1];
  long elem_start[GMAX + 1];  // split-K reduce: prefix of M*N
  int n, splits;
  int vec;  // every operand satisfies stage_load_vec's alignment contract
  int vepi;  // every problem can take the LDS-staged vector epilogue (see gemm_dma_kernel)
  // split-K arrival tickets, one per output tile of the launch (zero between launches: each
  // tile's combining workgroup resets its own); null -> gemm_splitk_reduce combines
  int* cnt;
  // step counters advanced once by workgroup 0 (dn_gemm_arm_bump: the training step whose fused
  // Adam also packs the next step's weights and batch, optim.hip adam_pack_kernel)
  int* bump_t;
  long long* bump_c;
  // optional slot -> tile map (a permutation of the launch's tiles): consecutive slots share an
  // XCD (8 contiguous slot ranges), so the host orders tiles that read the same operand blocks
  // next to each other (ops.gemm._xcd_order) and each block is fetched into one XCD's L2
  const int* perm;
};

// problem of a launch-wide tile / element index: a count over the (monotone) prefix, unrolled so
// every prefix load issues at once (a search loop was one dependent kernarg load per problem
// before a workgroup could start its own loads)
template <typename T>
__device__ __forceinline__ int group_prob(const GemmGroup& g, const T* start, T v) {
  int pi = 0;
#pragma unroll
  for (int i = 1; i < GMAX; ++i) pi += (i < g.n && v >= start[i]) ? 1 : 0;
  return pi;
}

// the armed bump rides in the next launch of one group only
__device__ __forceinline__ void group_bump(const GemmGroup& g) {
  if (g.bump_t && blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0) {
    *g.bump_t += 1;
    if (g.bump_c) *g.bump_c += 1;
  }
}

typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ void epi_store(const Epi& epi, void* C, long ldc, int row, int col, float v) {
  v *= epi.alpha;
  if (epi.bias) v += epi.bias[col];
  if (epi.relu) v = fmaxf(v, 0.f);
  if (epi.mask && !((float)epi.mask[(long)row * epi.ldm + col] > 0.f)) v = 0.f;
  const long orow = epi.row_map ? epi.row_map[row] : row;
  if (orow < 0) return;  // dropped row (e.g. zero-padded LSTM units)
  if (epi.xcol >= 0 && col >= epi.xcol) {
    if (col > epi.xcol) return;
    for (int o = 0; o < (epi.X2 ? 2 : 1); ++o) {
      float* xp = (o ? epi.X2 : epi.X1) + orow;
      *xp = epi.beta != 0.f ? v + epi.beta * *xp : v;
    }
    return;
  }
  for (int o = 0; o < (epi.C2 ? 2 : 1); ++o) {
    void* Co = o ? epi.C2 : C;
    if (epi.out_bf16) {
      bf16* cp = reinterpret_cast<bf16*>(Co) + orow * ldc + col;
      *cp = (bf16)(epi.beta != 0.f ? v + epi.beta * (float)*cp : v);
    } else {
      float* cp = reinterpret_cast<float*>(Co) + orow * ldc + col;
      *cp = epi.beta != 0.f ? v + epi.beta * *cp : v;
    }
  }
}

// Split-K epilogue of one workgroup (cdna_hip_programming §5, in-launch split-K reduction, sc1
// form): its fp32 partial goes to the slab with write-through (sc1) stores; every wave drains;
// one lane draws an arrival ticket; the workgroup drawing splits-1 is the tile's combiner: it
// resets the ticket, reads the other splits' partials with sc1 loads and sums all of them in
// split order 0..S-1 (its own from registers), so the result does not depend on arrival order.
// `flag`: one int of the kernel's (single) LDS array, free after the K loop.
// accumulator fragments (16x16) per wave up to which a tile carries the in-launch combine
constexpr int SPLITK_INLAUNCH_FRAGS = 4;

template <int FM, int FN, int WM, int WN>
__device__ __forceinline__ void splitk_epilogue(const GemmGroup& g, const GemmProb& P,
                                                const f32x4 (&acc)[FM][FN], int gtile, int row0,
                                                int col0, int wm, int wn, int lane, int* flag) {
  const int M = P.M, N = P.N, z = blockIdx.z;
  float* slab = P.slab;
  // write-through (sc1 = aux bit 4) buffer stores / L1-bypassing loads of the slab; the launcher
  // guarantees splits * M * N * 4 < 2^31 (32-bit offsets)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slab, 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = col0 + wn * WN + 16 * j + (lane & 15);
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * WM + 16 * i + 4 * (lane >> 4) + r;
        if (row >= M) continue;
        const float val = acc[i][j][r];  // (bit_cast of the vector-element lvalue itself
                                         //  read element 0 for every r: clang, ROCm 7.2)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, val), rs,
                                              4 * ((z * M + row) * N + col), 0, 16);
      }
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add((gu32*)(g.cnt + gtile), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    const bool last = prev == (unsigned)(g.splits - 1);
    if (last) __hip_atomic_store((gu32*)(g.cnt + gtile), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last ? 1 : 0;
  }
  __syncthreads();
  if (!*flag) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int nst = P.epi.ncol > 0 ? min(N, P.epi.ncol) : N;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = col0 + wn * WN + 16 * j + (lane & 15);
      float part[4][8];  // the other splits' partials, all loads issued before any use
      const int ns = g.splits < 8 ? g.splits : 8;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * WM + 16 * i + 4 * (lane >> 4) + r;
        const bool ok = row < M && col < nst;
#pragma unroll
        for (int s = 0; s < 8; ++s)
          part[r][s] = (ok && s < ns && s != z)
                           ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                 rs, 4 * ((s * M + row) * N + col), 0, 16))
                           : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * WM + 16 * i + 4 * (lane >> 4) + r;
        if (row >= M || col >= nst) continue;
        float v = 0.f;
#pragma unroll
        for (int s = 0; s < 8; ++s)
          if (s < ns) v += s == z ? acc[i][j][r] : part[r][s];
        for (int s = 8; s < g.splits; ++s)
          v += s == z ? acc[i][j][r]
                      : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                            rs, 4 * ((s * M + row) * N + col), 0, 16));
        epi_store(P.epi, P.C, P.ldc, row, col, v);
      }
    }
}


template <int BM, int BN, bool TA, bool TB, typename TAe, typename TBe, bool VEC>
__global__ void __launch_bounds__(256)
gemm_kernel(GemmGroup g) {
  typedef GemmTile<BM, BN, TA, TB> T;
  // one LDS array (A images then B images, double-buffered)
  // ONE LDS tile (the next tiles wait in registers): 18 KB per 64x64 workgroup, so ~7
  // workgroups share a CU and hide each other's load / store latency
  __shared__ __attribute__((aligned(16))) bf16 smem[T::IA::ELEMS + T::IB::ELEMS];
#define As (smem)
#define Bs (smem + T::IA::ELEMS)

  // XCD-aware tile order: the hardware deals workgroups round-robin over the 8 XCDs (blocks b
  // and b+8 share one L2), so give every XCD a CONTIGUOUS run of row-major tiles -- the tiles
  // of one row band (same A rows) then share that XCD's L2 instead of fetching A 8 times.
  // gridDim.x is padded to a multiple of 8 by the launcher; surplus blocks exit.
  const int ntiles = g.tile_start[g.n];
  const int bid = (int)blockIdx.x;
  const int slot = (bid & 7) * ((int)gridDim.x >> 3) + (bid >> 3);
  if (slot >= ntiles) return;
  group_bump(g);
  const int gtile = g.perm ? g.perm[slot] : slot;
  const int pi = group_prob(g, g.tile_start, gtile);
  const GemmProb& P = g.p[pi];
  const TAe* __restrict__ A = reinterpret_cast<const TAe*>(P.A);
  const TBe* __restrict__ B = reinterpret_cast<const TBe*>(P.B);
  const long lda = P.lda, ldb = P.ldb;
  const int M = P.M, N = P.N, K = P.K;
  const int tile = gtile - g.tile_start[pi];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (N + BN - 1) / BN;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int kbeg = blockIdx.z * P.kchunk;
  const int kend = min(K, kbeg + P.kchunk);

  // Two register stages + two LDS buffers: tile it+2's global loads are issued at the top of
  // iteration it and land during two tiles' MFMAs (not one); the barriers are raw s_barrier +
  // lgkmcnt(0) (a __syncthreads would drain vmcnt and kill the loads in flight).  The loop is
  // unrolled by two so every stage index is a compile-time constant (no register-array
  // indexing -> no scratch).
  typedef typename StagerSel<VEC, BM, !TA, TAe>::type SA;
  typedef typename StagerSel<VEC, BN, TB, TBe>::type SB;
  SA sa0, sa1;
  SB sb0, sb1;
  f32x4 acc[T::FM][T::FN];
#pragma unroll
  for (int i = 0; i < T::FM; ++i)
#pragma unroll
    for (int j = 0; j < T::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kend > kbeg ? (kend - kbeg + T::BK - 1) / T::BK : 0;
  sa0.load(A, lda, row0, kbeg, M, kend, tid);
  sb0.load(B, ldb, col0, kbeg, N, kend, tid);
  sa1.load(A, lda, row0, kbeg + T::BK, M, kend, tid);
  sb1.load(B, ldb, col0, kbeg + T::BK, N, kend, tid);
  if (nk > 0) {
    sa0.store(As, tid);
    sb0.store(Bs, tid);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  auto mfma_tile = [&]() {
#pragma unroll
    for (int ks = 0; ks < T::BK / 32; ++ks) {
      bf16x8 af[T::FM], bfr[T::FN];
#pragma unroll
      for (int i = 0; i < T::FM; ++i) af[i] = frag<BM, !TA>(As, wm * T::WM + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < T::FN; ++j) bfr[j] = frag<BN, TB>(Bs, wn * T::WN + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < T::FM; ++i)
#pragma unroll
        for (int j = 0; j < T::FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  };
  // Per tile: refill loads (tile it+2) -> MFMAs on the LDS tile -> barrier -> tile it+1 from
  // registers into LDS -> barrier.  The refill loads are UNCONDITIONAL (past kend they read
  // clamped addresses and are zeroed / never stored): conditional loads make the compiler's
  // wait counting merge paths and emit vmcnt(0), which would wait for the tile just issued.
  for (int it = 0; it < nk; it += 2) {
    sa0.load(A, lda, row0, kbeg + (it + 2) * T::BK, M, kend, tid);
    sb0.load(B, ldb, col0, kbeg + (it + 2) * T::BK, N, kend, tid);
    mfma_tile();
    if (it + 1 >= nk) break;
    asm volatile("s_barrier" ::: "memory");
    sa1.store(As, tid);
    sb1.store(Bs, tid);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    sa1.load(A, lda, row0, kbeg + (it + 3) * T::BK, M, kend, tid);
    sb1.load(B, ldb, col0, kbeg + (it + 3) * T::BK, N, kend, tid);
    mfma_tile();
    if (it + 2 >= nk) break;
    asm volatile("s_barrier" ::: "memory");
    sa0.store(As, tid);
    sb0.store(Bs, tid);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

#undef As
#undef Bs
  // epilogue
  float* slab = P.slab;
  if constexpr (T::FM * T::FN <= SPLITK_INLAUNCH_FRAGS) {
    if (slab && g.cnt) {
      asm volatile("s_barrier" ::: "memory");  // the last tile's LDS reads are done: reuse smem
      splitk_epilogue<T::FM, T::FN, T::WM, T::WN>(g, P, acc, gtile, row0, col0, wm, wn, lane,
                                                  reinterpret_cast<int*>(smem));
      return;
    }
  }
  const int nst = (slab || P.epi.ncol <= 0) ? N : min(N, P.epi.ncol);
#pragma unroll
  for (int i = 0; i < T::FM; ++i)
#pragma unroll
    for (int j = 0; j < T::FN; ++j) {
      const int col = col0 + wn * T::WN + 16 * j + (lane & 15);
      if (col >= nst) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * T::WM + 16 * i + 4 * (lane >> 4) + r;
        if (row >= M) continue;
        if (slab) slab[((long)blockIdx.z * M + row) * N + col] = acc[i][j][r];
        else epi_store(P.epi, P.C, P.ldc, row, col, acc[i][j][r]);
      }
    }
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA GEMM for bf16 operands (the common case: every ICA-step GEMM).  Tiles go global -> LDS
// by global_load_lds_dwordx4 (16 B per lane, no VGPR round trip, no conversion pass), into two
// LDS stages: tile t+1's DMA is in flight under tile t's MFMAs, one vmcnt(0) + barrier per K tile.
// The DMA writes LDS lane-linearly (1 KB per wave instruction), so the bank-conflict swizzles are
// applied on the per-lane SOURCE address and undone on the read:
//  k-contiguous image [rows][64 k] (128-B rows): chunk slot = chunk ^ ((row >> 1) & 7) -> the 16
//    rows of a ds_read_b128 group hit 16 distinct bank quads;
//  k-major image [64 k][C cols]: C = 128 (256-B rows) slot = chunk ^ sw256(k), C = 64 (128-B rows)
//    slot = chunk ^ sw128(k) -> each 32-lane half of a ds_read_b64_tr_b16 fragment read (8 k-rows x
//    2 chunks) covers 64 distinct banks.
// Out-of-range 16-B chunks (ragged M / N / K, split-K slice ends) read a zero page instead, so the
// loop carries no masks.  Contract (host-checked): both operands bf16, GemmGroup::vec.
__device__ const uint4 g_gemm_zero[1] = {};
// a 16-B chunk of 8 bf16 columns {1, 0, ..., 0}: the virtual ones column (Epi::xcol)
__device__ const uint4 g_gemm_unit[1] = {{0x3f80u, 0u, 0u, 0u}};

__device__ __forceinline__ int sw_kc(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int sw_km256(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }
__device__ __forceinline__ int sw_km128(int k) { return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1; }

typedef __attribute__((address_space(3))) void lds_void;

template <int ROWS, bool KCONTIG, int NW = 4>
struct DmaImg {
  static constexpr int BYTES = ROWS * 64 * 2;    // one 64-deep K tile
  static constexpr int PER_WAVE = BYTES / 1024 / NW;  // 1 KB DMA instructions per wave
};

// This wave's share of the DMA of operand rows [row0, row0 + ROWS) x k [k, k + 64), as per-lane
// source pointers fixed for the whole K loop (row / column part and swizzle folded in once; a K
// tile only adds its k offset).  A lane whose row (column) is out of range keeps a null pointer
// and reads the zero page; the k range is checked per tile (K % 8 == 0: chunks are all in or out).
template <int ROWS, bool KCONTIG, int NW = 4>
struct DmaStream {
  static constexpr int PW = DmaImg<ROWS, KCONTIG, NW>::PER_WAVE;
  const bf16* p[PW];
  int kofs[PW];  // the chunk's k offset within the tile
  long kstep;    // elements per unit of k
  int ins0;
  unsigned unit;  // bit j: chunk j is the virtual ones column (k-major operands only)
  // k-major row gather (RowGather on this operand): p[j] holds the column part only, the row
  // part comes from the subjects of each K tile (two scalar loads per tile: gs >= 64)
  const long long* subj;
  int gs;
  long ldr;
  // unitcol >= 0 (k-major only, a multiple of 8): the 8 columns from unitcol read {1, 0, .., 0}
  __device__ __forceinline__ void init(const bf16* __restrict__ base, long ld, int row0, int nrows,
                                       int wid, int lane, int unitcol = -1,
                                       const bf16* ggx = nullptr,
                                       const long long* gsubj = nullptr, int ggs = 1,
                                       int ggr0 = 0) {
    ins0 = wid * PW;
    kstep = KCONTIG ? 1 : ld;
    unit = 0;
    subj = nullptr;
    gs = 1;
    ldr = ld;
    if (ggx) {  // gathered rows (RowGather): read the dataset, not the operand pointer
      base = ggx;
      subj = gsubj;
      gs = ggs;
    }
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int ins = ins0 + j;
      if constexpr (KCONTIG) {
        const int r = ins * 8 + (lane >> 3);
        const int ch = (lane & 7) ^ sw_kc(r);
        const int gr = row0 + r;
        kofs[j] = 8 * ch;
        long row = gr;
        if (subj && gr < nrows) {  // operand row gr -> dataset row (once per workgroup)
          const int gg = gr + ggr0;
          const int b = gg / gs;
          row = subj[b] * gs + (gg - b * gs);
        }
        p[j] = gr < nrows ? base + row * ld + 8 * ch : nullptr;
      } else {
        constexpr int CPR = ROWS / 8;
        constexpr int RPI = 64 / CPR;
        const int kr = ins * RPI + lane / CPR;
        // (512-B rows of a 256-column image take the 256-B rule: the bank of a chunk only sees
        // the row offset mod 256 B, which is 0 for both)
        const int ch = (lane % CPR) ^ (ROWS >= 128 ? sw_km256(kr) : sw_km128(kr));
        const int gc = row0 + 8 * ch;
        kofs[j] = kr;
        p[j] = gc < nrows ? base + (subj ? 0L : (long)kr * ld) + gc : nullptr;
        if (gc == unitcol) {
          unit |= 1u << j;
          p[j] = reinterpret_cast<const bf16*>(g_gemm_unit);
        }
      }
    }
  }
  __device__ __forceinline__ void issue(int k0, int K, char* img) const {
    if (!KCONTIG && subj) {  // k rows k0 .. k0 + 63 span at most two subjects (gs >= 64)
      typedef const __attribute__((address_space(4))) long long csubj;
      const int b0 = __builtin_amdgcn_readfirstlane(k0 / gs);
      const long long s0 = ((csubj*)subj)[b0], s1 = ((csubj*)subj)[b0 + 1];
      const int kb = (b0 + 1) * gs;
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        const int k = k0 + kofs[j];
        const bool ok = p[j] != nullptr && k < K;
        const long row = k < kb ? s0 * gs + (k - b0 * gs) : s1 * gs + (k - kb);
        const bf16* src = !ok ? reinterpret_cast<const bf16*>(g_gemm_zero)
                          : ((unit >> j) & 1u) ? p[j] : p[j] + row * ldr;
        __builtin_amdgcn_global_load_lds(src, (lds_void*)(img + (ins0 + j) * 1024), 16, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const bool ok = p[j] != nullptr && k0 + kofs[j] < K;
      const bf16* src = !ok ? reinterpret_cast<const bf16*>(g_gemm_zero)
                        : ((unit >> j) & 1u) ? p[j] : p[j] + (long)k0 * kstep;
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(img + (ins0 + j) * 1024), 16, 0, 0);
    }
  }
};

// ds_read_b64_tr_b16 as inline asm: hipcc treats the builtin as an LDS read it cannot alias-check
// against the LDS-DMA ring, and waits vmcnt(0) before it -- draining the prefetched tiles.  The
// asm form is invisible to that bookkeeping, so the caller waits lgkmcnt(0) (+ sched_barrier)
// itself before the MFMAs consume the result.
__device__ __forceinline__ s16x4 tr16_asm(const char* p) {
  s16x4 v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

// 16x32 MFMA operand fragment (operand rows r0 .. r0 + 15, k = 32 ks .. +31) from a DMA image
template <int ROWS, bool KCONTIG>
__device__ __forceinline__ bf16x8 dma_frag(const char* img, int r0, int ks, int lane) {
  if constexpr (KCONTIG) {
    const int r = r0 + (lane & 15);
    const int ch = 4 * ks + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * (ch ^ sw_kc(r)));
  } else {
    constexpr int RB = ROWS * 2;
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k0 = 32 * ks + 8 * g + q, k1 = k0 + 4;
    const int ch = (r0 >> 3) + (p >> 1);
    const int s0 = ROWS >= 128 ? sw_km256(k0) : sw_km128(k0);
    const int s1 = ROWS >= 128 ? sw_km256(k1) : sw_km128(k1);
    const s16x4 x0 = tr16_asm(img + k0 * RB + 16 * (ch ^ s0) + 8 * (p & 1));
    const s16x4 x1 = tr16_asm(img + k1 * RB + 16 * (ch ^ s1) + 8 * (p & 1));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

// LDS bytes of gemm_dma_kernel<BM, BN, TA, TB, S>: the S-stage ring or the epilogue staging
template <int BM, int BN, bool TA, bool TB, int S>
constexpr int dma_smem() {
  constexpr int STAGE = DmaImg<BM, !TA>::BYTES + DmaImg<BN, TB>::BYTES;
  constexpr int EBYTES = 4 * (BM / 2) * (BN / 2 + 4) * 4;
  return S * STAGE > EBYTES ? S * STAGE : EBYTES;
}

// s_waitcnt vmcnt(n), 0 <= n < 64 (vmcnt bits [3:0] and [15:14])
#define DN_VMWAIT(n) __builtin_amdgcn_s_waitcnt(DN_VMCNT0 | ((n) & 15) | (((n) >> 4) << 14))

template <int BM, int BN, bool TA, bool TB, int S>
__global__ void __launch_bounds__(256)
gemm_dma_kernel(GemmGroup g) {
  static_assert(S >= 2 && S <= 8, "ring depth");
  typedef DmaImg<BM, !TA> IA;
  typedef DmaImg<BN, TB> IB;
  constexpr int STAGE = IA::BYTES + IB::BYTES;
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  constexpr int ES = WN + 4;                 // fp32 epilogue row stride (per-wave WM x WN block)
  // one dynamic LDS array (dma_smem bytes; a second __shared__ object beside a glds ring can
  // make hipcc drain vmcnt before LDS reads): the 8-stage ring is 128 KB, past the static limit
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int ntiles = g.tile_start[g.n];
  const int bid = (int)blockIdx.x;
  const int slot = (bid & 7) * ((int)gridDim.x >> 3) + (bid >> 3);  // XCD-contiguous slots
  if (slot >= ntiles) return;
  group_bump(g);
  const int gtile = g.perm ? g.perm[slot] : slot;
  const int pi = group_prob(g, g.tile_start, gtile);
  const GemmProb& P = g.p[pi];
  const bf16* __restrict__ A = reinterpret_cast<const bf16*>(P.A);
  const bf16* __restrict__ B = reinterpret_cast<const bf16*>(P.B);
  const int M = P.M, N = P.N, K = P.K;
  const int tile = gtile - g.tile_start[pi];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: the DMA's LDS base (M0)
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (N + BN - 1) / BN;
  const int row0 = (tile / tiles_n) * BM, col0 = (tile % tiles_n) * BN;
  const int kbeg = blockIdx.z * P.kchunk;
  const int kend = min(K, kbeg + P.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + 63) / 64 : 0;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  DmaStream<BM, !TA> sa;
  DmaStream<BN, TB> sb;
  sa.init(A, P.lda, row0, M, wid, lane, -1, P.rg.op == 1 ? P.rg.gx : nullptr, P.rg.subj, P.rg.gs,
          P.rg.r0);
  sb.init(B, P.ldb, col0, P.epi.xcol >= 0 ? P.epi.xcol : N, wid, lane, P.epi.xcol,
          P.rg.op == 2 ? P.rg.gx : nullptr, P.rg.subj, P.rg.gs);
  // S-stage ring, tiles prefetched D = S - 1 ahead: at the top of iteration t this wave waits
  // until only the glds of tiles t+1 .. t+D-1 are outstanding (counted vmcnt, never 0 in the
  // steady state), one raw barrier makes every wave's share of tile t visible and retires the
  // reads of iteration t-1 (whose buffer tile t+D then refills), then the MFMAs run on tile t.
  constexpr int D = S - 1;
  constexpr int G = DmaStream<BM, !TA>::PW + DmaStream<BN, TB>::PW;  // glds per wave per tile
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < nk) {
      sa.issue(kbeg + 64 * d, kend, smem + d * STAGE);
      sb.issue(kbeg + 64 * d, kend, smem + d * STAGE + IA::BYTES);
    }
  for (int t = 0; t < nk; ++t) {
    const int ahead = min(D - 1, nk - 1 - t);  // tiles after t already issued
    static_assert((D - 1) * G < 64, "vmcnt range");
    // (an immediate per count: one wave-uniform branch)
    if (D - 1 >= 6 && ahead >= 6) DN_VMWAIT(6 * G);
    else if (D - 1 >= 5 && ahead == 5) DN_VMWAIT(5 * G);
    else if (D - 1 >= 4 && ahead == 4) DN_VMWAIT(4 * G);
    else if (D - 1 >= 3 && ahead == 3) DN_VMWAIT(3 * G);
    else if (ahead >= 2) DN_VMWAIT(2 * G);
    else if (ahead == 1) DN_VMWAIT(G);
    else DN_VMWAIT(0);
    __builtin_amdgcn_s_barrier();
    if (t + D < nk) {
      char* nxt = smem + ((t + D) % S) * STAGE;
      sa.issue(kbeg + 64 * (t + D), kend, nxt);
      sb.issue(kbeg + 64 * (t + D), kend, nxt + IA::BYTES);
    }
    const char* cur = smem + (t % S) * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = dma_frag<BM, !TA>(cur, wm * WM + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = dma_frag<BN, TB>(cur + IA::BYTES, wn * WN + 16 * j, ks, lane);
      if constexpr (TA || !TB) {  // asm transposed reads: retire them before the MFMAs
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the ring

  if (g.vepi) {
    // LDS-staged epilogue: alpha / bias / ReLU applied in registers, the wave's WM x WN block
    // goes through LDS (the K loop's last barrier freed it), then out as 16-B row vectors (the
    // MFMA layout alone would store 2- or 4-byte pieces, 16 lanes per row segment)
    float* E = reinterpret_cast<float*>(smem) + wid * WM * ES;
    const Epi& ep = P.epi;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int lc = 16 * j + (lane & 15);
      const int col = col0 + wn * WN + lc;
      const float bias = (ep.bias && col < N) ? ep.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] * ep.alpha + bias;
          if (ep.relu) v = fmaxf(v, 0.f);
          E[(16 * i + 4 * (lane >> 4) + r) * ES + lc] = v;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    const int gr0 = row0 + wm * WM, gc0 = col0 + wn * WN;
    if (ep.out_bf16) {
      constexpr int CPR = WN / 8, RPI = 64 / CPR;  // 8-column vectors per row, rows per pass
#pragma unroll
      for (int it = 0; it < WM / RPI; ++it) {
        const int lr = it * RPI + lane / CPR, lc = 8 * (lane % CPR);
        const int row = gr0 + lr, col = gc0 + lc;
        if (row >= M || col >= N) continue;
        const f32x4 a = *reinterpret_cast<const f32x4*>(E + lr * ES + lc);
        const f32x4 b = *reinterpret_cast<const f32x4*>(E + lr * ES + lc + 4);
        bf16x8* cp = reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(P.C) + (long)row * P.ldc + col);
        float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
        if (ep.mask) {
          const bf16x8 m = *reinterpret_cast<const bf16x8*>(ep.mask + (long)row * ep.ldm + col);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (float)m[e] > 0.f ? v[e] : 0.f;
        }
        if (ep.beta != 0.f) {
          const bf16x8 o = *cp;
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += ep.beta * (float)o[e];
        }
        bf16x8 w;
#pragma unroll
        for (int e = 0; e < 8; ++e) w[e] = (bf16)v[e];
        *cp = w;
      }
    } else {
      constexpr int CPR = WN / 4, RPI = 64 / CPR;
#pragma unroll
      for (int it = 0; it < WM / RPI; ++it) {
        const int lr = it * RPI + lane / CPR, lc = 4 * (lane % CPR);
        const int row = gr0 + lr, col = gc0 + lc;
        if (row >= M || col >= N) continue;
        f32x4 v = *reinterpret_cast<const f32x4*>(E + lr * ES + lc);
        f32x4* cp = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(P.C) + (long)row * P.ldc + col);
        if (ep.mask) {
          const bf16x4 m = *reinterpret_cast<const bf16x4*>(ep.mask + (long)row * ep.ldm + col);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (float)m[e] > 0.f ? v[e] : 0.f;
        }
        if (ep.beta != 0.f) {
          const f32x4 o = *cp;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += ep.beta * o[e];
        }
        *cp = v;
      }
    }
    return;
  }
  float* slab = P.slab;
  if constexpr (FM * FN <= SPLITK_INLAUNCH_FRAGS) {
    if (slab && g.cnt) {
      splitk_epilogue<FM, FN, WM, WN>(g, P, acc, gtile, row0, col0, wm, wn, lane,
                                      reinterpret_cast<int*>(smem));
      return;
    }
  }
  const int nst = (slab || P.epi.ncol <= 0) ? N : min(N, P.epi.ncol);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = col0 + wn * WN + 16 * j + (lane & 15);
      if (col >= nst) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * WM + 16 * i + 4 * (lane >> 4) + r;
        if (row >= M) continue;
        if (slab) slab[((long)blockIdx.z * M + row) * N + col] = acc[i][j][r];
        else epi_store(P.epi, P.C, P.ldc, row, col, acc[i][j][r]);
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Large GEMMs of the ICA step at B >= 1024 (M = B*S rows; the weight gradients' K = B*S):
// 256 x 256 tiles, 8 waves (2 x 4, 128 x 64 outputs and 32 accumulator fragments each), BK = 64,
// every operand layout (k-major images read with ds_read_b64_tr_b16), staged by LDS-DMA into two
// 64 KB stages of dynamic LDS: one workgroup per CU at two waves per SIMD, tile t+1's DMA in
// flight under tile t's 64 MFMAs per wave.  Against the 128 x 128 kernel a tile reads half the
// operand bytes per MFMA, and at N = 256 one workgroup streams its A rows exactly once
// (cdna_hip_programming §5: the 256^2 tile with a glds pipeline).  Epilogue: the LDS-staged vector
// path in four passes of 32 rows per wave (the ring's 128 KB cannot hold eight 128 x 64 fp32
// blocks at once), into C (bias / ReLU / mask / beta) or, split-K, raw into the fp32 slab that
// gemm_splitk_reduce combines (which also applies row maps and the virtual ones column).
constexpr int G256_SMEM = 2 * (256 * 64 * 2) * 2;  // two stages of A + B images

template <bool TA, bool TB>
__global__ void __launch_bounds__(512)
gemm256_kernel(GemmGroup g) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  constexpr int BM = 256, BN = 256, NW = 8, WM = 128, WN = 64, FM = WM / 16, FN = WN / 16;
  typedef DmaImg<BM, !TA, NW> IA;
  typedef DmaImg<BN, TB, NW> IB;
  constexpr int STAGE = IA::BYTES + IB::BYTES;

  const int ntiles = g.tile_start[g.n];
  const int bid = (int)blockIdx.x;
  const int slot = (bid & 7) * ((int)gridDim.x >> 3) + (bid >> 3);  // XCD-contiguous slots
  if (slot >= ntiles) return;
  group_bump(g);
  const int gtile = g.perm ? g.perm[slot] : slot;
  const int pi = group_prob(g, g.tile_start, gtile);
  const GemmProb& P = g.p[pi];
  const bf16* __restrict__ A = reinterpret_cast<const bf16*>(P.A);
  const bf16* __restrict__ B = reinterpret_cast<const bf16*>(P.B);
  const int M = P.M, N = P.N, K = P.K;
  const int tile = gtile - g.tile_start[pi];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int tiles_n = (N + BN - 1) / BN;
  const int row0 = (tile / tiles_n) * BM, col0 = (tile % tiles_n) * BN;
  const int kbeg = blockIdx.z * P.kchunk;
  const int kend = min(K, kbeg + P.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + 63) / 64 : 0;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  DmaStream<BM, !TA, NW> sa;
  DmaStream<BN, TB, NW> sb;
  sa.init(A, P.lda, row0, M, wid, lane, -1, P.rg.op == 1 ? P.rg.gx : nullptr, P.rg.subj, P.rg.gs,
          P.rg.r0);
  sb.init(B, P.ldb, col0, P.epi.xcol >= 0 ? P.epi.xcol : N, wid, lane, P.epi.xcol,
          P.rg.op == 2 ? P.rg.gx : nullptr, P.rg.subj, P.rg.gs);
  if (nk > 0) {
    sa.issue(kbeg, kend, smem);
    sb.issue(kbeg, kend, smem + IA::BYTES);
  }
  for (int t = 0; t < nk; ++t) {
    __builtin_amdgcn_s_waitcnt(DN_VMCNT0);  // this wave's share of tile t has landed
    __builtin_amdgcn_s_barrier();           // ... every wave's; stage (t+1)&1 is free again
    if (t + 1 < nk) {
      char* nxt = smem + ((t + 1) & 1) * STAGE;
      sa.issue(kbeg + 64 * (t + 1), kend, nxt);
      sb.issue(kbeg + 64 * (t + 1), kend, nxt + IA::BYTES);
    }
    const char* cur = smem + (t & 1) * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = dma_frag<BN, TB>(cur + IA::BYTES, wn * WN + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = dma_frag<BM, !TA>(cur, wm * WM + 16 * i, ks, lane);
      if constexpr (TA || !TB) {  // asm transposed reads: retire them before the MFMAs
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the ring

  const Epi& ep = P.epi;
  // split-K: raw partials into this split's fp32 slab [M][N] (the reduce kernel applies Epi);
  // else (host contract: g.vepi) bias / ReLU / mask / beta into C, no row map, 16-B rows
  const bool raw = P.slab != nullptr;
  void* const Cd = raw ? (void*)(P.slab + (long)blockIdx.z * M * N) : P.C;
  const long ldc = raw ? (long)N : P.ldc;
  const float alpha = raw ? 1.f : ep.alpha, beta = raw ? 0.f : ep.beta;
  const float* const ebias = raw ? nullptr : ep.bias;
  const bf16* const emask = raw ? nullptr : ep.mask;
  const int relu = raw ? 0 : ep.relu, obf = raw ? 0 : ep.out_bf16;
  {
    constexpr int ES = WN + 4;  // fp32 staging row stride
    float* E = reinterpret_cast<float*>(smem) + wid * 32 * ES;
#pragma unroll
    for (int pass = 0; pass < FM / 2; ++pass) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int lc = 16 * j + (lane & 15);
        const int col = col0 + wn * WN + lc;
        const float bias = (ebias && col < N) ? ebias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[2 * pass + i][j][r] * alpha + bias;
            if (relu) v = fmaxf(v, 0.f);
            E[(16 * i + 4 * (lane >> 4) + r) * ES + lc] = v;
          }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
      const int gr0 = row0 + wm * WM + 32 * pass, gc0 = col0 + wn * WN;
      if (obf) {
        constexpr int CPR = WN / 8, RPI = 64 / CPR;  // 8 vectors per row, 8 rows per round
#pragma unroll
        for (int it = 0; it < 32 / RPI; ++it) {
          const int lr = it * RPI + lane / CPR, lc = 8 * (lane % CPR);
          const int row = gr0 + lr, col = gc0 + lc;
          if (row >= M || col >= N) continue;
          const f32x4 a = *reinterpret_cast<const f32x4*>(E + lr * ES + lc);
          const f32x4 b = *reinterpret_cast<const f32x4*>(E + lr * ES + lc + 4);
          bf16x8* cp = reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(Cd) + (long)row * ldc + col);
          float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
          if (emask) {
            const bf16x8 m = *reinterpret_cast<const bf16x8*>(emask + (long)row * ep.ldm + col);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (float)m[e] > 0.f ? v[e] : 0.f;
          }
          if (beta != 0.f) {
            const bf16x8 o = *cp;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += beta * (float)o[e];
          }
          bf16x8 w;
#pragma unroll
          for (int e = 0; e < 8; ++e) w[e] = (bf16)v[e];
          *cp = w;
        }
      } else {
        constexpr int CPR = WN / 4, RPI = 64 / CPR;
#pragma unroll
        for (int it = 0; it < 32 / RPI; ++it) {
          const int lr = it * RPI + lane / CPR, lc = 4 * (lane % CPR);
          const int row = gr0 + lr, col = gc0 + lc;
          if (row >= M || col >= N) continue;
          f32x4 v = *reinterpret_cast<const f32x4*>(E + lr * ES + lc);
          f32x4* cp = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Cd) + (long)row * ldc + col);
          if (emask) {
            const bf16x4 m = *reinterpret_cast<const bf16x4*>(emask + (long)row * ep.ldm + col);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (float)m[e] > 0.f ? v[e] : 0.f;
          }
          if (beta != 0.f) {
            const f32x4 o = *cp;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += beta * o[e];
          }
          *cp = v;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();  // the next pass rewrites this wave's staging rows
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
  }
}

// 4 consecutive outputs of one row: v (already alpha-free split sum) -> epilogue -> vector store
__device__ __forceinline__ void epi_store4(const Epi& epi, void* C, long ldc, int row, int col, f32x4 v,
                                           long orow = -2) {
  if (epi.xcol >= 0 && col + 3 >= epi.xcol) {  // the column-sum group (xcol % 4 == 0)
    epi_store(epi, C, ldc, row, col, v[0]);
    return;
  }
  if (orow == -2) orow = epi.row_map ? epi.row_map[row] : row;  // else: the caller's, loaded early
  if (orow < 0) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] *= epi.alpha;
    if (epi.bias) v[e] += epi.bias[col + e];
    if (epi.relu) v[e] = fmaxf(v[e], 0.f);
    if (epi.mask && !((float)epi.mask[(long)row * epi.ldm + col + e] > 0.f)) v[e] = 0.f;
  }
  for (int oo = 0; oo < (epi.C2 ? 2 : 1); ++oo) {
    void* Co = oo ? epi.C2 : C;
    f32x4 u = v;
    if (epi.out_bf16) {
      bf16x4* cp = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(Co) + orow * ldc + col);
      if (epi.beta != 0.f) {
        const bf16x4 o = *cp;
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] += epi.beta * (float)o[e];
      }
      bf16x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (bf16)u[e];
      *cp = w;
    } else {
      f32x4* cp = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Co) + orow * ldc + col);
      if (epi.beta != 0.f) {
        const f32x4 o = *cp;
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] += epi.beta * o[e];
      }
      *cp = u;
    }
  }
}

// deterministic split-K combine + epilogue over every problem of a group; each thread handles
// 4 consecutive columns of one row.  Rows of N % 4 == 0 problems (every ICA shape) take 16-B
// slab loads (all splits issued together) and 16-B stores; others the scalar path.
__global__ void __launch_bounds__(256) gemm_splitk_reduce(GemmGroup g) {
  const long total = g.elem_start[g.n];
  for (long i4 = blockIdx.x * (long)blockDim.x + threadIdx.x; 4 * i4 < total;
       i4 += (long)gridDim.x * blockDim.x) {
    const long idx0 = 4 * i4;
    const int pi = group_prob(g, g.elem_start, idx0);
    const GemmProb& P = g.p[pi];
    const long base = g.elem_start[pi];
    const long mn = (long)P.M * P.N;
    const long idx = idx0 - base;
    if (idx >= mn) continue;
    const bool vec = P.epi.ncol <= 0 && (P.N & 3) == 0 && (P.ldc & 3) == 0 &&
                     ((((uintptr_t)P.C) & 15) == 0) &&
                     ((((uintptr_t)P.slab) & 15) == 0);
    if (vec) {
      // the output row (and its row-map entry) first: that load then overlaps the slab loads
      // instead of following them
      const int row = (int)(idx / P.N), col = (int)(idx - (long)row * P.N);
      const long orow = P.epi.row_map ? P.epi.row_map[row] : row;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      int s = 0;
      for (; s + 4 <= g.splits; s += 4) {  // four slab loads in flight per round
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(P.slab + (long)s * mn + idx);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(P.slab + (long)(s + 1) * mn + idx);
        const f32x4 a2 = *reinterpret_cast<const f32x4*>(P.slab + (long)(s + 2) * mn + idx);
        const f32x4 a3 = *reinterpret_cast<const f32x4*>(P.slab + (long)(s + 3) * mn + idx);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += ((a0[e] + a1[e]) + a2[e]) + a3[e];
      }
      for (; s < g.splits; ++s) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(P.slab + (long)s * mn + idx);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += a[e];
      }
      epi_store4(P.epi, P.C, P.ldc, row, col, v, orow);
      continue;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long ie = idx + e;
      if (ie < mn && (P.epi.ncol <= 0 || ie % P.N < P.epi.ncol)) {
        float v = 0.f;
        for (int s = 0; s < g.splits; ++s) v += P.slab[(long)s * mn + ie];
        const int row = (int)(ie / P.N), col = (int)(ie - (long)row * P.N);
        epi_store(P.epi, P.C, P.ldc, row, col, v);
      }
    }
  }
}

static int g_gemm_dma = 1;  // bf16 x bf16 aligned groups take gemm_dma_kernel (A/B switch)
// largest grid (workgroups) of 64 x 64 tiles that takes the 8-stage ring (DN_GEMM_RING8_MAX; default
// 0 = off: measured slower at the B = 32 step, encoder 10.2 vs 9.2 us and input gradient 15.5 vs
// 14.2 -- those K loops are not bound by the tiles in flight, 0.3146 vs 0.3116 ms/step)
static const long g_ring8_max = [] {
  const char* e = getenv("DN_GEMM_RING8_MAX");
  return e ? atol(e) : 0L;
}();

// largest grid (exclusive) of 64 x 64 tiles that takes the 4-stage ring (DN_GEMM_RING4_MAX, default
// 512: from there two workgroups per CU hold the 2-stage ring's tile in flight each; the B = 32
// step's grouped weight gradients, 568 workgroups, took 26.7 vs 21.1 us on the 4-stage ring,
// 0.3181-0.3192 vs 0.3107-0.3110 ms/step)
static const long g_ring4_max = [] {
  const char* e = getenv("DN_GEMM_RING4_MAX");
  return e ? atol(e) : 512L;
}();

static int kchunk_for(int K, int& splits) {
  int kchunk = K;
  if (splits > 1) {
    kchunk = (K + splits - 1) / splits;
    kchunk = (kchunk + 63) / 64 * 64;
  }
  return kchunk;
}

template <int BM, int BN, bool TA, bool TB, typename TAe, typename TBe>
int launch(GemmGroup& g, hipStream_t st) {
  // the combiner's partial loads do not fit beside a 128x128 tile's accumulators (they spilled
  // to scratch): those tiles always reduce in the second kernel
  if constexpr ((BM / 32) * (BN / 32) > SPLITK_INLAUNCH_FRAGS) g.cnt = nullptr;  // 2x2 waves
  int tiles = 0;
  long elems = 0;
  for (int i = 0; i < g.n; ++i) {
    g.tile_start[i] = tiles;
    g.elem_start[i] = elems;
    tiles += ((g.p[i].M + BM - 1) / BM) * ((g.p[i].N + BN - 1) / BN);
    elems += ((long)g.p[i].M * g.p[i].N + 3) / 4 * 4;
  }
  g.tile_start[g.n] = tiles;
  g.elem_start[g.n] = elems;
  dim3 grid((tiles + 7) / 8 * 8, 1, g.splits);
  if constexpr (sizeof(TAe) == 2 && sizeof(TBe) == 2) {
    // ring depth: a grid that fills the chip several times over hides the DMA latency with
    // resident workgroups (2 stages, 32 KB at 64x64 -> 5 per CU); a small grid (the B = 32
    // step's ~200-tile GEMMs) needs the deeper 4-stage ring inside each workgroup
    // (DN_GEMM_RING8_MAX: a grid of at most that many workgroups takes the 8-stage ring, 128 KB
    // of LDS and seven tiles in flight per workgroup)
    const long wgs = (long)tiles * g.splits;
    if (g.vec && g_gemm_dma && BM == 64 && wgs <= g_ring8_max) {
      constexpr int SM = dma_smem<BM, BN, TA, TB, 8>();
      static bool init = false;
      if (!init) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_dma_kernel<BM, BN, TA, TB, 8>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, SM);
        init = true;
      }
      hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, TA, TB, 8>), grid, dim3(256), SM, st, g);
    } else if (g.vec && g_gemm_dma && BM == 64 && wgs < g_ring4_max)
      hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, TA, TB, 4>), grid, dim3(256),
                         (dma_smem<BM, BN, TA, TB, 4>()), st, g);
    else if (g.vec && g_gemm_dma)
      hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, TA, TB, 2>), grid, dim3(256),
                         (dma_smem<BM, BN, TA, TB, 2>()), st, g);
    else if (g.vec)
      hipLaunchKernelGGL((gemm_kernel<BM, BN, TA, TB, TAe, TBe, true>), grid, dim3(256), 0, st, g);
    else
      hipLaunchKernelGGL((gemm_kernel<BM, BN, TA, TB, TAe, TBe, false>), grid, dim3(256), 0, st, g);
  } else if (g.vec)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, TA, TB, TAe, TBe, true>), grid, dim3(256), 0, st, g);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, TA, TB, TAe, TBe, false>), grid, dim3(256), 0, st, g);
  if (g.splits > 1 && !g.cnt) {
    const long t4 = elems / 4;
    const int blocks = (int)((t4 + 255) / 256 < 4096 ? (t4 + 255) / 256 : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, st, g);
  }
  return dn_launch_status();
}

template <bool TA, bool TB>
static void launch256_t(GemmGroup& g, int tiles, hipStream_t st) {
  static bool init = false;
  if (!init) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm256_kernel<TA, TB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, G256_SMEM);
    init = true;
  }
  hipLaunchKernelGGL((gemm256_kernel<TA, TB>), dim3((tiles + 7) / 8 * 8, 1, g.splits), dim3(512),
                     G256_SMEM, st, g);
}

// 256 x 256 tiles (tile 2): bf16 operands on the LDS-DMA contract, split-K through the reduce
// kernel (no in-launch combine)
static int launch256(GemmGroup& g, int ta, int tb, hipStream_t st) {
  g.cnt = nullptr;
  int tiles = 0;
  long elems = 0;
  for (int i = 0; i < g.n; ++i) {
    g.tile_start[i] = tiles;
    g.elem_start[i] = elems;
    tiles += ((g.p[i].M + 255) / 256) * ((g.p[i].N + 255) / 256);
    elems += ((long)g.p[i].M * g.p[i].N + 3) / 4 * 4;
  }
  g.tile_start[g.n] = tiles;
  g.elem_start[g.n] = elems;
  if (!ta && !tb) launch256_t<false, false>(g, tiles, st);
  else if (!ta && tb) launch256_t<false, true>(g, tiles, st);
  else if (ta && !tb) launch256_t<true, false>(g, tiles, st);
  else launch256_t<true, true>(g, tiles, st);
  if (g.splits > 1) {
    const long t4 = elems / 4;
    const int blocks = (int)((t4 + 255) / 256 < 4096 ? (t4 + 255) / 256 : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, st, g);
  }
  return dn_launch_status();
}

template <int BM, int BN, typename TAe, typename TBe>
int dispatch_t(int ta, int tb, GemmGroup& g, hipStream_t st) {
  if (!ta && !tb) return launch<BM, BN, false, false, TAe, TBe>(g, st);
  if (!ta && tb) return launch<BM, BN, false, true, TAe, TBe>(g, st);
  if (ta && !tb) return launch<BM, BN, true, false, TAe, TBe>(g, st);
  return launch<BM, BN, true, true, TAe, TBe>(g, st);
}

template <int BM, int BN>
int dispatch_tile(int a_bf16, int b_bf16, int ta, int tb, GemmGroup& g, hipStream_t st) {
  if (a_bf16 && b_bf16) return dispatch_t<BM, BN, bf16, bf16>(ta, tb, g, st);
  if (a_bf16 && !b_bf16) return dispatch_t<BM, BN, bf16, float>(ta, tb, g, st);
  if (!a_bf16 && b_bf16) return dispatch_t<BM, BN, float, bf16>(ta, tb, g, st);
  return dispatch_t<BM, BN, float, float>(ta, tb, g, st);
}

// tile: 0 -> 64x64, 1 -> 128x128 (BM x BN), 2 -> 256x256 (bf16 operands on the LDS-DMA
// contract; other problems fall back to 128x128)
static bool aligned16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

// stage_load_vec's contract for one operand: contiguous-axis extent and leading dim % 8 == 0
static bool vec_ok(const void* base, int kcontig, int rows, int K, long ld) {
  return aligned16(base) && ld % 8 == 0 && (kcontig ? K % 8 == 0 : rows % 8 == 0);
}

int* g_bump_t = nullptr;
long long* g_bump_c = nullptr;

static int run_group(GemmGroup& g, int a_bf16, int b_bf16, int ta, int tb, int tile, hipStream_t st) {
  g.bump_t = g_bump_t;
  g.bump_c = g_bump_c;
  g_bump_t = nullptr;
  g_bump_c = nullptr;
  g.vec = 1;
  g.vepi = 1;
  bool xcol = false;
  for (int i = 0; i < g.n; ++i) {
    const GemmProb& P = g.p[i];
    const int nb = P.epi.xcol >= 0 ? P.epi.xcol : P.N;  // B's real columns
    if (!vec_ok(P.A, !ta, P.M, P.K, P.lda) || !vec_ok(P.B, tb, nb, P.K, P.ldb)) g.vec = 0;
    if (P.epi.xcol >= 0) {
      g.vepi = 0;
      xcol = true;
    }
    // 16-B output vectors: 8 columns (bf16) / 4 (fp32) never straddle N or a misaligned row
    const int cv = P.epi.out_bf16 ? 8 : 4;
    if (P.slab || P.epi.row_map || P.epi.ncol > 0 || P.N % cv || P.ldc % cv || !aligned16(P.C))
      g.vepi = 0;
    if (P.epi.mask && (P.epi.ldm % 8 || !aligned16(P.epi.mask))) g.vepi = 0;
  }
  // the virtual ones column exists only in the LDS-DMA kernel's k-major B stream
  if (xcol && (!g.vec || !g_gemm_dma || !a_bf16 || !b_bf16 || tb)) return DN_UNSUPPORTED;
  // gathered rows: the LDS-DMA kernels' streams only (A rows of a k-contiguous A, k rows of a
  // k-major B), whole 16-B chunks of an aligned dataset, at most two subjects per K tile
  for (int i = 0; i < g.n; ++i) {
    const RowGather& r = g.p[i].rg;
    if (!r.op) continue;
    if (!g.vec || !g_gemm_dma || !a_bf16 || !b_bf16 || !r.gx || !r.subj || r.gs < 64 ||
        !aligned16(r.gx) || (r.op == 1 && ta) || (r.op == 2 && tb) || r.op > 2)
      return DN_BAD_SHAPE;
  }
  if (tile == 2 && g.vec && g_gemm_dma && a_bf16 && b_bf16) {
    // the staged epilogue's contract: 16-B rows into C (vepi), or fp32 slabs of N % 4 == 0
    bool ok = g.splits > 1 || g.vepi;
    for (int i = 0; i < g.n && ok; ++i)
      if (g.splits > 1 && (g.p[i].N % 4 || (((uintptr_t)g.p[i].slab) & 15))) ok = false;
    if (ok) return launch256(g, ta, tb, st);
  }
  if (tile == 1 || tile == 2) return dispatch_tile<128, 128>(a_bf16, b_bf16, ta, tb, g, st);
  return dispatch_tile<64, 64>(a_bf16, b_bf16, ta, tb, g, st);
}

}  // namespace

// Arm a one-shot step-counter bump: the NEXT GEMM launch of this process advances *t (and *c when
// given) once, from workgroup 0, before any other kernel of the step reads them.  Issued at
// capture time, the pointers are baked into the captured launch.  dn_gemm_bump_armed reports a
// bump no launch consumed.
DN_API int dn_gemm_arm_bump(int* t, long long* c) {
  g_bump_t = t;  // null: disarm
  g_bump_c = t ? c : nullptr;
  return DN_OK;
}

DN_API int dn_gemm_bump_armed() { return g_bump_t != nullptr; }

// Hand the armed bump to a launch that is not a GEMM but starts with the encoder GEMM's work (the
// overlapped LSTM forward, lstm.hip dn_lstm_fwd_ov), disarming it; null pointers when none is armed.
DN_API int dn_gemm_take_bump(int** t, long long** c) {
  *t = g_bump_t;
  *c = g_bump_c;
  g_bump_t = nullptr;
  g_bump_c = nullptr;
  return DN_OK;
}

// 1: bf16 x bf16 GEMMs use the LDS-DMA kernel (default); 0: the register-staged kernel.
DN_API int dn_gemm_set_dma(int on) {
  g_gemm_dma = on != 0;
  return DN_OK;
}

// the current dn_gemm_set_dma setting (1: LDS-DMA kernel)
DN_API int dn_gemm_dma_on() { return g_gemm_dma; }

// Output tiles of a launch (the split-K ticket count `counters` must provide): 64x64 tiles
// (tile 0) or 128x128 (tile 1) summed over the problems.
DN_API long dn_gemm_tiles(int n, const int* M, const int* N, int tile) {
  const int b = tile == 1 ? 128 : 64;
  long t = 0;
  for (int i = 0; i < n; ++i) t += (long)((M[i] + b - 1) / b) * ((N[i] + b - 1) / b);
  return t;
}

// Returns the fp32 slab elements the caller must provide for a split-K launch (0 if none).
DN_API long dn_gemm_workspace(int M, int N, int K, int splits) {
  return splits > 1 ? (long)splits * M * N : 0;
}

// tile: see run_group
DN_API int dn_gemm(const void* A, int a_bf16, int ta, long lda, const void* B, int b_bf16, int tb,
                   long ldb, void* C, int c_bf16, long ldc, int M, int N, int K, float alpha,
                   float beta, const float* bias, int relu, const int* row_map, int tile,
                   int splits, float* slab, const void* mask, long ldm, int* counters,
                   const void* gx, const long long* subj, int gs, int gop, int gr0,
                   hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return DN_BAD_SHAPE;
  if (splits > 1 && !slab) return DN_BAD_SHAPE;
  GemmGroup g;
  g.cnt = splits > 1 && (long)splits * M * N < (1L << 29) ? counters : nullptr;
  g.perm = nullptr;
  g.n = 1;
  g.splits = splits > 1 ? splits : 1;
  GemmProb& P = g.p[0];
  P.A = A; P.B = B; P.C = C;
  P.lda = lda; P.ldb = ldb; P.ldc = ldc;
  P.M = M; P.N = N; P.K = K;
  P.kchunk = kchunk_for(K, g.splits);
  if (g.splits > 1) g.splits = (K + P.kchunk - 1) / P.kchunk;
  P.slab = g.splits > 1 ? slab : nullptr;
  P.epi = Epi{bias, row_map, alpha, beta, relu, c_bf16, 0, (const bf16*)mask, ldm, nullptr, -1,
              nullptr, nullptr};
  P.rg = RowGather{(const bf16*)gx, subj, gs, gx ? gop : 0, gx && gop == 1 ? gr0 : 0};
  return run_group(g, a_bf16, b_bf16, ta, tb, tile, st);
}

// Grouped GEMM: n <= GMAX (12) independent problems with the same operand layouts / element types /
// output type in ONE launch (+ one split-K reduce).  Per-problem arrays (`ncol` may be null: see
// Epi::ncol); `slab` holds
// splits * sum(M_i * N_i) fp32 when splits > 1.  Every problem uses the same K split count.
DN_API int dn_gemm_grouped(int n, const void* const* A, const long* lda, const void* const* B,
                           const long* ldb, void* const* C, const long* ldc, const int* M,
                           const int* N, const int* K, const float* alpha, const float* beta,
                           const void* const* bias, const void* const* row_map,
                           const int* ncol, void* const* C2, const int* xcol,
                           void* const* X1, void* const* X2, const int* perm, int relu,
                           int a_bf16, int b_bf16, int ta, int tb, int c_bf16, int tile,
                           int splits, float* slab, int* counters, void* const* GX,
                           void* const* SUBJ, const int* GS, const int* GOP, hipStream_t st) {
  if (n < 1 || n > GMAX) return DN_BAD_SHAPE;
  if (splits > 1 && !slab) return DN_BAD_SHAPE;
  GemmGroup g;
  g.cnt = splits > 1 ? counters : nullptr;
  g.perm = perm;
  g.n = n;
  g.splits = splits > 1 ? splits : 1;
  long soff = 0;
  for (int i = 0; i < n; ++i) {
    if (M[i] <= 0 || N[i] <= 0 || K[i] <= 0) return DN_BAD_SHAPE;
    GemmProb& P = g.p[i];
    P.A = A[i]; P.B = B[i]; P.C = C[i];
    P.lda = lda[i]; P.ldb = ldb[i]; P.ldc = ldc[i];
    P.M = M[i]; P.N = N[i]; P.K = K[i];
    int sp = g.splits;
    P.kchunk = kchunk_for(K[i], sp);
    P.slab = g.splits > 1 ? slab + soff : nullptr;
    soff += (long)g.splits * M[i] * N[i];
    if ((long)g.splits * M[i] * N[i] >= (1L << 29)) g.cnt = nullptr;  // 32-bit slab offsets
    P.epi = Epi{(const float*)bias[i], (const int*)row_map[i], alpha[i], beta[i], relu, c_bf16,
                ncol ? ncol[i] : 0, nullptr, 0, C2 ? C2[i] : nullptr,
                xcol ? xcol[i] : -1, X1 ? (float*)X1[i] : nullptr, X2 ? (float*)X2[i] : nullptr};
    P.rg = RowGather{};
    if (GX && GX[i])
      P.rg = RowGather{(const bf16*)GX[i], (const long long*)SUBJ[i], GS[i], GOP[i], 0};
    if (P.epi.C2 && !P.epi.ncol) return DN_BAD_SHAPE;  // second outputs: column sums only
    if (P.epi.xcol >= 0 && (N[i] != P.epi.xcol + 4 || P.epi.xcol % 8 || !P.epi.X1 || c_bf16 ||
                            P.epi.ncol > 0 || bias[i]))
      return DN_BAD_SHAPE;  // the ones column is the last one, fp32 outputs
  }
  return run_group(g, a_bf16, b_bf16, ta, tb, tile, st);
}
