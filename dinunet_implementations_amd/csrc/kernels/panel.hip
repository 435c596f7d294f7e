// Row-panel GEMM for the LSTM input projection at large batch:  C[M, N] (bf16) = A[M, K] W[N, K]^T
// with K <= 256 (the ICA input projection: M = B*S, K = 256, N = both directions' 4 * 192 gate
// columns = 1536).
//
// Why not the 256 x 256 tile kernel (gemm.hip gemm256_kernel): with K = 256 a tile's K loop is
// four 64-deep steps, so each tile is mostly its own prologue (operand DMA latency) and epilogue
// (128 KB of bf16 output through LDS staging) with one workgroup per CU and nothing overlapping
// them; and each 256-row block of A is re-read once per 256-column tile.  Here a persistent
// workgroup owns a contiguous range of (128-row block, column group) items:
//  * the 128 x K block of A is DMA'd into LDS ONCE per row block (global_load_lds, 64 KB), double
//    buffered: the next row block's DMA flies under the current block's items;
//  * W fragments come straight from global memory (W is 768 KB: L2-resident on every XCD) into
//    registers, each slot reloaded with the next 32-column pass's fragment once consumed;
//  * the product is formed transposed (MFMA A operand = W rows, B operand = A rows), so each lane
//    ends with 4 consecutive output columns of one row: bf16 stores straight from the
//    accumulators (8 B per lane, buffer stores range-checked per 128-row block), no LDS staging,
//    no barrier between passes -- a wave's stores drain under its next pass.
// 8 waves = 2 (64 rows each) x 4 (ncol / 4 columns each, in passes of 32).  The per-element sums
// are the same MFMA dot products in the same k order as gemm256_kernel's (bitwise equal output).
#include "common.h"

namespace {

constexpr int PN_BM = 128;                  // rows per A block
constexpr int PN_KMAX = 256;                // K <= 256 (one 512-B LDS row per A row)
constexpr int PN_ABYTES = PN_BM * PN_KMAX * 2;
constexpr int PN_SMEM = 2 * PN_ABYTES;      // double-buffered A block

__device__ const uint4 pn_zero[1] = {};
typedef __attribute__((address_space(3))) void pn_lds;
typedef unsigned pn_u32x2 __attribute__((ext_vector_type(2)));

struct PnArgs {
  const bf16* A;
  const bf16* W;
  bf16* C;
  long lda, ldw, ldc, M;
  int N, K, ncol;
  long nrb;  // 128-row blocks
};

// DMA A rows [row0, row0 + 128) x k [0, K) into img: [128 rows][32 slots of 16 B], slot =
// chunk ^ (row & 15) (a fragment read's 16 rows then hit 16 distinct bank quads).  global_load_lds
// writes LDS lane-linearly (1 KB per wave instruction = 2 rows), so the swizzle is applied on the
// source address.  Rows >= M and chunks >= K read a zero page.  8 waves x 8 instructions.
__device__ __forceinline__ void pn_issue_a(const PnArgs& a, long row0, char* img, int wid,
                                           int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int ins = wid * 8 + j;
    const int row = 2 * ins + (lane >> 5);
    const int ch = (lane & 31) ^ (row & 15);
    const long gr = row0 + row;
    const bool ok = gr < a.M && 8 * ch < a.K;
    const bf16* src = ok ? a.A + gr * a.lda + 8 * ch : reinterpret_cast<const bf16*>(pn_zero);
    __builtin_amdgcn_global_load_lds(src, (pn_lds*)(img + ins * 1024), 16, 0, 0);
  }
}

// ds_read_b128 as inline asm: hipcc cannot alias-check a plain LDS read against the in-flight
// LDS-DMA of the other buffer and would wait vmcnt(0) (the W prefetch and the stores) before
// every fragment; the caller waits lgkmcnt itself
__device__ __forceinline__ bf16x8 pn_ld128(const char* p) {
  bf16x8 v;
  const unsigned ad = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(ad) : "memory");
  return v;
}

// fragment of A rows r0 .. r0 + 15 (r0 % 16 == 0), k = 32 ks .. + 31, from the swizzled image
__device__ __forceinline__ bf16x8 pn_afrag(const char* img, int r0, int ks, int lane) {
  const int i = lane & 15;
  const int ch = 4 * ks + (lane >> 4);
  return pn_ld128(img + (r0 + i) * 512 + 16 * (ch ^ i));
}

template <int KS>  // K = 32 KS
__global__ void __launch_bounds__(512) panel_kernel(PnArgs a) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int nt = a.N / a.ncol;  // column groups per row block
  const long items = a.nrb * nt;
  const int G = (int)gridDim.x, bid = (int)blockIdx.x;
  // XCD-contiguous ranges (blocks b, b + 8, ... share an XCD): neighbouring row blocks' W and A
  // traffic stays in one L2 (G % 8 == 0, host-checked)
  const int w = (bid & 7) * (G >> 3) + (bid >> 3);
  const long i0 = items * w / G, i1 = items * (w + 1) / G;
  if (i0 >= i1) return;
  const int wcols = a.ncol >> 2;   // this wave's columns per item
  const int passes = wcols >> 5;   // 32 columns per pass
  const int mrow = 64 * wm;
  long rb = -1;
  int buf = 1;
  pn_issue_a(a, (i0 / nt) * PN_BM, smem, wid, lane);
  for (long it = i0; it < i1; ++it) {
    const long r = it / nt;
    if (r != rb) {
      // the block's DMA has landed for every wave, and every wave is done with the other buffer
      // (its last items belong to the previous block): free to take the next block's DMA
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      rb = r;
      buf ^= 1;
      if ((rb + 1) * nt < i1) pn_issue_a(a, (rb + 1) * PN_BM, smem + (buf ^ 1) * PN_ABYTES, wid, lane);
    }
    const char* img = smem + buf * PN_ABYTES;
    const long row0 = rb * PN_BM;
    const long vrows = a.M - row0 < PN_BM ? a.M - row0 : PN_BM;
    // stores of this block, range-checked by the hardware (rows >= M dropped)
    const __amdgpu_buffer_rsrc_t rc =
        dn_rsrc(a.C + row0 * a.ldc, (uint32_t)(vrows * a.ldc * 2));
    const int c0 = (int)(it - r * nt) * a.ncol + wn * wcols;
    // W fragments of a pass: [ni][ks], lane = column (lane & 15), k = 32 ks + 8 (lane >> 4)
    const bf16* wl = a.W + (long)(c0 + (lane & 15)) * a.ldw + 8 * (lane >> 4);
    bf16x8 bc[2][KS];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        bc[ni][ks] = *reinterpret_cast<const bf16x8*>(wl + (long)(16 * ni) * a.ldw + 32 * ks);
    for (int p = 0; p < passes; ++p) {
      // the next pass's W fragment of a slot is loaded into it as soon as this pass's MFMAs
      // have consumed it: a whole pass of latency, one register set (the last pass reloads its
      // own: unconditional loads keep hipcc's vmcnt bookkeeping exact, no branch joins)
      const bf16* wp = wl + (long)(32 * (p + 1 < passes ? p + 1 : p)) * a.ldw;
      f32x4 acc[2][4];
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) acc[ni][mi] = f32x4{0.f, 0.f, 0.f, 0.f};
      bf16x8 af[2][4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[0][mi] = pn_afrag(img, mrow + 16 * mi, 0, lane);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) {
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) af[(ks + 1) & 1][mi] = pn_afrag(img, mrow + 16 * mi, ks + 1, lane);
          asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) acc[ni][mi] = mfma16(bc[ni][ks], af[ks & 1][mi], acc[ni][mi]);
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          bc[ni][ks] = *reinterpret_cast<const bf16x8*>(wp + (long)(16 * ni) * a.ldw + 32 * ks);
      }
      // lane: rows mrow + 16 mi + (lane & 15), columns c0 + 32 p + 16 ni + 4 (lane >> 4) + 0..3
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const int row = mrow + 16 * mi + (lane & 15);
          const int col = c0 + 32 * p + 16 * ni + 4 * (lane >> 4);
          bf16x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (bf16)acc[ni][mi][e];
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(pn_u32x2, v), rc,
                                                (int)(((long)row * a.ldc + col) * 2), 0, 0);
        }
    }
  }
}

}  // namespace

// Column group per item: `ncol` > 0 forces it (a multiple of 128 dividing N), else the widest of
// 512 / 384 / 256 / 128 that still gives every workgroup of the grid an item.
static int pn_ncol(long nrb, int N, int G, int want) {
  if (want > 0) return (want % 128 == 0 && N % want == 0) ? want : 0;
  const int opts[4] = {512, 384, 256, 128};
  int best = 0;
  for (int o : opts) {
    if (N % o) continue;
    if (!best) best = o;
    if (nrb * (N / o) >= G) return o;
    best = o;
  }
  return best;
}

static int pn_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

// C[M, N] (bf16, row stride ldc) = A[M, K] (bf16, row stride lda) . W[N, K]^T (bf16, row stride
// ldw).  Contract: K in {64, 128, 256}; N % 128 == 0; lda, ldw % 8 == 0 and A, W 16-B aligned;
// ldc % 4 == 0 and C 8-B aligned; 128 * ldc * 2 < 2^31.  DN_UNSUPPORTED otherwise (the caller
// takes the tile GEMM).  ncol: column group per item (0 = automatic).
DN_API int dn_panel_gemm(const void* A, long lda, const void* W, long ldw, void* C, long ldc,
                         long M, int N, int K, int ncol, hipStream_t st) {
  if (M <= 0 || N <= 0) return DN_OK;
  if ((K != 64 && K != 128 && K != 256) || N % 128 || lda % 8 || ldw % 8 || ldc % 4 ||
      lda < K || ldw < K || ldc < N || ((uintptr_t)A & 15) || ((uintptr_t)W & 15) ||
      ((uintptr_t)C & 7) || (long)PN_BM * ldc * 2 >= (1L << 31))
    return DN_UNSUPPORTED;
  PnArgs a{};
  a.A = (const bf16*)A;
  a.W = (const bf16*)W;
  a.C = (bf16*)C;
  a.lda = lda;
  a.ldw = ldw;
  a.ldc = ldc;
  a.M = M;
  a.N = N;
  a.K = K;
  a.nrb = (M + PN_BM - 1) / PN_BM;
  const int cus = pn_cus();
  a.ncol = pn_ncol(a.nrb, N, cus, ncol);
  if (!a.ncol) return DN_UNSUPPORTED;
  const long items = a.nrb * (N / a.ncol);
  int G = (int)(items < cus ? items : cus);
  G = (G + 7) / 8 * 8;  // whole XCD rounds (empty ranges return)
  void (*kl)(PnArgs) = K == 256 ? panel_kernel<8> : K == 128 ? panel_kernel<4> : panel_kernel<2>;
  static bool init[3] = {false, false, false};
  const int ki = K == 256 ? 0 : K == 128 ? 1 : 2;
  if (!init[ki]) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kl),
                              hipFuncAttributeMaxDynamicSharedMemorySize, PN_SMEM);
    init[ki] = true;
  }
  hipLaunchKernelGGL(kl, dim3(G), dim3(512), PN_SMEM, st, a);
  return dn_launch_status();
}
