// Fused ICA encoder + LSTM input projection for gfx950 (reference comps/icalstm/models.py:87,107
// and the i2h Linear of every direction, models.py:13,31):
//
//   enc = relu(X We^T + be)          [N, 256]   (bf16, kept for the backward / rank-dAD)
//   xp  = enc Wp^T                   [N, N2]    (fp32, N2 = ndir * 4 * HD gate columns)
//
// One workgroup owns 64 rows end to end: phase 1 accumulates its enc tile over K = C*W with the
// four waves on 64 output columns each (4x4 16x16x32 MFMA fragments per wave), writes the
// bias+ReLU result to LDS and global; phase 2 multiplies the LDS-resident tile by the packed
// W_ih (B fragments straight from global/L2, 16 B per lane) in 64-column chunks.
//
// Why not two GEMM launches: both GEMMs are latency-bound at these sizes (each K step of a
// 64x64-tile GEMM is 8 MFMAs per wave against a ~1 us load round trip), and between them the
// enc tile makes a round trip through HBM.  Here a K step is 32 MFMAs per wave, the encoder
// weight tile streams through one LDS buffer with the next two tiles in registers, and phase 2
// never waits on a global store.  Grid = ceil(N / 64) workgroups of 256 threads.
//
// Measured on MI355X at the bench shape (N = 3136, K = 1000, N2 = 1536): 63 us, vs 38 us for the
// encoder + projection GEMM launches -- every one of the 49 workgroups streams all of We and
// W_ih (1.8 MB) through ONE CU with ~72 KB in flight, i.e. per-CU memory-level parallelism,
// not MFMA, bounds it.  Kept opt-in (DINUNET_FUSED_ENCPROJ=1) and tested; a variant worth trying
// splits phase 2 columns over several workgroups per row chunk and reads bf16 weights.
#include "common.h"

namespace {

constexpr int EP_BM = 64;         // rows per workgroup
constexpr int EP_I = 256;         // encoder width (input_size)
constexpr int EP_BK = 64;         // K step of phase 1
constexpr int EP_XS = EP_BK + 8;  // LDS row stride (elements) of the k-contiguous X / We tiles
constexpr int EP_ES = EP_I + 8;   // LDS row stride of the enc tile

// phase-1 stage: X tile [64 rows][64 k] (bf16, 2 x 16 B per thread) and We tile [256 rows][64 k]
// (fp32 master weights, 16 x 16 B per thread), raw in registers until the LDS store
struct EpStage {
  bf16x8 x[2];
  f32x4 w[16];
  bool xok[2], wok[8];
};

__device__ __forceinline__ void ep_load(EpStage& s, const bf16* __restrict__ X, long ldx,
                                        const float* __restrict__ We, int row0, int N, int KX,
                                        int k0, int tid) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int idx = tid + c * 256;
    const int r = idx >> 3, kc = (idx & 7) * 8;
    const int gr = row0 + r, gk = k0 + kc;
    s.xok[c] = gr < N && gk < KX;
    const int grc = min(gr, N - 1), gkc = min(gk, KX - 8);
    s.x[c] = *reinterpret_cast<const bf16x8*>(X + (long)grc * ldx + gkc);
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int idx = tid + c * 256;
    const int r = idx >> 3, kc = (idx & 7) * 8;  // r < 256 (encoder output row)
    const int gk = k0 + kc;
    s.wok[c] = gk < KX;
    const float* p = We + (long)r * KX + min(gk, KX - 8);
    s.w[2 * c] = *reinterpret_cast<const f32x4*>(p);
    s.w[2 * c + 1] = *reinterpret_cast<const f32x4*>(p + 4);
  }
}

__device__ __forceinline__ void ep_store(const EpStage& s, bf16* __restrict__ Xs,
                                         bf16* __restrict__ Ws, int tid) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int idx = tid + c * 256;
    const int r = idx >> 3, kc = (idx & 7) * 8;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = s.xok[c] ? s.x[c][e] : (bf16)0.f;
    *reinterpret_cast<bf16x8*>(Xs + r * EP_XS + kc) = v;
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int idx = tid + c * 256;
    const int r = idx >> 3, kc = (idx & 7) * 8;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = (bf16)(s.wok[c] ? s.w[2 * c][e] : 0.f);
      v[4 + e] = (bf16)(s.wok[c] ? s.w[2 * c + 1][e] : 0.f);
    }
    *reinterpret_cast<bf16x8*>(Ws + r * EP_XS + kc) = v;
  }
}

__global__ void __launch_bounds__(256)
enc_proj_kernel(const bf16* __restrict__ X, long ldx, int N, int KX,
                const float* __restrict__ We, const float* __restrict__ be,
                const bf16* __restrict__ Wp, int N2,
                bf16* __restrict__ enc, float* __restrict__ xp) {
  __shared__ __attribute__((aligned(16))) bf16 sm[EP_BM * EP_XS + EP_I * EP_XS + EP_BM * EP_ES];
  bf16* Xs = sm;
  bf16* Ws = sm + EP_BM * EP_XS;
  bf16* Es = Ws + EP_I * EP_XS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int row0 = blockIdx.x * EP_BM;
  const int l15 = lane & 15, lq = lane >> 4;

  // ---------------- phase 1: enc tile = relu(X We^T + be), wave w owns columns [64w, 64w+64)
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (KX + EP_BK - 1) / EP_BK;
  EpStage s0, s1;
  ep_load(s0, X, ldx, We, row0, N, KX, 0, tid);
  ep_load(s1, X, ldx, We, row0, N, KX, EP_BK, tid);
  ep_store(s0, Xs, Ws, tid);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  auto mfma_step = [&]() {
#pragma unroll
    for (int ks = 0; ks < EP_BK / 32; ++ks) {
      bf16x8 af[4], bq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(Xs + (16 * i + l15) * EP_XS + 32 * ks + 8 * lq);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bq[j] = *reinterpret_cast<const bf16x8*>(Ws + (64 * w + 16 * j + l15) * EP_XS + 32 * ks + 8 * lq);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bq[j], acc[i][j]);
    }
  };
  // unconditional (clamped) refills keep the compiler's vmcnt counting exact (see gemm.hip)
  for (int it = 0; it < nk; it += 2) {
    ep_load(s0, X, ldx, We, row0, N, KX, (it + 2) * EP_BK, tid);
    mfma_step();
    if (it + 1 >= nk) break;
    asm volatile("s_barrier" ::: "memory");
    ep_store(s1, Xs, Ws, tid);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    ep_load(s1, X, ldx, We, row0, N, KX, (it + 3) * EP_BK, tid);
    mfma_step();
    if (it + 2 >= nk) break;
    asm volatile("s_barrier" ::: "memory");
    ep_store(s0, Xs, Ws, tid);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // epilogue: bias + ReLU -> bf16 enc tile in LDS (phase 2's A operand) and in global memory
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 64 * w + 16 * j + l15;
    const float b = be[col];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + 4 * lq + r;
        const bf16 v = (bf16)fmaxf(acc[i][j][r] + b, 0.f);
        Es[row * EP_ES + col] = v;
        if (row0 + row < N) enc[(long)(row0 + row) * EP_I + col] = v;
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---------------- phase 2: xp rows = enc tile Wp^T, 64-column chunks round-robin over waves
  const int nch = N2 / 64;
  for (int ch = w; ch < nch; ch += 4) {
    f32x4 a2[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) a2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // B fragments of the whole chunk (64 columns x K 256) straight from global, issued together
    bf16x8 bq[EP_I / 32][4];
#pragma unroll
    for (int ks = 0; ks < EP_I / 32; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bq[ks][j] = *reinterpret_cast<const bf16x8*>(Wp + (long)(64 * ch + 16 * j + l15) * EP_I +
                                                     32 * ks + 8 * lq);
#pragma unroll
    for (int ks = 0; ks < EP_I / 32; ++ks) {
      bf16x8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(Es + (16 * i + l15) * EP_ES + 32 * ks + 8 * lq);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) a2[i][j] = mfma16(af[i], bq[ks][j], a2[i][j]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 16 * i + 4 * lq + r;
        if (row < N) {
          float* o = xp + (long)row * N2 + 64 * ch + l15;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[16 * j] = a2[i][j][r];
        }
      }
  }
}

}  // namespace

// enc = relu(X We^T + be) (bf16 [N][256]) and xp = enc Wp^T (fp32 [N][N2]) in one launch.
// X: bf16 [N][ldx] (KX used), KX % 8 == 0; We fp32 [256][KX]; Wp bf16 [N2][256]; N2 % 64 == 0.
DN_API int dn_enc_proj(const void* X, long ldx, int N, int KX, const float* We, const float* be,
                       const void* Wp, int N2, void* enc, float* xp, hipStream_t st) {
  if (N <= 0 || KX < 8 || KX % 8 || ldx % 8 || N2 <= 0 || N2 % 64) return DN_BAD_SHAPE;
  if ((((uintptr_t)X) | ((uintptr_t)We) | ((uintptr_t)Wp)) & 15) return DN_BAD_SHAPE;
  hipLaunchKernelGGL(enc_proj_kernel, dim3((N + EP_BM - 1) / EP_BM), dim3(256), 0, st,
                     (const bf16*)X, ldx, N, KX, We, be, (const bf16*)Wp, N2, (bf16*)enc, xp);
  return dn_launch_status();
}

DN_API int dn_enc_proj_width() { return EP_I; }
