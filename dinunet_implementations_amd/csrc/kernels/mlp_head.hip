// Fused MLP head + loss for gfx950: the ICA classifier (reference comps/icalstm/models.py:95-103
// + comps/icalstm/__init__.py:59-63) and the FreeSurfer MSANNet (comps/fs/models.py:4-31 +
// comps/fs/__init__.py:54-57) in two launches forward and two backward (instead of ~40 kernels).
//
// A head is a chain of at most HMAXL layers, each
//     [dropout on the input] -> Linear (+bias) -> [BatchNorm1d] -> [ReLU]
// ending in softmax cross-entropy (probabilities out) or log-softmax + NLL (log-probs out).
// Batch <= 64: everything is latency / per-CU-bandwidth bound (one CU streams only ~50 GB/s),
// so the launches are split by where the bytes are:
//  fwd0  (grid = layer-0 column tiles): the widest layer.  Each workgroup builds the bf16 input
//        image in LDS, its four waves split K, and wave 0 owns 16 output columns for ALL batch
//        rows, so BatchNorm column statistics are an in-register reduction (lanes l, l^16, l^32,
//        l^48 hold one column).  Output activations go to the workspace.
//  fwd1  (one workgroup): the remaining (narrow) layers from LDS, softmax/CE, argmax, loss.
//  bwd1  (one workgroup): the output-gradient chain dZ_l -> dA = dZ W -> dropout / ReLU /
//        BatchNorm backward in the epilogue (wave-owned columns again) down to dZ_0, plus the
//        bias / BatchNorm parameter gradients (column sums).
//  bwd0  (grid = every layer's 16-row dW slices + the 16-column slices of dX): dW = dZ^T A as
//        MFMA over the batch with operands from the CDNA4 LDS transpose read
//        (ds_read_b64_tr_b16), accumulated into the caller's fp32 .grad buffers; dX = dZ_0 W_0.
// GEMMs are 16x16x32 bf16 MFMA with fp32 accumulation; the fp32 master weights are read straight
// from global memory and rounded while loading.  Kernel boundaries are the only inter-workgroup
// synchronisation.  Dropout masks come from a counter-based hash of (seed, layer, row, col); the
// seed is a device word bumped by fwd1, so a captured HIP graph draws fresh masks on every replay,
// and the backward regenerates the mask from the seed saved in the workspace.
#include "head_common.h"

namespace {

constexpr int HMAXL = 6;
constexpr int HW_NT = 256;  // fwd0 / bwd0 workgroups (4 waves)
constexpr int HS_NT = 512;  // fwd1 / bwd1 single workgroup (8 waves, 256-VGPR budget)


struct HLayer {
  const float* W;  // [out][in]
  const float* b;  // [out] or null
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  long long* nbt;  // num_batches_tracked
  float* gW;
  float* gb;
  float* ggamma;
  float* gbeta;
  int in, out;
  int bn;    // 0 none, 1 batch statistics always, 2 batch stats + running update (train) / running (eval)
  int relu;
  float drop;  // dropout probability applied to this layer's INPUT (training only)
  float eps, momentum;
  int S_a;   // row stride (elements) of the input activation image   = rup32(in) + 8
  int S_z;   // row stride of the output-gradient image                = rup32(out) + 8
  int Np;    // rup32(out)
  long a_off, xhat_off, rstd_off, dz_off;  // byte offsets into the workspace
  long st_off;  // stash of the bias / BatchNorm grads [gb | ggamma | gbeta] (fused fwd+bwd1)
};

struct HArgs {
  HLayer L[HMAXL];
  int nl, B;
  int buf_a1;        // LDS elements of the largest activation image of layers >= 1
  int buf_z;         // LDS elements of the largest output-gradient image
  int buf_aall;      // LDS elements of the largest activation image of any layer
  long dzl_off;      // fp32 [Mp][16] d loss / d logits (unscaled)
  long logit_off;    // fp32 [Mp][16] logits of a one-layer head (fwd0 -> fwd1)
  int dw_jobs[HMAXL + 1];  // bwd0: prefix sums of 16-row dW slices per layer
  int train, log_out;
};

// Optional phase timestamps (s_memrealtime, 100 MHz) written by thread 0 when a stamp buffer is
// installed with dn_head_set_stamps (diagnostics: tools/bench_head.py --stamps).
#define HSTAMP(i) do { if (stamps && threadIdx.x == 0) stamps[(i)] = __builtin_amdgcn_s_memrealtime(); } while (0)



// B fragment from weight ROWS: lane -> row n, k .. k+7 (contiguous).  Branchless (clamped
// address + select) so a batch of these issues all its loads before the first use.
template <bool VEC>
__device__ __forceinline__ bf16x8 wfrag_rows(const float* __restrict__ W, int N, int K, int n, int k) {
  bf16x8 f;
  if constexpr (VEC) {  // K % 8 == 0: the 8 elements are all in or all out
    const bool ok = n < N && k < K;
    const float* p = W + (ok ? (long)n * K + k : 0);
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(p);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f[e] = (bf16)(ok ? v0[e] : 0.f);
      f[4 + e] = (bf16)(ok ? v1[e] : 0.f);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool ok = n < N && k + e < K;
      const float v = W[ok ? (long)n * K + k + e : 0];
      f[e] = (bf16)(ok ? v : 0.f);
    }
  }
  return f;
}

// B fragment from weight COLUMNS: lane -> column kk, rows n .. n+7 (stride K)
__device__ __forceinline__ bf16x8 wfrag_cols(const float* __restrict__ W, int N, int K, int n, int kk) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool ok = n + j < N && kk < K;
    const float v = W[ok ? (long)(n + j) * K + kk : 0];
    f[j] = (bf16)(ok ? v : 0.f);
  }
  return f;
}

// Raw fp32 weight-row fragment (lane -> row n, k .. k+7) held as two f32x4 so the loads can be
// issued long before the MFMA that consumes them.  Out-of-range lanes load a clamped (valid)
// address and are zeroed at conversion: zeroing the registers right after the load would make
// the compiler wait for the load first (write-after-write on a pending VGPR).
template <bool VEC>
__device__ __forceinline__ void wraw_rows(const float* __restrict__ W, int N, int K, int n, int k,
                                          f32x4 (&r)[2]) {
  if constexpr (VEC) {
    const int idx = (n < N && k < K) ? n * K + k : 0;  // weights < 2^31 elements
    r[0] = *reinterpret_cast<const f32x4*>(W + idx);
    r[1] = *reinterpret_cast<const f32x4*>(W + idx + 4);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = (n < N && k + e < K) ? n * K + k + e : 0;
      r[e >> 2][e & 3] = W[idx];
    }
  }
}

// bf16 operand from a raw fragment; elements with k + e >= K (or a row n >= N) become 0
__device__ __forceinline__ bf16x8 cvt_raw(const f32x4 (&r)[2], int N, int K, int n, int k) {
  bf16x8 f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bool ok = n < N && k + e < K;
    f[e] = (bf16)(ok ? r[e >> 2][e & 3] : 0.f);
  }
  return f;
}

// Per-column epilogue parameters of one layer, loaded early (their latency hides under the GEMM).
struct ColP {
  float bias, gamma, beta, rmean, rvar;
};

// Raw loads (clamped index, no use): the validity select happens in the epilogue, so nothing
// waits on these loads (or on the loads issued before them) until the GEMM is done.
__device__ __forceinline__ ColP load_colp(const HLayer& L, int n, bool train) {
  ColP c{0.f, 1.f, 0.f, 0.f, 1.f};
  const int i = n < L.out ? n : 0;
  if (L.b) c.bias = L.b[i];
  if (L.bn) {
    c.gamma = L.gamma[i];
    c.beta = L.beta[i];
    if (L.bn == 2) {
      c.rmean = L.rmean[i];
      c.rvar = L.rvar[i];
    }
  }
  return c;
}



// bias -> BatchNorm -> ReLU -> (next layer's dropout) epilogue of one 16-column tile of layer l,
// held as MFMA accumulators for every batch row by one wave.  Activations go to the LDS image
// `nxt` (if given) and to the workspace image; logits of the last layer to `logit`.
template <int MT>
__device__ __forceinline__ void fwd_epilogue(const HArgs& a, int l, const f32x4 (&acc)[MT], int n,
                                             int lane, uint64_t seed, char* __restrict__ ws,
                                             bf16* nxt, float* logit, const ColP& cp) {
  const HLayer& L = a.L[l];
  const int N = L.out, B = a.B;
  const bool train = a.train != 0;
  const bool last = l == a.nl - 1;
  const bool cv = n < N;
  const float bias = cv ? cp.bias : 0.f;
  float z[MT][4];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) z[mt][r] = acc[mt][r] + bias;
  if (L.bn) {
    float mean, rstd;
    if (train || L.bn == 1) {
      float s = 0.f;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += (16 * mt + 4 * (lane >> 4) + r < B) ? z[mt][r] : 0.f;
      mean = colsum4(s) / (float)B;
      float v = 0.f;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = z[mt][r] - mean;
          v += (16 * mt + 4 * (lane >> 4) + r < B) ? d * d : 0.f;
        }
      v = colsum4(v) / (float)B;
      rstd = rsqrtf(v + L.eps);
      if (train && L.bn == 2 && lane < 16 && cv) {
        const float mo = L.momentum;
        L.rmean[n] = (1.f - mo) * cp.rmean + mo * mean;
        L.rvar[n] = (1.f - mo) * cp.rvar + mo * v * ((float)B / (float)(B > 1 ? B - 1 : 1));
      }
    } else {
      mean = cv ? cp.rmean : 0.f;
      rstd = cv ? rsqrtf(cp.rvar + L.eps) : 0.f;
    }
    const float ga = cv ? cp.gamma : 0.f, be = cv ? cp.beta : 0.f;
    float* xhat_ws = reinterpret_cast<float*>(ws + L.xhat_off);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * mt + 4 * (lane >> 4) + r;
        const float xh = (z[mt][r] - mean) * rstd;
        if (train) xhat_ws[row * L.Np + n] = (row < B && cv) ? xh : 0.f;
        z[mt][r] = ga * xh + be;
      }
    if (train && lane < 16) reinterpret_cast<float*>(ws + L.rstd_off)[n] = cv ? rstd : 0.f;
  }
  const HLayer& Ln = a.L[last ? l : l + 1];
  const int Sn = Ln.S_a;
  const float pn = (last || !train) ? 0.f : Ln.drop;
  const float invn = pn > 0.f ? 1.f / (1.f - pn) : 1.f;
  bf16* wnext = reinterpret_cast<bf16*>(ws + Ln.a_off);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * mt + 4 * (lane >> 4) + r;
      float v = z[mt][r];
      if (L.relu) v = fmaxf(v, 0.f);
      if (last) {
        logit[row * 16 + (lane & 15)] = v;
      } else {
        v = (row < B && cv) ? v : 0.f;
        if (pn > 0.f && v != 0.f) v = hkeep(seed, l + 1, row, n, N, pn) ? v * invn : 0.f;
        const bf16 bv = (bf16)v;
        if (nxt) nxt[row * Sn + n] = bv;
        wnext[row * Sn + n] = bv;
      }
    }
}

// Copy a bf16 workspace image (rows x S elements, S % 8 == 0) into LDS, loads batched.
template <int NT>
__device__ __forceinline__ void ws_to_lds(bf16* __restrict__ dst_, const char* __restrict__ src_,
                                          int elems, int tid) {
  const bf16x8* src = reinterpret_cast<const bf16x8*>(src_);
  bf16x8* dst = reinterpret_cast<bf16x8*>(dst_);
  const int nv = elems / 8;
  for (int base = tid; base < nv; base += 4 * NT) {
    bf16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = src[base + u * NT < nv ? base + u * NT : 0];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (base + u * NT < nv) dst[base + u * NT] = v[u];
  }
}

// ---------------------------------------------------------------------------------------------
// fwd0: layer 0, one 16-column tile per workgroup; the four waves split K.
template <int MT, bool VECW>
__global__ void __launch_bounds__(HW_NT)
head_fwd0_kernel(HArgs a, const float* __restrict__ x, long ldx,
                 const unsigned long long* __restrict__ rng, char* __restrict__ ws,
                 unsigned long long* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int Mp = 16 * MT, NT = HW_NT, NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int B = a.B;
  const bool train = a.train != 0;
  const HLayer& L0 = a.L[0];
  const int K = L0.in, N = L0.out, Kp = rup32(K), S = L0.S_a;
  bf16* img = reinterpret_cast<bf16*>(smem);
  float* red = reinterpret_cast<float*>(smem + ((2 * Mp * S + 15) & ~15));  // [NW][MT*4][64]
  const uint64_t seed = rng ? *rng : 0ull;
  if (blockIdx.x == 0) HSTAMP(0);

  // weights of this wave's first four k-steps and the epilogue parameters: issued before the
  // input image so their latency overlaps it
  const int n = 16 * blockIdx.x + (lane & 15);
  const int nks = Kp / 32;
  f32x4 wr[4][2];
  auto load_w = [&](int kb) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ks = kb + u * NW;
      const int k0 = 32 * (ks < nks ? ks : 0) + 8 * (lane >> 4);
      wraw_rows<VECW>(L0.W, N, K, n, k0, wr[u]);
    }
  };
  const ColP cp = load_colp(L0, n, train);
  load_w(wid);

  {  // input image (layer-0 dropout applied); workgroup 0 saves it for the backward
    const float inv = L0.drop > 0.f ? 1.f / (1.f - L0.drop) : 1.f;
    const bool save = train && blockIdx.x == 0;
    bf16* wimg = reinterpret_cast<bf16*>(ws + L0.a_off);
    constexpr int R = 16;         // chunk loads per thread in flight
    const int nch = Mp * Kp / 4;  // 4-element chunks (Kp % 32 == 0: chunks never straddle rows)
    const bool vec = (K % 4) == 0 && (ldx % 4) == 0 && (((uintptr_t)x) & 15) == 0;
    // chunk c -> (row m, element k) advanced incrementally (c grows by NT per unrolled slot): a
    // runtime integer division per chunk made this loop VALU-issue bound (one wave per SIMD;
    // 6.6 us at B=32, linear in B)
    const int KC = Kp / 4, dm = NT / KC, dk = NT - (NT / KC) * KC;
    int cm = tid / KC, ck = tid - (tid / KC) * KC;  // coordinates of chunk `base`
    for (int base = tid; base < nch; base += R * NT) {
      f32x4 v[R];
      int ms[R], ks[R];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        ms[u] = cm;
        ks[u] = 4 * ck;
        ck += dk;
        cm += dm;
        if (ck >= KC) { ck -= KC; ++cm; }
      }
      if (vec) {  // (uniform) all loads of the round first
#pragma unroll
        for (int u = 0; u < R; ++u) {
          const int m = ms[u], k = ks[u];
          const int idx = (m < B && k < K) ? m * (int)ldx + k : 0;
          v[u] = *reinterpret_cast<const f32x4*>(x + idx);
        }
      } else {
#pragma unroll
        for (int u = 0; u < R; ++u) {
          const int m = ms[u], k = ks[u];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[u][e] = x[(m < B && k + e < K) ? m * (int)ldx + k + e : 0];
        }
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int m = ms[u], k = ks[u];
        if (m >= Mp) continue;  // chunk past the image (not break: keeps v[] in VGPRs)
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = (m < B && k + e < K) ? v[u][e] : 0.f;
          if (train && L0.drop > 0.f && t != 0.f) t = hkeep(seed, 0, m, k + e, K, L0.drop) ? t * inv : 0.f;
          o[e] = (bf16)t;
        }
        *reinterpret_cast<bf16x4*>(img + m * S + k) = o;
        if (save) *reinterpret_cast<bf16x4*>(wimg + m * S + k) = o;
      }
    }
  }
  __syncthreads();
  if (blockIdx.x == 0) HSTAMP(1);

  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kb = wid; kb < nks; kb += 4 * NW) {  // this wave's k-steps, four loads in flight
    if (kb != wid) load_w(kb);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ks = kb + u * NW;
      if (ks >= nks) break;
      const bf16x8 bq = cvt_raw(wr[u], N, K, n, 32 * ks + 8 * (lane >> 4));
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(img + (16 * mt + (lane & 15)) * S + 32 * ks + 8 * (lane >> 4));
        acc[mt] = mfma16(af, bq, acc[mt]);
      }
    }
  }
  if (wid > 0) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((wid - 1) * MT * 4 + mt * 4 + r) * 64 + lane] = acc[mt][r];
  }
  __syncthreads();
  if (wid == 0) {
#pragma unroll
    for (int w = 0; w < NW - 1; ++w)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[mt][r] += red[(w * MT * 4 + mt * 4 + r) * 64 + lane];
    fwd_epilogue<MT>(a, 0, acc, n, lane, seed, ws, nullptr,
                     reinterpret_cast<float*>(ws + a.logit_off), cp);
    if (blockIdx.x == 0) HSTAMP(2);
  }
}

// ---------------------------------------------------------------------------------------------
// fwd1: layers 1.. and the loss in one workgroup.
// dzl_lds (fused fwd1+bwd1 only): d loss / d logits also parked in LDS for the backward chain.
// Returns the dropout seed of this forward.
template <int MT, bool VECW>
__device__ __forceinline__ uint64_t fwd1_body(const HArgs& a, const long long* __restrict__ y,
                                              float* __restrict__ out, float* __restrict__ loss,
                                              long long* __restrict__ pred,
                                              unsigned long long* __restrict__ rng,
                                              char* __restrict__ ws,
                                              unsigned long long* __restrict__ stamps, char* smem,
                                              float* dzl_lds = nullptr) {
  constexpr int Mp = 16 * MT, NT = HS_NT, NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int B = a.B;
  const bool train = a.train != 0;
  bf16* cur = reinterpret_cast<bf16*>(smem);
  bf16* nxt = cur + a.buf_a1;
  float* logit = reinterpret_cast<float*>(nxt + a.buf_a1);  // [Mp][16]
  const uint64_t seed = rng ? *rng : 0ull;
  // labels requested now and parked in LDS with the activation image: the loss phase at the end
  // no longer waits on a global round trip
  int* ylds = reinterpret_cast<int*>(logit + Mp * 16);  // [64] (no static LDS: see lds_fwd1)
  // (MT 4 has no register to spare for it: the label load stays in the loss phase)
  const long long ypre = (MT <= 2 && wid == 0 && lane < B) ? y[lane] : 0ll;
  HSTAMP(3);
  // this wave's first layer-1 tile: weights (first 8 k-steps) and epilogue parameters are
  // requested before the activation image is copied in, so their latency overlaps it
  f32x4 wr[8][2];
  ColP cp1{0.f, 0.f, 0.f, 0.f, 1.f};
  auto load_w = [&](const HLayer& L, int n, int kb) {
    const int Kp = rup32(L.in);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k0 = kb + 32 * u;
      const int kk = (k0 < Kp ? k0 : 0) + 8 * (lane >> 4);
      wraw_rows<VECW>(L.W, L.out, L.in, n, kk, wr[u]);
    }
  };
  const int tiles1 = a.nl >= 2 ? (a.nl == 2 ? 1 : a.L[1].Np / 16) : 0;
  if (wid < tiles1) {
    load_w(a.L[1], 16 * wid + (lane & 15), 0);
    cp1 = load_colp(a.L[1], 16 * wid + (lane & 15), train);
  }
  if (a.nl >= 2) {
    ws_to_lds<NT>(cur, ws + a.L[1].a_off, Mp * a.L[1].S_a, tid);
  } else {
    const float* src = reinterpret_cast<const float*>(ws + a.logit_off);
    for (int i = tid; i < Mp * 16; i += NT) logit[i] = src[i];
  }
  if (MT <= 2 && wid == 0) ylds[lane] = (int)(ypre < 0 ? -1 : (ypre > 0x7fffffffll ? 0x7fffffff : ypre));
  __syncthreads();
  HSTAMP(4);
  for (int l = 1; l < a.nl; ++l) {
    const HLayer& L = a.L[l];
    const int Kp = rup32(L.in), S = L.S_a;
    const bool last = l == a.nl - 1;
    const int ntiles = last ? 1 : L.Np / 16;  // cover rup32(out): the next image's pad is zeroed
    for (int t = wid; t < ntiles; t += NW) {
      const int n = 16 * t + (lane & 15);
      const bool first = l == 1 && t == wid;  // prefetched above
      const ColP cp = first ? cp1 : load_colp(L, n, train);
      f32x4 acc[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int kb = 0; kb < Kp; kb += 8 * 32) {  // 8 k-steps of weight loads in flight
        if (!(first && kb == 0)) load_w(L, n, kb);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k0 = kb + 32 * u;
          if (k0 >= Kp) break;
          const bf16x8 bq = cvt_raw(wr[u], L.out, L.in, n, k0 + 8 * (lane >> 4));
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(cur + (16 * mt + (lane & 15)) * S + k0 + 8 * (lane >> 4));
            acc[mt] = mfma16(af, bq, acc[mt]);
          }
        }
      }
      fwd_epilogue<MT>(a, l, acc, n, lane, seed, ws, nxt, logit, cp);
    }
    __syncthreads();
    HSTAMP(4 + l);
    bf16* t = cur;
    cur = nxt;
    nxt = t;
  }

  // softmax / log-softmax + CE / NLL, argmax; wave 0, lane = batch row
  if (wid == 0) {
    const int C = a.L[a.nl - 1].out;
    const int m = lane;
    float ls = 0.f;
    if (m < B) {
      float mx = -INFINITY;
      int am = 0;
      for (int c = 0; c < C; ++c) {
        const float v = logit[m * 16 + c];
        if (v > mx) { mx = v; am = c; }
      }
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(logit[m * 16 + c] - mx);
      const float lse = mx + logf(se);
      long long yc = MT <= 2 ? (long long)ylds[m] : y[m];
      yc = yc < 0 ? 0 : (yc >= C ? C - 1 : yc);
      float* dzl = reinterpret_cast<float*>(ws + a.dzl_off);
      for (int c = 0; c < C; ++c) {
        const float lp = logit[m * 16 + c] - lse;
        const float p = expf(lp);
        out[(long)m * C + c] = a.log_out ? lp : p;
        const float dl = (p - (c == yc ? 1.f : 0.f)) / (float)B;
        if (train) dzl[m * 16 + c] = dl;
        if (dzl_lds) dzl_lds[m * 16 + c] = dl;
      }
      ls = lse - logit[m * 16 + yc];
      pred[m] = am;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) ls += __shfl_xor(ls, off);
    if (lane == 0) {
      *loss = ls / (float)B;
      if (train) {
        *reinterpret_cast<unsigned long long*>(ws) = seed;
        if (rng) *rng = seed + 1ull;
        // no-return atomic: a read-modify-write here was one more global round trip
        for (int l = 0; l < a.nl; ++l)
          if (a.L[l].bn == 2 && a.L[l].nbt)
            __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(a.L[l].nbt), 1ull,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    HSTAMP(12);
  }
  return seed;
}

template <int MT, bool VECW>
__global__ void __launch_bounds__(HS_NT)
head_fwd1_kernel(HArgs a, const long long* __restrict__ y, float* __restrict__ out,
                 float* __restrict__ loss, long long* __restrict__ pred,
                 unsigned long long* __restrict__ rng, char* __restrict__ ws,
                 unsigned long long* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  fwd1_body<MT, VECW>(a, y, out, loss, pred, rng, ws, stamps, smem);
}

// ---------------------------------------------------------------------------------------------
// bwd1: output-gradient chain down to dZ_0 (+ bias / BatchNorm parameter gradients).
// stash = 1 (fused forward): the bias / BatchNorm gradients go to the workspace stash (not
// accumulated: bwd0 adds them into .grad once the backward is known to use this d loss)
// pre (fused fwd1+bwd1): d out / d loss, the forward's dropout seed and d loss / d logits in
// LDS come from the forward half instead of global round trips
struct Bwd1Pre {
  float gs;
  uint64_t seed;
  const float* dzl_lds;
};

template <int MT>
__device__ __forceinline__ void bwd1_body(const HArgs& a, char* __restrict__ ws,
                                          const float* __restrict__ dloss,
                                          unsigned long long* __restrict__ stamps, char* smem,
                                          int stash, const Bwd1Pre* pre = nullptr) {
  constexpr int Mp = 16 * MT, NT = HS_NT, NW = NT / 64;
  constexpr int CB = 2;  // weight-column k-steps per load batch (x2 register sets: see pipe)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int B = a.B;
  bf16* dz = reinterpret_cast<bf16*>(smem);
  bf16* dzn = dz + a.buf_z;
  bf16* abuf = dzn + a.buf_z;
  const float gs = pre ? pre->gs : *dloss;
  const uint64_t seed = pre ? pre->seed : *reinterpret_cast<const unsigned long long*>(ws);
  const float* dzl = pre ? pre->dzl_lds : reinterpret_cast<const float*>(ws + a.dzl_off);
  HSTAMP(16);
  {  // gradient of the logits
    const HLayer& L = a.L[a.nl - 1];
    const int C = L.out, Cp = rup32(C), S = L.S_z;
    bf16* wdz = reinterpret_cast<bf16*>(ws + L.dz_off);
    float gbold = 0.f, colv[Mp];
    float* const gbw = stash ? reinterpret_cast<float*>(ws + L.st_off) : L.gb;
    if (L.gb && tid < C) {  // bias-gradient loads first (old value + the column of dL/dz)
      gbold = stash ? 0.f : L.gb[tid];
#pragma unroll
      for (int m = 0; m < Mp; ++m) colv[m] = dzl[m * 16 + tid];
    }
    for (int idx = tid; idx < Mp * Cp; idx += NT) {
      const int m = idx / Cp, c = idx - m * Cp;
      const float v = (m < B && c < C) ? gs * dzl[m * 16 + c] : 0.f;
      dz[m * S + c] = (bf16)v;
      wdz[m * S + c] = (bf16)v;
    }
    if (L.gb && tid < C) {
      float s = 0.f;
#pragma unroll
      for (int m = 0; m < Mp; ++m) s += m < B ? colv[m] : 0.f;
      gbw[tid] = gbold + gs * s;
    }
  }
  for (int l = a.nl - 1; l >= 1; --l) {
    const HLayer& L = a.L[l];
    const HLayer& P = a.L[l - 1];
    const int K = L.in, N = L.out, Kp = rup32(K), Np = L.Np, Sa = L.S_a, Sz = L.S_z;
    const int ntl = Kp / 16;
    const float inv = L.drop > 0.f ? 1.f / (1.f - L.drop) : 1.f;
    const float* xhat_ws = reinterpret_cast<const float*>(ws + P.xhat_off);
    const float* rstd_ws = reinterpret_cast<const float*>(ws + P.rstd_off);
    bf16* wdz = reinterpret_cast<bf16*>(ws + P.dz_off);
    float* const st = reinterpret_cast<float*>(ws + P.st_off);
    float* const gbw = stash ? st : P.gb;
    float* const ggw = stash ? st + P.out : P.ggamma;
    float* const gbew = stash ? st + 2 * P.out : P.gbeta;

    // Everything a tile needs from global memory, requested in one go (clamped addresses, no
    // use until the MFMAs / epilogue): weight columns of the first CB k-steps, the saved
    // BatchNorm xhat / rstd, gamma and the old values of the parameter gradients it updates.
    // One column batch covers the whole K loop (Np <= CB * 32, the ICA head): the NEXT tile's
    // operands are requested into a second register set before this tile's MFMAs, so a wave's
    // later tiles do not start with a global round trip.  Otherwise the K loop reloads wc.
    const bool pipe = Np <= CB * 32;
    float wc[CB][8], xhp[MT][4];
    float rsp = 0.f, gap = 0.f, ggo = 0.f, gbeo = 0.f, gbo = 0.f;
    float wn[CB][8], xhn[MT][4];
    float rsn = 0.f, gan = 0.f, ggn = 0.f, gben = 0.f, gbn = 0.f;
#define HB1_LOAD_W(w, nb, kk)                                                   \
  _Pragma("unroll") for (int u = 0; u < CB; ++u)                                \
  _Pragma("unroll") for (int j = 0; j < 8; ++j) {                               \
    const int n_ = (nb) + 32 * u + 8 * (lane >> 4) + j;                         \
    w[u][j] = L.W[(n_ < N && (kk) < K) ? n_ * K + (kk) : 0];                    \
  }
#define HB1_PREFETCH(t, w, xh, rs, ga, gg, gbe, gbv)                            \
  do {                                                                          \
    const int kk_ = 16 * (t) + (lane & 15);                                     \
    const int kc_ = kk_ < K ? kk_ : 0;                                          \
    HB1_LOAD_W(w, 0, kk_)                                                       \
    if (P.bn) {                                                                 \
      _Pragma("unroll") for (int mt = 0; mt < MT; ++mt)                         \
      _Pragma("unroll") for (int r = 0; r < 4; ++r)                             \
        xh[mt][r] = xhat_ws[(16 * mt + 4 * (lane >> 4) + r) * P.Np + kc_];      \
      rs = rstd_ws[kc_];                                                        \
      ga = P.gamma[kc_];                                                        \
      gg = stash ? 0.f : P.ggamma[kc_];                                         \
      gbe = stash ? 0.f : P.gbeta[kc_];                                         \
    }                                                                           \
    if (P.gb) gbv = stash ? 0.f : P.gb[kc_];                                    \
  } while (0)
    auto load_wc = [&](int nb, int kk) { HB1_LOAD_W(wc, nb, kk) };
    auto prefetch = [&](int t) { HB1_PREFETCH(t, wc, xhp, rsp, gap, ggo, gbeo, gbo); };
    if (wid < ntl) prefetch(wid);
    ws_to_lds<NT>(abuf, ws + L.a_off, Mp * Sa, tid);  // relu mask of the layer below
    __syncthreads();
    HSTAMP(26 + (a.nl - 1 - l));  // operands in (diagnostic stamps)
    for (int t = wid; t < ntl; t += NW) {
      if (t != wid) {
        if (pipe) {
#pragma unroll
          for (int u = 0; u < CB; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) wc[u][j] = wn[u][j];
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) xhp[mt][r] = xhn[mt][r];
          rsp = rsn; gap = gan; ggo = ggn; gbeo = gben; gbo = gbn;
        } else {
          prefetch(t);
        }
      }
      if (pipe && t + NW < ntl) HB1_PREFETCH(t + NW, wn, xhn, rsn, gan, ggn, gben, gbn);
      const int kk = 16 * t + (lane & 15);
      const bool kv = kk < K;
      f32x4 acc[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int nb = 0; nb < Np; nb += CB * 32) {  // CB k-steps of column loads in flight
        if (nb > 0) load_wc(nb, kk);
#pragma unroll
        for (int u = 0; u < CB; ++u) {
          const int ns = nb + 32 * u;
          if (ns >= Np) break;
          bf16x8 bq;
#pragma unroll
          for (int j = 0; j < 8; ++j) bq[j] = (bf16)((ns + 8 * (lane >> 4) + j < N && kv) ? wc[u][j] : 0.f);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(dz + (16 * mt + (lane & 15)) * Sz + ns + 8 * (lane >> 4));
            acc[mt] = mfma16(af, bq, acc[mt]);
          }
        }
      }
      float d[MT][4];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * mt + 4 * (lane >> 4) + r;
          float v = (row < B && kv) ? acc[mt][r] : 0.f;
          if (L.drop > 0.f && v != 0.f) v = hkeep(seed, l, row, kk, K, L.drop) ? v * inv : 0.f;
          if (P.relu && !((float)abuf[row * Sa + kk] > 0.f)) v = 0.f;
          d[mt][r] = v;
        }
      if (P.bn) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s1 += d[mt][r];
            s2 += d[mt][r] * xhp[mt][r];
          }
        s1 = colsum4(s1);
        s2 = colsum4(s2);
        if (lane < 16 && kv) {
          ggw[kk] = ggo + s2;
          gbew[kk] = gbeo + s1;
        }
        const float ga = kv ? gap : 0.f;
        const float m1 = s1 / (float)B, m2 = s2 / (float)B;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + 4 * (lane >> 4) + r;
            d[mt][r] = (row < B && kv) ? ga * rsp * (d[mt][r] - m1 - xhp[mt][r] * m2) : 0.f;
          }
      }
      if (P.gb) {
        float sb = 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) sb += d[mt][r];
        sb = colsum4(sb);
        if (lane < 16 && kv) gbw[kk] = gbo + sb;
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * mt + 4 * (lane >> 4) + r;
          const bf16 bv = (bf16)d[mt][r];
          dzn[row * P.S_z + kk] = bv;
          wdz[row * P.S_z + kk] = bv;
        }
    }
    __syncthreads();
    HSTAMP(17 + (a.nl - 1 - l));
    bf16* t = dz;
    dz = dzn;
    dzn = t;
  }
}

template <int MT>
__global__ void __launch_bounds__(HS_NT)
head_bwd1_kernel(HArgs a, char* __restrict__ ws, const float* __restrict__ dloss,
                 unsigned long long* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bwd1_body<MT>(a, ws, dloss, stamps, smem, 0);
}

// Training step whose d loss is known at forward time (a persistent 1 the step's backward
// passes): fwd1 and bwd1 in ONE single-workgroup launch, so the output-gradient chain starts
// without a kernel boundary and on an L2-hot workspace.
template <int MT, bool VECW>
__global__ void __launch_bounds__(HS_NT)
head_fwd1_bwd1_kernel(HArgs a, const long long* __restrict__ y, float* __restrict__ out,
                      float* __restrict__ loss, long long* __restrict__ pred,
                      unsigned long long* __restrict__ rng, char* __restrict__ ws,
                      const float* __restrict__ dloss, unsigned long long* __restrict__ stamps,
                      int dzl_lds_off) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const float gs = *dloss;  // requested now: used after the whole forward half
  float* dzl_lds = reinterpret_cast<float*>(smem + dzl_lds_off);  // clear of both halves' LDS
  const uint64_t seed = fwd1_body<MT, VECW>(a, y, out, loss, pred, rng, ws, stamps, smem, dzl_lds);
  __threadfence_block();
  __syncthreads();
  const Bwd1Pre pre{gs, seed, dzl_lds};
  bwd1_body<MT>(a, ws, dloss, stamps, smem, 1, &pre);
}

// ---------------------------------------------------------------------------------------------
// bwd0: blocks [0, dw_jobs[nl]) -> 16-row slices of every layer's dW (read-modify-write into the
// fp32 gradient); blocks after that -> 16-column slices of dX = dZ_0 W_0 (+ layer-0 dropout).
template <int MT>
__global__ void __launch_bounds__(HW_NT)
head_bwd0_kernel(HArgs a, const char* __restrict__ ws, float* __restrict__ dx, long lddx,
                 int apply_stash, unsigned long long* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int Mp = 16 * MT, NT = HW_NT, NW = NT / 64;
  constexpr int G = 6;  // dW tiles per wave batch (global read-modify-write in flight together)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int B = a.B;
  const int job = blockIdx.x;
  if (job == 0) HSTAMP(24);
  if (apply_stash && job == gridDim.x - 1) {  // bias / BatchNorm grads of the fused forward
    for (int l = 0; l < a.nl; ++l) {
      const HLayer& L = a.L[l];
      const float* st = reinterpret_cast<const float*>(ws + L.st_off);
      for (int i = tid; i < L.out; i += NT) {
        if (L.gb) L.gb[i] += st[i];
        if (L.bn) {
          L.ggamma[i] += st[L.out + i];
          L.gbeta[i] += st[2 * L.out + i];
        }
      }
    }
  }
  if (job < a.dw_jobs[a.nl]) {
    int l = 0;
    while (job >= a.dw_jobs[l + 1]) ++l;
    const HLayer& L = a.L[l];
    const int K = L.in, N = L.out, Sa = L.S_a, Sz = L.S_z;
    const int n0 = 16 * (job - a.dw_jobs[l]);
    constexpr int SD = 24;  // LDS row stride of the 16-column dZ slice
    bf16* abuf = reinterpret_cast<bf16*>(smem);
    bf16* dzs = abuf + a.buf_aall;
    {
      const bf16* src = reinterpret_cast<const bf16*>(ws + L.dz_off);
      for (int i = tid; i < Mp * 2; i += NT) {  // two 16-B vectors per row
        const int m = i >> 1, h = i & 1;
        *reinterpret_cast<bf16x8*>(dzs + m * SD + 8 * h) =
            *reinterpret_cast<const bf16x8*>(src + m * Sz + n0 + 8 * h);
      }
    }
    ws_to_lds<NT>(abuf, ws + L.a_off, Mp * Sa, tid);
    __syncthreads();
    const int tk = (K + 15) / 16;
    for (int t0 = wid * G; t0 < tk; t0 += NW * G) {
      float old[G][4];
#pragma unroll
      for (int gi = 0; gi < G; ++gi) {  // gradient reads first
        const int k = 16 * (t0 + gi) + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + 4 * (lane >> 4) + r;
          const bool ok = t0 + gi < tk && n < N && k < K;
          const float v = L.gW[ok ? (long)n * K + k : 0];
          old[gi][r] = ok ? v : 0.f;
        }
      }
      f32x4 acc[G];
#pragma unroll
      for (int gi = 0; gi < G; ++gi) {
        acc[gi] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (t0 + gi < tk) {
#pragma unroll
          for (int ms = 0; ms < Mp; ms += 32)
            acc[gi] = mfma16(tr_frag(dzs, SD, 0, ms, lane), tr_frag(abuf, Sa, 16 * (t0 + gi), ms, lane), acc[gi]);
        }
      }
#pragma unroll
      for (int gi = 0; gi < G; ++gi) {
        const int k = 16 * (t0 + gi) + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + 4 * (lane >> 4) + r;
          if (t0 + gi < tk && n < N && k < K) L.gW[(long)n * K + k] = old[gi][r] + acc[gi][r];
        }
      }
    }
    return;
  }
  // dX slice: dx[:, kk] = sum_n dZ_0[:, n] W_0[n, kk]; the four waves split n
  const HLayer& L = a.L[0];
  const int K = L.in, N = L.out, Np = L.Np, Sz = L.S_z;
  const int kk = 16 * (job - a.dw_jobs[a.nl]) + (lane & 15);
  const bf16* dz0 = reinterpret_cast<const bf16*>(ws + L.dz_off);
  float* red = reinterpret_cast<float*>(smem);
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nks = Np / 32;
  for (int kb = wid; kb < nks; kb += 4 * NW) {
    bf16x8 bq[4];
    bf16x8 aq[4][MT];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ks = kb + u * NW < nks ? kb + u * NW : 0;
      bq[u] = wfrag_cols(L.W, N, K, 32 * ks + 8 * (lane >> 4), kk);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        aq[u][mt] = *reinterpret_cast<const bf16x8*>(dz0 + (16 * mt + (lane & 15)) * Sz + 32 * ks + 8 * (lane >> 4));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (kb + u * NW >= nks) break;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma16(aq[u][mt], bq[u], acc[mt]);
    }
  }
  if (wid > 0) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((wid - 1) * MT * 4 + mt * 4 + r) * 64 + lane] = acc[mt][r];
  }
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int w = 0; w < NW - 1; ++w)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mt][r] += red[(w * MT * 4 + mt * 4 + r) * 64 + lane];
  const uint64_t seed = *reinterpret_cast<const unsigned long long*>(ws);
  const float inv = L.drop > 0.f ? 1.f / (1.f - L.drop) : 1.f;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * mt + 4 * (lane >> 4) + r;
      float v = acc[mt][r];
      if (L.drop > 0.f && v != 0.f) v = hkeep(seed, 0, row, kk, K, L.drop) ? v * inv : 0.f;
      if (row < B && kk < K) dx[(long)row * lddx + kk] = v;
    }
}

struct Plan {
  HArgs a;
  long ws_bytes;
  int Mp;
  int grid_fwd0, grid_bwd0_dw, grid_bwd0_dx;
  long lds_fwd0, lds_fwd1, lds_bwd1, lds_bwd0;
  long lds_fused_base, lds_fused;  // fused fwd1+bwd1: both halves, then d loss / d logits
};

static long al256(long v) { return (v + 255) & ~255L; }

// Lay out the workspace and LDS images; false if the head does not fit the fused kernels.
static bool make_plan(int nl, const int* dims, const int* flags, const float* drops,
                      const float* bnp, void* const* ptrs, int B, Plan& p) {
  // ptrs == null: shape-only planning (workspace query)
  if (nl < 1 || nl > HMAXL || B < 1 || B > 64) return false;
  if (dims[nl] < 1 || dims[nl] > 16) return false;
  p.Mp = B <= 32 ? 32 : 64;
  const int Mp = p.Mp;
  HArgs& a = p.a;
  a.nl = nl;
  a.B = B;
  long off = 256;  // header: dropout seed
  int buf_a1 = 8, buf_z = 8, buf_aall = 8;
  a.dw_jobs[0] = 0;
  for (int l = 0; l < nl; ++l) {
    HLayer& L = a.L[l];
    L.in = dims[l];
    L.out = dims[l + 1];
    if (L.in < 1 || L.out < 1 || L.in > 2048 || L.out > 2048) return false;
    L.bn = flags[l] & 3;
    L.relu = (flags[l] >> 2) & 1;
    L.drop = drops ? drops[l] : 0.f;
    if (L.drop < 0.f || L.drop >= 1.f) return false;
    L.eps = bnp ? bnp[2 * l] : 1e-5f;
    L.momentum = bnp ? bnp[2 * l + 1] : 0.1f;
    static void* const none[11] = {};
    void* const* q = ptrs ? ptrs + 11 * l : none;
    L.W = (const float*)q[0];
    L.b = (const float*)q[1];
    L.gamma = (const float*)q[2];
    L.beta = (const float*)q[3];
    L.rmean = (float*)q[4];
    L.rvar = (float*)q[5];
    L.nbt = (long long*)q[6];
    L.gW = (float*)q[7];
    L.gb = (float*)q[8];
    L.ggamma = (float*)q[9];
    L.gbeta = (float*)q[10];
    if (ptrs) {
      if (!L.W) return false;
      if (L.bn && (!L.gamma || !L.beta)) return false;
      if (L.bn == 2 && (!L.rmean || !L.rvar)) return false;
    }
    L.S_a = rup32(L.in) + 8;
    L.S_z = rup32(L.out) + 8;
    L.Np = rup32(L.out);
    L.a_off = off;
    off = al256(off + 2L * Mp * L.S_a);
    L.xhat_off = off;
    if (L.bn) off = al256(off + 4L * Mp * L.Np);
    L.rstd_off = off;
    if (L.bn) off = al256(off + 4L * L.Np);
    L.dz_off = off;
    off = al256(off + 2L * Mp * L.S_z);
    L.st_off = off;
    off = al256(off + 12L * L.out);
    if (l >= 1) buf_a1 = buf_a1 > Mp * L.S_a ? buf_a1 : Mp * L.S_a;
    buf_aall = buf_aall > Mp * L.S_a ? buf_aall : Mp * L.S_a;
    buf_z = buf_z > Mp * L.S_z ? buf_z : Mp * L.S_z;
    a.dw_jobs[l + 1] = a.dw_jobs[l] + (L.out + 15) / 16;
  }
  a.dzl_off = off;
  off = al256(off + 4L * Mp * 16);
  a.logit_off = off;
  off = al256(off + 4L * Mp * 16);
  a.buf_a1 = (buf_a1 + 7) & ~7;
  a.buf_z = (buf_z + 7) & ~7;
  a.buf_aall = (buf_aall + 7) & ~7;
  p.ws_bytes = off;
  p.grid_fwd0 = nl == 1 ? 1 : a.L[0].Np / 16;
  p.grid_bwd0_dw = a.dw_jobs[nl];
  p.grid_bwd0_dx = (a.L[0].in + 15) / 16;
  const long red = 4L * (HW_NT / 64) * (Mp / 16) * 4 * 64;
  p.lds_fwd0 = ((2L * Mp * a.L[0].S_a + 15) & ~15L) + red;
  p.lds_fwd1 = 2L * 2 * a.buf_a1 + 4L * Mp * 16 + 4L * 64;  // + the label slots
  p.lds_bwd1 = 2L * (2 * a.buf_z + a.buf_a1);
  const long dwl = 2L * (a.buf_aall + Mp * 24);
  p.lds_bwd0 = dwl > red ? dwl : red;
  p.lds_fused_base = ((p.lds_fwd1 > p.lds_bwd1 ? p.lds_fwd1 : p.lds_bwd1) + 15) & ~15L;
  p.lds_fused = p.lds_fused_base + 4L * Mp * 16;
  const long lim = 160 * 1024;
  return p.lds_fwd0 <= lim && p.lds_fwd1 <= lim && p.lds_bwd1 <= lim && p.lds_bwd0 <= lim &&
         p.lds_fused <= lim;
}

template <typename K>
static void allow_lds(K kern) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

static bool g_head_init = false;
static unsigned long long* g_head_stamps = nullptr;
static void head_init() {
  if (g_head_init) return;
  allow_lds(head_fwd0_kernel<2, true>);
  allow_lds(head_fwd0_kernel<2, false>);
  allow_lds(head_fwd0_kernel<4, true>);
  allow_lds(head_fwd0_kernel<4, false>);
  allow_lds(head_fwd1_kernel<2, true>);
  allow_lds(head_fwd1_kernel<2, false>);
  allow_lds(head_fwd1_kernel<4, true>);
  allow_lds(head_fwd1_kernel<4, false>);
  allow_lds(head_bwd1_kernel<2>);
  allow_lds(head_bwd1_kernel<4>);
  allow_lds(head_bwd0_kernel<2>);
  allow_lds(head_bwd0_kernel<4>);
  allow_lds(head_fwd1_bwd1_kernel<2, true>);
  allow_lds(head_fwd1_bwd1_kernel<2, false>);
  g_head_init = true;
}

template <int MT, bool V0, bool V1>
static void launch_fwd_t(const Plan& p, const float* x, long ldx, const long long* y, float* out,
                         float* loss, long long* pred, unsigned long long* rng, void* ws,
                         const float* dloss, hipStream_t st) {
  hipLaunchKernelGGL((head_fwd0_kernel<MT, V0>), dim3(p.grid_fwd0), dim3(HW_NT), p.lds_fwd0, st,
                     p.a, x, ldx, rng, (char*)ws, g_head_stamps);
  // (no fused variant for 64-row batches: the bwd1 phase spills at MT = 4)
  if constexpr (MT == 2) {
    if (dloss) {
      hipLaunchKernelGGL((head_fwd1_bwd1_kernel<MT, V1>), dim3(1), dim3(HS_NT), p.lds_fused, st,
                         p.a, y, out, loss, pred, rng, (char*)ws, dloss, g_head_stamps,
                         (int)p.lds_fused_base);
      return;
    }
  }
  {
    hipLaunchKernelGGL((head_fwd1_kernel<MT, V1>), dim3(1), dim3(HS_NT), p.lds_fwd1, st, p.a, y,
                       out, loss, pred, rng, (char*)ws, g_head_stamps);
  }
}

// weight rows may be read as 16-B vectors when every K of the launch is a multiple of 8
template <int MT>
static void launch_fwd(const Plan& p, const float* x, long ldx, const long long* y, float* out,
                       float* loss, long long* pred, unsigned long long* rng, void* ws,
                       const float* dloss, hipStream_t st) {
  const bool v0 = p.a.L[0].in % 8 == 0;
  bool v1 = true;
  for (int l = 1; l < p.a.nl; ++l) v1 = v1 && p.a.L[l].in % 8 == 0;
  if (v0 && v1) launch_fwd_t<MT, true, true>(p, x, ldx, y, out, loss, pred, rng, ws, dloss, st);
  else if (v1) launch_fwd_t<MT, false, true>(p, x, ldx, y, out, loss, pred, rng, ws, dloss, st);
  else if (v0) launch_fwd_t<MT, true, false>(p, x, ldx, y, out, loss, pred, rng, ws, dloss, st);
  else launch_fwd_t<MT, false, false>(p, x, ldx, y, out, loss, pred, rng, ws, dloss, st);
}

}  // namespace

// Install (or clear with null) a device buffer of >= 64 u64 phase timestamps for the next launches.
DN_API int dn_head_set_stamps(void* p) {
  g_head_stamps = (unsigned long long*)p;
  return DN_OK;
}

// Workspace layout of the fused head for batch B: out[0] = workspace bytes, then per layer
// {input image byte offset, its row stride, output-gradient image byte offset, its row stride}
// (bf16 images, rows = batch; used to hand rank-dAD its (A, Delta) pairs).  DN_UNSUPPORTED if
// the head does not fit the fused kernels.
// Per layer: dims[l] -> dims[l+1]; flags[l] = bn (0 none / 1 batch stats / 2 running) | relu << 2.
DN_API int dn_head_layout(int nl, const int* dims, const int* flags, int B, long* out) {
  if (B > 64) return headb_layout(nl, dims, flags, B, out);
  Plan p;
  if (!make_plan(nl, dims, flags, nullptr, nullptr, nullptr, B, p)) return DN_UNSUPPORTED;
  out[0] = p.ws_bytes;
  for (int l = 0; l < nl; ++l) {
    out[1 + 4 * l] = p.a.L[l].a_off;
    out[2 + 4 * l] = p.a.L[l].S_a;
    out[3 + 4 * l] = p.a.L[l].dz_off;
    out[4 + 4 * l] = p.a.L[l].S_z;
  }
  return DN_OK;
}

// ptrs: 11 per layer {W, b, gamma, beta, running_mean, running_var, num_batches_tracked,
//                     gW, gb, ggamma, gbeta} (null where absent; grads only for the backward)
DN_API int dn_head_fwd(int nl, const int* dims, const int* flags, const float* drops,
                       const float* bnp, void* const* ptrs, const float* x, long ldx, int B,
                       const long long* y, float* out, float* loss, long long* pred,
                       unsigned long long* rng, void* ws, int train, int log_out, hipStream_t st) {
  if (B > 64)
    return headb_fwd(nl, dims, flags, drops, bnp, ptrs, x, ldx, B, y, out, loss, pred, rng, ws,
                     train, log_out, st);
  Plan p;
  if (!make_plan(nl, dims, flags, drops, bnp, ptrs, B, p)) return DN_UNSUPPORTED;
  head_init();
  p.a.train = train;
  p.a.log_out = log_out;
  if (p.Mp == 32)
    launch_fwd<2>(p, x, ldx, y, out, loss, pred, rng, ws, nullptr, st);
  else
    launch_fwd<4>(p, x, ldx, y, out, loss, pred, rng, ws, nullptr, st);
  return dn_launch_status();
}

// Training forward that also runs the output-gradient chain (bwd1) for the d loss already held
// at `dloss` (the step's persistent 1): ptrs must carry the gradient buffers; the bias /
// BatchNorm gradients wait in the workspace stash until dn_head_bwd0 (apply_stash = 1) adds
// them, so a backward with a different d loss can still run the full dn_head_bwd instead.
DN_API int dn_head_fwd_train(int nl, const int* dims, const int* flags, const float* drops,
                             const float* bnp, void* const* ptrs, const float* x, long ldx, int B,
                             const long long* y, float* out, float* loss, long long* pred,
                             unsigned long long* rng, void* ws, int log_out, const float* dloss,
                             hipStream_t st) {
  Plan p;
  if (!dloss || !make_plan(nl, dims, flags, drops, bnp, ptrs, B, p)) return DN_UNSUPPORTED;
  if (p.Mp != 32) return DN_UNSUPPORTED;  // B <= 32 only; the caller runs dn_head_fwd instead
  for (int l = 0; l < nl; ++l) {
    const HLayer& L = p.a.L[l];
    if (!L.gW || (L.b && !L.gb) || (L.bn && (!L.ggamma || !L.gbeta))) return DN_BAD_SHAPE;
  }
  head_init();
  p.a.train = 1;
  p.a.log_out = log_out;
  if (p.Mp == 32)
    launch_fwd<2>(p, x, ldx, y, out, loss, pred, rng, ws, dloss, st);
  else
    launch_fwd<4>(p, x, ldx, y, out, loss, pred, rng, ws, dloss, st);
  return dn_launch_status();
}

// The rest of the backward after dn_head_fwd_train: dW of every layer, dX, and the stashed bias
// / BatchNorm gradients added into .grad.
DN_API int dn_head_bwd0(int nl, const int* dims, const int* flags, const float* drops,
                        const float* bnp, void* const* ptrs, int B, void* ws, float* dx, long lddx,
                        hipStream_t st) {
  Plan p;
  if (!make_plan(nl, dims, flags, drops, bnp, ptrs, B, p)) return DN_UNSUPPORTED;
  for (int l = 0; l < nl; ++l) {
    const HLayer& L = p.a.L[l];
    if (!L.gW || (L.b && !L.gb) || (L.bn && (!L.ggamma || !L.gbeta))) return DN_BAD_SHAPE;
  }
  head_init();
  p.a.train = 1;
  p.a.log_out = 0;
  const int grid0 = p.grid_bwd0_dw + (dx ? p.grid_bwd0_dx : 0);
  if (p.Mp == 32)
    hipLaunchKernelGGL(head_bwd0_kernel<2>, dim3(grid0), dim3(HW_NT), p.lds_bwd0, st, p.a,
                       (const char*)ws, dx, lddx, 1, g_head_stamps);
  else
    hipLaunchKernelGGL(head_bwd0_kernel<4>, dim3(grid0), dim3(HW_NT), p.lds_bwd0, st, p.a,
                       (const char*)ws, dx, lddx, 1, g_head_stamps);
  return dn_launch_status();
}

// Backward of a training-mode dn_head_fwd on the same workspace; dloss: device scalar d out/d loss;
// dx (may be null): d loss / d x, row stride lddx.
DN_API int dn_head_bwd(int nl, const int* dims, const int* flags, const float* drops,
                       const float* bnp, void* const* ptrs, int B, void* ws, const float* dloss,
                       float* dx, long lddx, hipStream_t st) {
  if (B > 64) return headb_bwd(nl, dims, flags, drops, bnp, ptrs, B, ws, dloss, dx, lddx, st);
  Plan p;
  if (!make_plan(nl, dims, flags, drops, bnp, ptrs, B, p)) return DN_UNSUPPORTED;
  for (int l = 0; l < nl; ++l) {
    const HLayer& L = p.a.L[l];
    if (!L.gW || (L.b && !L.gb) || (L.bn && (!L.ggamma || !L.gbeta))) return DN_BAD_SHAPE;
  }
  head_init();
  p.a.train = 1;
  p.a.log_out = 0;
  const int grid0 = p.grid_bwd0_dw + (dx ? p.grid_bwd0_dx : 0);
  if (p.Mp == 32) {
    hipLaunchKernelGGL(head_bwd1_kernel<2>, dim3(1), dim3(HS_NT), p.lds_bwd1, st, p.a, (char*)ws,
                       dloss, g_head_stamps);
    hipLaunchKernelGGL(head_bwd0_kernel<2>, dim3(grid0), dim3(HW_NT), p.lds_bwd0, st, p.a,
                       (const char*)ws, dx, lddx, 0, g_head_stamps);
  } else {
    hipLaunchKernelGGL(head_bwd1_kernel<4>, dim3(1), dim3(HS_NT), p.lds_bwd1, st, p.a, (char*)ws,
                       dloss, g_head_stamps);
    hipLaunchKernelGGL(head_bwd0_kernel<4>, dim3(grid0), dim3(HW_NT), p.lds_bwd0, st, p.a,
                       (const char*)ws, dx, lddx, 0, g_head_stamps);
  }
  return dn_launch_status();
}
