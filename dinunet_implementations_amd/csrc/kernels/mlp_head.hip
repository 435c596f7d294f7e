// Fused MLP head + loss for gfx950: the ICA classifier (reference comps/icalstm/models.py:95-103
// + comps/icalstm/__init__.py:59-63) and the FreeSurfer MSANNet (comps/fs/models.py:4-31 +
// comps/fs/__init__.py:54-57) as ONE forward launch and ONE backward launch.
//
// A head is a chain of at most HMAXL layers, each
//     [dropout on the input] -> Linear (+bias) -> [BatchNorm1d] -> [ReLU]
// ending in softmax cross-entropy (probabilities out) or log-softmax + NLL (log-probs out).
// At these sizes (batch <= 64, widths <= ~1k) the head is pure latency: the unfused graph is ~40
// tiny kernels.  Here one 16-wave workgroup keeps every activation in LDS:
//  * forward: wave w owns output-column tiles n = 16w.. for ALL batch rows, so BatchNorm column
//    statistics are an in-register reduction (lanes l, l^16, l^32, l^48 hold one column); the
//    layer GEMM is 16x16x32 bf16 MFMA, A = activation rows from LDS (ds_read_b128), B = the fp32
//    master weight rows read straight from global memory and rounded while loading.
//  * backward: dW = dZ^T A is an MFMA over the batch whose operands are built with the CDNA4 LDS
//    transpose read (ds_read_b64_tr_b16) from the same row-major activation images; dA = dZ W
//    again gives each wave whole columns, so ReLU/dropout masks and the BatchNorm backward
//    (two column sums) happen in the epilogue.  Parameter gradients are accumulated into the
//    caller's fp32 .grad buffers (flat gradient buffer views), so no autograd adds run.
//  * dropout masks come from a counter-based hash of (seed, layer, row, col); the seed lives in
//    device memory and is bumped by the kernel, so a captured HIP graph draws fresh masks on
//    every replay.  The backward regenerates the mask from the seed saved in the workspace.
#include "common.h"

namespace {

constexpr int HMAXL = 6;
// 16 waves for batches <= 32 (MT = 2); 8 waves (256-VGPR budget, no spills) for batches <= 64
template <int MT> struct HCfg { static constexpr int NT = MT == 2 ? 1024 : 512, NW = NT / 64; };

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

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
};

struct HArgs {
  HLayer L[HMAXL];
  int nl, B;
  int buf_a, buf_z;  // LDS image sizes (elements) for the activation / gradient buffers
  long dzl_off;      // fp32 [Mp][16] d loss / d logits (unscaled)
  int train, log_out;
};

__host__ __device__ constexpr int rup32(int v) { return (v + 31) & ~31; }

__device__ __forceinline__ uint32_t hmix(uint64_t seed, uint32_t layer, uint32_t idx) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + ((((uint64_t)layer) << 32) | idx) + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 40);
}

__device__ __forceinline__ bool hkeep(uint64_t seed, int layer, int m, int k, int K, float p) {
  return (float)hmix(seed, (uint32_t)layer, (uint32_t)(m * K + k)) * (1.f / 16777216.f) >= p;
}

// sum over the four lanes holding one accumulator column (l, l^16, l^32, l^48)
__device__ __forceinline__ float colsum4(float v) {
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

// B fragment from weight ROWS: lane -> n = n (row), k .. k+7 (contiguous)
__device__ __forceinline__ bf16x8 wfrag_rows(const float* __restrict__ W, int N, int K, int n, int k) {
  bf16x8 f;
  if (n < N && k + 8 <= K && (K & 3) == 0) {
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(W + (long)n * K + k);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(W + (long)n * K + k + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { f[e] = (bf16)v0[e]; f[4 + e] = (bf16)v1[e]; }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (n < N && k + e < K) ? (bf16)W[(long)n * K + k + e] : (bf16)0.f;
  }
  return f;
}

// B fragment from weight COLUMNS: lane -> column kk, rows n .. n+7 (stride K)
__device__ __forceinline__ bf16x8 wfrag_cols(const float* __restrict__ W, int N, int K, int n, int kk) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (n + j < N && kk < K) ? (bf16)W[(long)(n + j) * K + kk] : (bf16)0.f;
  return f;
}

// Fragment with lane i <- column c0 + (i & 15) and element j <- row k0 + 8 * (i >> 4) + j of a
// row-major LDS image (row stride S elements): two hardware-transposed 4x16 reads.
__device__ __forceinline__ bf16x8 tr_frag(const bf16* img, int S, int c0, int k0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const bf16* a0 = img + (k0 + 8 * g + q) * S + c0 + 4 * p;
  const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * S));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int MT>
__global__ void __launch_bounds__(HCfg<MT>::NT)
head_fwd_kernel(HArgs a, const float* __restrict__ x, long ldx, const long long* __restrict__ y,
                float* __restrict__ out, float* __restrict__ loss, long long* __restrict__ pred,
                unsigned long long* __restrict__ rng, char* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int Mp = 16 * MT;
  constexpr int HNT = HCfg<MT>::NT, HNW = HCfg<MT>::NW;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int B = a.B;
  const bool train = a.train != 0;
  bf16* cur = reinterpret_cast<bf16*>(smem);
  bf16* nxt = cur + a.buf_a;
  float* logit = reinterpret_cast<float*>(nxt + a.buf_a);  // [Mp][16]
  const uint64_t seed = rng ? *rng : 0ull;

  // ---- input image (dropout of layer 0 applied), also saved for the backward
  {
    const HLayer& L0 = a.L[0];
    const int K = L0.in, Kp = rup32(K), S = L0.S_a;
    const float inv = L0.drop > 0.f ? 1.f / (1.f - L0.drop) : 1.f;
    bf16* wimg = reinterpret_cast<bf16*>(ws + L0.a_off);
    for (int idx = tid; idx < Mp * Kp; idx += HNT) {
      const int m = idx / Kp, k = idx - m * Kp;
      float v = 0.f;
      if (m < B && k < K) {
        v = x[(long)m * ldx + k];
        if (train && L0.drop > 0.f) v = hkeep(seed, 0, m, k, K, L0.drop) ? v * inv : 0.f;
      }
      const bf16 bv = (bf16)v;
      cur[m * S + k] = bv;
      if (train) wimg[m * S + k] = bv;
    }
  }
  __syncthreads();

  for (int l = 0; l < a.nl; ++l) {
    const HLayer& L = a.L[l];
    const int K = L.in, N = L.out, Kp = rup32(K), S = L.S_a;
    const bool last = l == a.nl - 1;
    const int ntiles = last ? 1 : L.Np / 16;  // cover rup32(out): the next image's pad is zeroed
    const HLayer& Ln = a.L[last ? l : l + 1];
    const int Sn = Ln.S_a;
    const float pn = last ? 0.f : Ln.drop;
    const float invn = pn > 0.f ? 1.f / (1.f - pn) : 1.f;
    bf16* wnext = reinterpret_cast<bf16*>(ws + Ln.a_off);
    float* xhat_ws = reinterpret_cast<float*>(ws + L.xhat_off);
    float* rstd_ws = reinterpret_cast<float*>(ws + L.rstd_off);
    for (int t = wid; t < ntiles; t += HNW) {
      const int n = 16 * t + (lane & 15);
      f32x4 acc[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int k0 = 0; k0 < Kp; k0 += 32) {
        const bf16x8 bfr = wfrag_rows(L.W, N, K, n, k0 + 8 * (lane >> 4));
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(cur + (16 * mt + (lane & 15)) * S + k0 + 8 * (lane >> 4));
          acc[mt] = mfma16(af, bfr, acc[mt]);
        }
      }
      const bool cv = n < N;
      const float bias = (L.b && cv) ? L.b[n] : 0.f;
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
            L.rmean[n] = (1.f - mo) * L.rmean[n] + mo * mean;
            L.rvar[n] = (1.f - mo) * L.rvar[n] + mo * v * ((float)B / (float)(B > 1 ? B - 1 : 1));
          }
        } else {
          mean = cv ? L.rmean[n] : 0.f;
          rstd = cv ? rsqrtf(L.rvar[n] + L.eps) : 0.f;
        }
        const float ga = cv ? L.gamma[n] : 0.f, be = cv ? L.beta[n] : 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + 4 * (lane >> 4) + r;
            const float xh = (z[mt][r] - mean) * rstd;
            if (train) xhat_ws[row * L.Np + n] = (row < B && cv) ? xh : 0.f;
            z[mt][r] = ga * xh + be;
          }
        if (train && lane < 16) rstd_ws[n] = cv ? rstd : 0.f;
      }
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
            if (train && pn > 0.f && v != 0.f) v = hkeep(seed, l + 1, row, n, N, pn) ? v * invn : 0.f;
            const bf16 bv = (bf16)v;
            nxt[row * Sn + n] = bv;
            if (train) wnext[row * Sn + n] = bv;
          }
        }
    }
    if (train && L.bn == 2 && tid == 0 && L.nbt) *L.nbt += 1;
    __syncthreads();
    bf16* t = cur;
    cur = nxt;
    nxt = t;
  }

  // ---- softmax / log-softmax + CE / NLL, argmax; wave 0, lane = batch row
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
      long long yc = y[m];
      yc = yc < 0 ? 0 : (yc >= C ? C - 1 : yc);
      float* dzl = reinterpret_cast<float*>(ws + a.dzl_off);
      for (int c = 0; c < C; ++c) {
        const float lp = logit[m * 16 + c] - lse;
        const float p = expf(lp);
        out[(long)m * C + c] = a.log_out ? lp : p;
        if (train) dzl[m * 16 + c] = (p - (c == yc ? 1.f : 0.f)) / (float)B;
      }
      ls = lse - logit[m * 16 + yc];
      pred[m] = am;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) ls += __shfl_xor(ls, off);
    if (lane == 0) {
      *loss = ls / (float)B;
      if (train) *reinterpret_cast<unsigned long long*>(ws) = seed;
      if (train && rng) *rng = seed + 1ull;
    }
  }
}

template <int MT>
__global__ void __launch_bounds__(HCfg<MT>::NT)
head_bwd_kernel(HArgs a, char* __restrict__ ws, const float* __restrict__ dloss,
                float* __restrict__ dx, long lddx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int Mp = 16 * MT;
  constexpr int HNT = HCfg<MT>::NT, HNW = HCfg<MT>::NW;
  constexpr int G = 4;  // dW tiles per wave batch (global read-modify-write in flight together)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int B = a.B;
  bf16* dz = reinterpret_cast<bf16*>(smem);
  bf16* dzn = dz + a.buf_z;
  bf16* abuf = dzn + a.buf_z;
  const float gs = *dloss;
  const uint64_t seed = *reinterpret_cast<const unsigned long long*>(ws);
  const float* dzl = reinterpret_cast<const float*>(ws + a.dzl_off);

  {  // gradient of the logits
    const HLayer& L = a.L[a.nl - 1];
    const int C = L.out, Cp = rup32(C), S = L.S_z;
    bf16* wdz = reinterpret_cast<bf16*>(ws + L.dz_off);
    for (int idx = tid; idx < Mp * Cp; idx += HNT) {
      const int m = idx / Cp, c = idx - m * Cp;
      const float v = (m < B && c < C) ? gs * dzl[m * 16 + c] : 0.f;
      dz[m * S + c] = (bf16)v;
      wdz[m * S + c] = (bf16)v;
    }
    if (L.gb && tid < C) {
      float s = 0.f;
      for (int m = 0; m < B; ++m) s += dzl[m * 16 + tid];
      L.gb[tid] += gs * s;
    }
  }

  for (int l = a.nl - 1; l >= 0; --l) {
    const HLayer& L = a.L[l];
    const int K = L.in, N = L.out, Kp = rup32(K), Np = L.Np, Sa = L.S_a, Sz = L.S_z;
    {  // this layer's input activations (post-dropout, bf16) into LDS
      const bf16x8* src = reinterpret_cast<const bf16x8*>(ws + L.a_off);
      bf16x8* dst = reinterpret_cast<bf16x8*>(abuf);
      for (int i = tid; i < Mp * Sa / 8; i += HNT) dst[i] = src[i];
    }
    __syncthreads();

    // (i) dW[n][k] += sum_m dz[m][n] a[m][k]
    {
      const int tn = (N + 15) / 16, tk = (K + 15) / 16, T = tn * tk;
      for (int t0 = wid * G; t0 < T; t0 += HNW * G) {
        f32x4 acc[G];
#pragma unroll
        for (int gi = 0; gi < G; ++gi) {
          acc[gi] = f32x4{0.f, 0.f, 0.f, 0.f};
          const int t = t0 + gi;
          if (t < T) {
            const int n0 = 16 * (t / tk), k0 = 16 * (t % tk);
#pragma unroll
            for (int ms = 0; ms < Mp; ms += 32)
              acc[gi] = mfma16(tr_frag(dz, Sz, n0, ms, lane), tr_frag(abuf, Sa, k0, ms, lane), acc[gi]);
          }
        }
        float old[G][4];
#pragma unroll
        for (int gi = 0; gi < G; ++gi) {
          const int t = t0 + gi;
          const int n0 = 16 * (t / tk), k = 16 * (t % tk) + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = n0 + 4 * (lane >> 4) + r;
            old[gi][r] = (t < T && n < N && k < K) ? L.gW[(long)n * K + k] : 0.f;
          }
        }
#pragma unroll
        for (int gi = 0; gi < G; ++gi) {
          const int t = t0 + gi;
          const int n0 = 16 * (t / tk), k = 16 * (t % tk) + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = n0 + 4 * (lane >> 4) + r;
            if (t < T && n < N && k < K) L.gW[(long)n * K + k] = old[gi][r] + acc[gi][r];
          }
        }
      }
    }

    // (ii) dA = dz W, then (dropout, ReLU, BatchNorm, bias) backward of the layer below
    if (l > 0 || dx) {
      const HLayer& P = a.L[l > 0 ? l - 1 : 0];
      const float inv = L.drop > 0.f ? 1.f / (1.f - L.drop) : 1.f;
      const float* xhat_ws = reinterpret_cast<const float*>(ws + P.xhat_off);
      const float* rstd_ws = reinterpret_cast<const float*>(ws + P.rstd_off);
      bf16* wdz = reinterpret_cast<bf16*>(ws + P.dz_off);
      for (int t = wid; t < Kp / 16; t += HNW) {
        const int kk = 16 * t + (lane & 15);
        f32x4 acc[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
        for (int ns = 0; ns < Np; ns += 32) {
          const bf16x8 bfr = wfrag_cols(L.W, N, K, ns + 8 * (lane >> 4), kk);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(dz + (16 * mt + (lane & 15)) * Sz + ns + 8 * (lane >> 4));
            acc[mt] = mfma16(af, bfr, acc[mt]);
          }
        }
        const bool kv = kk < K;
        float d[MT][4];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + 4 * (lane >> 4) + r;
            float v = (row < B && kv) ? acc[mt][r] : 0.f;
            if (a.train && L.drop > 0.f && v != 0.f) v = hkeep(seed, l, row, kk, K, L.drop) ? v * inv : 0.f;
            d[mt][r] = v;
          }
        if (l == 0) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * mt + 4 * (lane >> 4) + r;
              if (row < B && kv) dx[(long)row * lddx + kk] = d[mt][r];
            }
          continue;
        }
        if (P.relu) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * mt + 4 * (lane >> 4) + r;
              if (!((float)abuf[row * Sa + kk] > 0.f)) d[mt][r] = 0.f;
            }
        }
        if (P.bn) {
          float xh[MT][4];
          float s1 = 0.f, s2 = 0.f;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * mt + 4 * (lane >> 4) + r;
              xh[mt][r] = xhat_ws[row * P.Np + kk];
              s1 += d[mt][r];
              s2 += d[mt][r] * xh[mt][r];
            }
          s1 = colsum4(s1);
          s2 = colsum4(s2);
          if (lane < 16 && kv) {
            P.ggamma[kk] += s2;
            P.gbeta[kk] += s1;
          }
          const float ga = kv ? P.gamma[kk] : 0.f, rs = rstd_ws[kk];
          const float m1 = s1 / (float)B, m2 = s2 / (float)B;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * mt + 4 * (lane >> 4) + r;
              d[mt][r] = (row < B && kv) ? ga * rs * (d[mt][r] - m1 - xh[mt][r] * m2) : 0.f;
            }
        }
        if (P.gb) {
          float sb = 0.f;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) sb += d[mt][r];
          sb = colsum4(sb);
          if (lane < 16 && kv) P.gb[kk] += sb;
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
    }
    __syncthreads();
    bf16* t = dz;
    dz = dzn;
    dzn = t;
  }
}

struct Plan {
  HArgs a;
  long ws_bytes;
  int Mp;
  long lds_fwd, lds_bwd;
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
  int buf_a = 0, buf_z = 0;
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
    buf_a = buf_a > Mp * L.S_a ? buf_a : Mp * L.S_a;
    buf_z = buf_z > Mp * L.S_z ? buf_z : Mp * L.S_z;
    if (l + 1 < nl && L.Np != rup32(dims[l + 1])) return false;
  }
  a.dzl_off = off;
  off = al256(off + 4L * Mp * 16);
  a.buf_a = (buf_a + 7) & ~7;
  a.buf_z = (buf_z + 7) & ~7;
  p.ws_bytes = off;
  p.lds_fwd = 2L * 2 * a.buf_a + 4L * Mp * 16;
  p.lds_bwd = 2L * (2 * a.buf_z + a.buf_a);
  return p.lds_fwd <= 160 * 1024 && p.lds_bwd <= 160 * 1024;
}

template <typename K>
static void allow_lds(K kern) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

static bool g_head_init = false;
static void head_init() {
  if (g_head_init) return;
  allow_lds(head_fwd_kernel<2>);
  allow_lds(head_fwd_kernel<4>);
  allow_lds(head_bwd_kernel<2>);
  allow_lds(head_bwd_kernel<4>);
  g_head_init = true;
}

}  // namespace

// Workspace layout of the fused head for batch B: out[0] = workspace bytes, then per layer
// {input image byte offset, its row stride, output-gradient image byte offset, its row stride}
// (bf16 images, rows = batch; used to hand rank-dAD its (A, Delta) pairs).  DN_UNSUPPORTED if
// the head does not fit the fused kernels.
// Per layer: dims[l] -> dims[l+1]; flags[l] = bn (0 none / 1 batch stats / 2 running) | relu << 2.
DN_API int dn_head_layout(int nl, const int* dims, const int* flags, int B, long* out) {
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
  Plan p;
  if (!make_plan(nl, dims, flags, drops, bnp, ptrs, B, p)) return DN_UNSUPPORTED;
  head_init();
  p.a.train = train;
  p.a.log_out = log_out;
  if (p.Mp == 32)
    hipLaunchKernelGGL(head_fwd_kernel<2>, dim3(1), dim3(HCfg<2>::NT), p.lds_fwd, st, p.a, x, ldx, y, out,
                       loss, pred, rng, (char*)ws);
  else
    hipLaunchKernelGGL(head_fwd_kernel<4>, dim3(1), dim3(HCfg<4>::NT), p.lds_fwd, st, p.a, x, ldx, y, out,
                       loss, pred, rng, (char*)ws);
  return dn_launch_status();
}

// Backward of a training-mode dn_head_fwd on the same workspace; dloss: device scalar d out/d loss.
DN_API int dn_head_bwd(int nl, const int* dims, const int* flags, const float* drops,
                       const float* bnp, void* const* ptrs, int B, void* ws, const float* dloss,
                       float* dx, long lddx, hipStream_t st) {
  Plan p;
  if (!make_plan(nl, dims, flags, drops, bnp, ptrs, B, p)) return DN_UNSUPPORTED;
  for (int l = 0; l < nl; ++l) {
    const HLayer& L = p.a.L[l];
    if (!L.gW || (L.b && !L.gb) || (L.bn && (!L.ggamma || !L.gbeta))) return DN_BAD_SHAPE;
  }
  head_init();
  p.a.train = 1;
  p.a.log_out = 0;
  if (p.Mp == 32)
    hipLaunchKernelGGL(head_bwd_kernel<2>, dim3(1), dim3(HCfg<2>::NT), p.lds_bwd, st, p.a, (char*)ws,
                       dloss, dx, lddx);
  else
    hipLaunchKernelGGL(head_bwd_kernel<4>, dim3(1), dim3(HCfg<4>::NT), p.lds_bwd, st, p.a, (char*)ws,
                       dloss, dx, lddx);
  return dn_launch_status();
}
