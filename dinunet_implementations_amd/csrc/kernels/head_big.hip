// Fused MLP head + loss for ANY batch size: the ICA classifier (reference
// comps/icalstm/models.py:95-103, trained at the large batches of its pretrain spec,
// compspec.json:120-148) and the FreeSurfer MSANNet (comps/fs/models.py:4-31).
//
// The batch <= 64 kernels (mlp_head.hip) keep every row of a 16-column tile in one wave, so
// BatchNorm statistics are an in-register reduction.  Here the batch is tiled over workgroups
// (64-row blocks) and the statistics become a deterministic two-level reduction: each row block
// writes per-column partials, and every consumer merges them in a fixed order (Chan's (mean, M2)
// merge forward, plain sums backward).  Launches (L layers):
//   fwd(l), l = 0..L-1   grid (row blocks x 64-column blocks), 4 waves, 16x16x32 bf16 MFMA.
//       prologue: merge layer l-1's partials into its BatchNorm scale / shift; block (0,0) saves
//       (mean, rstd) for the backward and updates the running statistics.
//       K loop: the input tile is staged in LDS with layer l-1's BN + ReLU and layer l's dropout
//       applied while loading (bf16; column block 0 also writes it to the workspace for dW and
//       for rank-dAD), the weight tile is rounded from the fp32 master weights.
//       epilogue: + bias -> Z_l (fp32), this row block's (mean, M2) per column.
//   loss                 one workgroup: softmax / log-softmax, CE / NLL, argmax, mean loss,
//       dlogits = p - onehot and its column sums; bumps the dropout seed.
//   backward, per layer l from the last: [bn(l) if layer l has BatchNorm] then bwd(l):
//       bwd(l) dA jobs (row block x 64 input columns): dA = dZ_l W_l, then layer l's dropout mask
//         and layer l-1's ReLU mask.  If layer l-1 has BatchNorm the result (dy) goes out in fp32
//         with per-row-block column sums (sum dy, sum dy xhat); otherwise it IS dZ_{l-1} (bf16
//         image + fp32 column partials for the bias gradient).  For l = 0 it is d input.
//       bwd(l) dW jobs (64 x 64 weight tiles x row splits): dZ_l^T A_l over the split's rows,
//         operands from the CDNA4 LDS transpose read, into gW (one split) or fp32 partials that
//         a small reduce launch adds in split order; the first split of column block 0 adds the
//         bias gradient.
//       bn(l) (row blocks): merges the column sums (= d beta, d gamma) and writes
//         dZ_l = gamma rstd (dy - mean(dy) - xhat mean(dy xhat)).
// The last layer must be a plain Linear (no BatchNorm / ReLU after the logits), as in both heads.
#include "head_common.h"

namespace {

constexpr int BMAXL = 6;
constexpr int BNT = 256;        // 4 waves per workgroup
constexpr int RB = 64;          // rows per row block
constexpr int TB = 64;          // columns per column block and per K chunk
constexpr int LS = TB + 8;      // LDS row stride (bf16 elements) of a staged tile: 144 B
constexpr int LOSS_NT = 1024;
constexpr int MAXD = 2048;      // widest layer

__host__ __device__ constexpr int rup8(int v) { return (v + 7) & ~7; }

struct F2 {
  float x, y;
};

struct BLayer {
  const float* W;  // [out][in]
  const float* b;
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  long long* nbt;
  float* gW;
  float* gb;
  float* ggamma;
  float* gbeta;
  int in, out;
  int bn;      // 0 none, 1 batch statistics always, 2 batch statistics + running update / running
  int relu;
  float drop;  // dropout on this layer's INPUT (training only)
  float eps, momentum;
  int S_a, S_z;  // row strides of the bf16 input-activation and output-gradient images
  long a_off;    // bf16 [B][S_a] input activations (post dropout)
  long z_off;    // fp32 [B][out] pre-BatchNorm outputs (bias included)
  long part_off; // F2 [nrb][out] per-row-block (mean, M2)
  long stat_off; // F2 [out] (mean, rstd) of the forward
  long dy_off;   // fp32 [B][out] d loss / d BN output (post ReLU mask)
  long part2_off;  // F2 [nrb][out] per-row-block (sum dy, sum dy xhat)
  long dz_off;   // bf16 [B][S_z] d loss / d Z
  long dbp_off;  // fp32 [nrb][out] per-row-block column sums of dZ (bias gradient)
  long dwp_off;  // fp32 [rs][out][in] row-split partial weight gradients of this layer
};

struct BArgs {
  BLayer L[BMAXL];
  int nl, B, nrb, train, log_out;
  long g_off;   // fp32 [B][C] p - onehot
  long gs_off;  // fp32 [16] its column sums
};

// gW of layer l += its RS row-split partials, added in split order (deterministic); workgroup
// `bid` of `nb`.  Run by the extra workgroups of the NEXT backward launch (each layer has its own
// partials, so layer l-1's kernels do not overwrite them), or by headb_dw_reduce_kernel for the
// first layer: a launch of its own is ~4.7 us of floor for a few microseconds of loads.
__device__ __forceinline__ void dw_reduce_body(const BArgs& a, int l, const char* ws, int RS,
                                               int bid, int nb) {
  const BLayer& L = a.L[l];
  const long NK = (long)L.out * L.in;
  const float* part = reinterpret_cast<const float*>(ws + L.dwp_off);
  for (long e = bid * 256L + threadIdx.x; e < NK; e += (long)nb * 256) {
    float v = 0.f;
    for (int s8 = 0; s8 < RS; s8 += 8) {  // 8 split loads in flight, added in split order
      float qs[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) qs[i] = part[min(s8 + i, RS - 1) * NK + e];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (s8 + i < RS) v += qs[i];
    }
    L.gW[e] += v;
  }
}

// a pending reduce riding on a launch: layer rl (< 0: none) with rs splits, in the launch's
// workgroups from r0 on
struct RedJob {
  int rl, rs, r0;
};

// Row splits of one layer's dW reduction: enough (tile, split) jobs for ~2 per CU, each split at
// least one 64-row block.
static inline int dw_splits(int nW, int nrb) {
  int rs = (512 + nW - 1) / nW;
  if (rs > 16) rs = 16;
  if (rs > nrb) rs = nrb;
  return rs < 1 ? 1 : rs;
}

template <bool V>
__device__ __forceinline__ void load4(const float* __restrict__ p, long ld, int r, int c, int R,
                                      int C, float (&v)[4]) {
  if constexpr (V) {  // C % 4 == 0, ld % 4 == 0: the quad is all in or all out
    const bool ok = r < R && c < C;
    const f32x4 q = *reinterpret_cast<const f32x4*>(p + (ok ? (long)r * ld + c : 0));
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = ok ? q[e] : 0.f;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool ok = r < R && c + e < C;
      const float q = p[ok ? (long)r * ld + c + e : 0];
      v[e] = ok ? q : 0.f;
    }
  }
}

__device__ __forceinline__ bf16x4 to_bf4(const float (&v)[4]) {
  bf16x4 b;
#pragma unroll
  for (int e = 0; e < 4; ++e) b[e] = (bf16)v[e];
  return b;
}

// BatchNorm scale / shift of layer P at column k (identity without BN).  Batch statistics come
// from the per-row-block partials merged in row-block order; the leader block records them for
// the backward and updates the running statistics.
__device__ __forceinline__ void bn_affine(const BArgs& a, const BLayer& P, const char* ws, int k,
                                          bool leader, char* wsw, float& s, float& t) {
  s = 1.f;
  t = 0.f;
  if (!P.bn) return;
  const bool train = a.train != 0;
  // the affine parameters and running statistics are loaded with the partials, not after the
  // merge (each was one more dependent round trip before the first chunk)
  const float gk = P.gamma[k], bk = P.beta[k];
  const bool upd = leader && train && P.bn == 2;
  const float rm0 = (upd || !(P.bn == 1 || train)) ? P.rmean[k] : 0.f;
  const float rv0 = (upd || !(P.bn == 1 || train)) ? P.rvar[k] : 0.f;
  float mean, rstd;
  if (P.bn == 1 || train) {
    const F2* part = reinterpret_cast<const F2*>(ws + P.part_off);
    float cnt = 0.f, m2 = 0.f;
    mean = 0.f;
    for (int r8 = 0; r8 < a.nrb; r8 += 16) {  // 16 partial loads in flight, merged in order
      F2 qs[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) qs[i] = part[(long)min(r8 + i, a.nrb - 1) * P.out + k];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int rb = r8 + i;
        if (rb < a.nrb) {
          const float nb = (float)min(RB, a.B - rb * RB);
          const F2 q = qs[i];
          const float tot = cnt + nb;
          const float d = q.x - mean;
          mean += d * (nb / tot);
          m2 += q.y + d * d * (cnt * nb / tot);
          cnt = tot;
        }
      }
    }
    const float var = m2 / (float)a.B;
    rstd = rsqrtf(var + P.eps);
    if (leader) {
      reinterpret_cast<F2*>(wsw + P.stat_off)[k] = F2{mean, rstd};
      if (upd) {
        const float mo = P.momentum;
        P.rmean[k] = (1.f - mo) * rm0 + mo * mean;
        P.rvar[k] = (1.f - mo) * rv0 + mo * var * ((float)a.B / (float)(a.B > 1 ? a.B - 1 : 1));
      }
    }
  } else {
    mean = rm0;
    rstd = rsqrtf(rv0 + P.eps);
  }
  s = gk * rstd;
  t = bk - mean * s;
}

// ---------------------------------------------------------------------------------------------
template <bool VX, bool VW>
__global__ void __launch_bounds__(BNT)
headb_fwd_kernel(BArgs a, int l, const float* __restrict__ x, long ldx,
                 const unsigned long long* __restrict__ rng, char* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const BLayer& L = a.L[l];
  const int K = L.in, N = L.out, B = a.B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rb = blockIdx.x, r0 = rb * RB, n0 = blockIdx.y * TB;
  const bool train = a.train != 0;
  bf16* At = reinterpret_cast<bf16*>(smem);            // [RB][LS]
  bf16* Wt = At + RB * LS;                             // [TB][LS]
  float* sc = reinterpret_cast<float*>(Wt + TB * LS);  // [K]
  float* sh = sc + K;
  const float pdrop = train ? L.drop : 0.f;
  const float inv = pdrop > 0.f ? 1.f / (1.f - pdrop) : 1.f;
  const uint64_t seed = (pdrop > 0.f && rng) ? *rng : 0ull;
  const float* src = x;
  long ld = ldx;
  bool prelu = false;
  if (l > 0) {
    src = reinterpret_cast<const float*>(ws + a.L[l - 1].z_off);
    ld = K;
    prelu = a.L[l - 1].relu != 0;
  }
  const int sr = tid >> 4, sq = (tid & 15) * 4;  // staging: 16 rows x 16 column quads per pass
  // two chunks of raw input / weight values in registers ahead of the MFMAs, the first two issued
  // before the BatchNorm prologue (they do not depend on it): at one chunk of prefetch the loop
  // was a chain of K / 64 global round trips (21.6 us for the 768-wide layer at B = 2048).
  float va0[4][4], vw0[4][4], va1[4][4], vw1[4][4];
  auto load_chunk = [&](int kc, float (&va)[4][4], float (&vw)[4][4]) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      load4<VX>(src, ld, r0 + sr + 16 * p, kc + sq, B, K, va[p]);
      load4<VW>(L.W, K, n0 + sr + 16 * p, kc + sq, N, K, vw[p]);
    }
  };
  load_chunk(0, va0, vw0);
  if (TB < K) load_chunk(TB, va1, vw1);
  if (l > 0) {
    const BLayer& P = a.L[l - 1];
    const bool leader = blockIdx.x == 0 && blockIdx.y == 0;
    for (int k = tid; k < K; k += BNT) {
      float s, t;
      bn_affine(a, P, ws, k, leader, ws, s, t);
      sc[k] = s;
      sh[k] = t;
    }
    __syncthreads();
  }
  bf16* aimg = reinterpret_cast<bf16*>(ws + L.a_off);
  const bool wimg = train && blockIdx.y == 0;
  f32x4 acc[4] = {};
  auto stage = [&](int kc, const float (&va)[4][4], const float (&vw)[4][4]) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = sr + 16 * p, gr = r0 + row, k = kc + sq;
      float v[4] = {va[p][0], va[p][1], va[p][2], va[p][3]};
      if (l > 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = gr < B && k + e < K;
          float y = sc[ok ? k + e : 0] * v[e] + sh[ok ? k + e : 0];
          if (prelu) y = fmaxf(y, 0.f);
          v[e] = ok ? y : 0.f;
        }
      }
      if (pdrop > 0.f) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (v[e] != 0.f) v[e] = hkeep(seed, l, gr, k + e, K, pdrop) ? v[e] * inv : 0.f;
      }
      const bf16x4 b4 = to_bf4(v);
      *reinterpret_cast<bf16x4*>(At + row * LS + sq) = b4;
      if (wimg && gr < B && k < L.S_a) *reinterpret_cast<bf16x4*>(aimg + (long)gr * L.S_a + k) = b4;
      *reinterpret_cast<bf16x4*>(Wt + row * LS + sq) = to_bf4(vw[p]);
    }
  };
  auto mma = [&]() {
#pragma unroll
    for (int ks = 0; ks < TB; ks += 32) {
      const int kk = ks + 8 * (lane >> 4);
      const bf16x8 bw = *reinterpret_cast<const bf16x8*>(Wt + (16 * wid + (lane & 15)) * LS + kk);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(At + (16 * mt + (lane & 15)) * LS + kk);
        acc[mt] = mfma16(av, bw, acc[mt]);
      }
    }
  };
  for (int kc = 0; kc < K; kc += 2 * TB) {
    stage(kc, va0, vw0);
    __syncthreads();
    if (kc + 2 * TB < K) load_chunk(kc + 2 * TB, va0, vw0);
    mma();
    __syncthreads();
    if (kc + TB >= K) break;
    stage(kc + TB, va1, vw1);
    __syncthreads();
    if (kc + 3 * TB < K) load_chunk(kc + 3 * TB, va1, vw1);
    mma();
    __syncthreads();
  }
  const int n = n0 + 16 * wid + (lane & 15);
  const bool cv = n < N;
  const float bias = (cv && L.b) ? L.b[n] : 0.f;
  float* Z = reinterpret_cast<float*>(ws + L.z_off);
  const int cnt = min(RB, B - r0);
  float s = 0.f;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * mt + 4 * (lane >> 4) + r;
      const float z = acc[mt][r] + bias;
      acc[mt][r] = z;
      if (row < cnt && cv) Z[(long)(r0 + row) * N + n] = z;
      s += row < cnt ? z : 0.f;
    }
  if (L.bn == 1 || (L.bn == 2 && train)) {
    const float mean = colsum4(s) / (float)cnt;
    float m2 = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * mt + 4 * (lane >> 4) + r;
        const float d = acc[mt][r] - mean;
        m2 += row < cnt ? d * d : 0.f;
      }
    m2 = colsum4(m2);
    if (lane < 16 && cv) reinterpret_cast<F2*>(ws + L.part_off)[(long)rb * N + n] = F2{mean, m2};
  }
}

// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(LOSS_NT)
headb_loss_kernel(BArgs a, const long long* __restrict__ y, float* __restrict__ out,
                  float* __restrict__ loss, long long* __restrict__ pred,
                  unsigned long long* __restrict__ rng, char* __restrict__ ws) {
  __shared__ float red[LOSS_NT / 64][17];
  const BLayer& L = a.L[a.nl - 1];
  const int C = L.out, B = a.B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* Z = reinterpret_cast<const float*>(ws + L.z_off);
  float* g = reinterpret_cast<float*>(ws + a.g_off);
  const bool train = a.train != 0;
  // the seed and the BatchNorm step counters are read here, not after the reductions: the tail
  // of this one-workgroup launch was a chain of dependent global round trips
  unsigned long long seed = 0ull;
  long long nbt[BMAXL];
  if (tid == 0 && train) {
    seed = rng ? *rng : 0ull;
#pragma unroll
    for (int l = 0; l < BMAXL; ++l)
      nbt[l] = (l < a.nl && a.L[l].bn == 2 && a.L[l].nbt) ? *a.L[l].nbt : 0;
  }
  float ls = 0.f;
  float gs[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) gs[c] = 0.f;
  for (int m = tid; m < B; m += LOSS_NT) {
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = c < C ? Z[(long)m * C + c] : 0.f;
    float mx = v[0];
    int am = 0;
#pragma unroll
    for (int c = 1; c < 16; ++c)
      if (c < C && v[c] > mx) {
        mx = v[c];
        am = c;
      }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) se += c < C ? expf(v[c] - mx) : 0.f;
    const float lse = mx + logf(se);
    long long yc = y[m];
    yc = yc < 0 ? 0 : (yc >= C ? C - 1 : yc);
    float vy = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      if (c >= C) continue;
      const float lp = v[c] - lse;
      const float p = expf(lp);
      out[(long)m * C + c] = a.log_out ? lp : p;
      const float gv = p - (c == yc ? 1.f : 0.f);
      if (train) g[(long)m * C + c] = gv;
      gs[c] += gv;
      vy = c == yc ? v[c] : vy;
    }
    ls += lse - vy;
    pred[m] = am;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) ls += __shfl_xor(ls, off);
  // (only the C real classes: a wave-wide sum is 6 cross-lane steps, 96 for all 16 slots)
#pragma unroll
  for (int c = 0; c < 16; ++c)
    if (c < C) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) gs[c] += __shfl_xor(gs[c], off);
    }
  if (lane == 0) {
    red[wid][16] = ls;
#pragma unroll
    for (int c = 0; c < 16; ++c) red[wid][c] = c < C ? gs[c] : 0.f;
  }
  __syncthreads();
  if (tid < 17) {
    float t = 0.f;
    for (int w = 0; w < LOSS_NT / 64; ++w) t += red[w][tid];
    if (tid == 16) {
      *loss = t / (float)B;
    } else if (train) {
      reinterpret_cast<float*>(ws + a.gs_off)[tid] = t;
    }
  }
  if (tid == 0 && train) {
    *reinterpret_cast<unsigned long long*>(ws) = seed;
    if (rng) *rng = seed + 1ull;
#pragma unroll
    for (int l = 0; l < BMAXL; ++l)
      if (l < a.nl && a.L[l].bn == 2 && a.L[l].nbt) *a.L[l].nbt = nbt[l] + 1;
  }
}

// ---------------------------------------------------------------------------------------------
// BatchNorm backward of layer l: dZ_l from dy_l and the merged column sums.
__global__ void __launch_bounds__(BNT)
headb_bn_bwd_kernel(BArgs a, int l, char* __restrict__ ws, RedJob rj) {
  if (rj.rl >= 0 && (int)blockIdx.x >= rj.r0) {
    dw_reduce_body(a, rj.rl, ws, rj.rs, blockIdx.x - rj.r0, gridDim.x - rj.r0);
    return;
  }
  extern __shared__ float cf[];  // [4][N]: gamma rstd, mean, rstd, (sum dy) / B | (sum dy xhat) / B
  const BLayer& L = a.L[l];
  const int N = L.out, B = a.B, tid = threadIdx.x;
  const F2* part2 = reinterpret_cast<const F2*>(ws + L.part2_off);
  const F2* stat = reinterpret_cast<const F2*>(ws + L.stat_off);
  float* cA = cf;
  float* cm = cf + N;
  float* cr = cf + 2 * N;
  F2* cs = reinterpret_cast<F2*>(cf + 3 * N);
  for (int c = tid; c < N; c += BNT) {
    // everything this column needs is loaded before the partial sums are merged
    const F2 st = stat[c];
    const float gmc = L.gamma[c];
    const float gg0 = blockIdx.x == 0 ? L.ggamma[c] : 0.f;
    const float gb0 = blockIdx.x == 0 ? L.gbeta[c] : 0.f;
    float s1 = 0.f, s2 = 0.f;
    for (int r8 = 0; r8 < a.nrb; r8 += 16) {  // 16 partial loads in flight, summed in order
      F2 qs[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) qs[i] = part2[(long)min(r8 + i, a.nrb - 1) * N + c];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (r8 + i < a.nrb) {
          s1 += qs[i].x;
          s2 += qs[i].y;
        }
    }
    if (blockIdx.x == 0) {
      L.ggamma[c] = gg0 + s2;
      L.gbeta[c] = gb0 + s1;
    }
    cA[c] = gmc * st.y;
    cm[c] = st.x;
    cr[c] = st.y;
    cs[c] = F2{s1 / (float)B, s2 / (float)B};
  }
  __syncthreads();
  const int r0 = blockIdx.x * RB, cnt = min(RB, B - r0);
  const float* dy = reinterpret_cast<const float*>(ws + L.dy_off);
  const float* Z = reinterpret_cast<const float*>(ws + L.z_off);
  bf16* img = reinterpret_cast<bf16*>(ws + L.dz_off);
  float* dbp = reinterpret_cast<float*>(ws + L.dbp_off);
  for (int c = tid; c < L.S_z; c += BNT) {
    const bool cv = c < N;
    const int cc = cv ? c : 0;
    const float A = cA[cc], m = cm[cc], rs = cr[cc];
    const F2 q = cs[cc];
    float sum = 0.f;
    // rows in groups of 32 with every load of a group issued before its first use: a thread
    // walks 64 rows of one column, and one dependent L2 round trip per row made this launch
    // ~30 us at B = 2048 (12.7 us at groups of 16)
    constexpr int RG = 32;
    for (int rg = 0; rg < cnt; rg += RG) {
      float zv[RG], dv[RG];
#pragma unroll
      for (int i = 0; i < RG; ++i) {
        const long o = (long)(r0 + min(rg + i, cnt - 1)) * N + cc;
        zv[i] = Z[o];
        dv[i] = dy[o];
      }
#pragma unroll
      for (int i = 0; i < RG; ++i) {
        if (rg + i < cnt) {
          const float xh = (zv[i] - m) * rs;
          const float dz = cv ? A * (dv[i] - q.x - xh * q.y) : 0.f;
          img[(long)(r0 + rg + i) * L.S_z + c] = (bf16)dz;
          sum += dz;
        }
      }
    }
    if (cv) dbp[(long)blockIdx.x * N + c] = sum;
  }
}

// ---------------------------------------------------------------------------------------------
template <bool LAST, bool VW>
__global__ void __launch_bounds__(BNT)
headb_bwd_kernel(BArgs a, int l, char* __restrict__ ws, const float* __restrict__ dloss,
                 float* __restrict__ dx, long lddx, int nA, int RS, RedJob rj) {
  if (rj.rl >= 0 && (int)blockIdx.x >= rj.r0) {
    dw_reduce_body(a, rj.rl, ws, rj.rs, blockIdx.x - rj.r0, gridDim.x - rj.r0);
    return;
  }
  __shared__ __attribute__((aligned(16))) bf16 T0[RB * LS];
  __shared__ __attribute__((aligned(16))) bf16 T1[RB * LS];
  const BLayer& L = a.L[l];
  const int K = L.in, N = L.out, B = a.B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nkb = (K + TB - 1) / TB;
  const float gscale = LAST ? *dloss / (float)B : 1.f;
  const float* g = reinterpret_cast<const float*>(ws + a.g_off);
  bf16* dz = reinterpret_cast<bf16*>(ws + L.dz_off);
  const int sr = tid >> 4, sq = (tid & 15) * 4;
  const bool dA_job = (int)blockIdx.x < nA;
  const int job = dA_job ? blockIdx.x : blockIdx.x - nA;
  const int kb = job % nkb;
  const int k0 = kb * TB;

  // rows [r0, r0 + RB) x columns [c0, c0 + TB) of dZ_l (bf16, zero outside): loaded into
  // registers one chunk ahead of the MFMAs (load_dz), written to T0 when the chunk is staged
  // (put_dz).  Both loops below were a chain of one global round trip per 64-wide chunk.
  struct DzRegs {
    float f[4][4];
    bf16x4 h[4];
  };
  auto load_dz = [&](int r0, int c0, DzRegs& d) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int gr = r0 + sr + 16 * p, c = c0 + sq;
      if constexpr (LAST) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = gr < B && c + e < N;
          const float q = g[ok ? (long)gr * N + c + e : 0];
          d.f[p][e] = ok ? q * gscale : 0.f;
        }
      } else {
        const bool ok = gr < B && c < L.S_z;
        const bf16x4 q = *reinterpret_cast<const bf16x4*>(dz + (ok ? (long)gr * L.S_z + c : 0));
        const bf16x4 zero = {};
        d.h[p] = ok ? q : zero;
      }
    }
  };
  auto put_dz = [&](int r0, int c0, const DzRegs& d, bool write_img) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = sr + 16 * p, gr = r0 + row, c = c0 + sq;
      bf16x4 b4;
      if constexpr (LAST) {
        b4 = to_bf4(d.f[p]);
        if (write_img && gr < B && c < L.S_z) *reinterpret_cast<bf16x4*>(dz + (long)gr * L.S_z + c) = b4;
      } else {
        b4 = d.h[p];
      }
      *reinterpret_cast<bf16x4*>(T0 + row * LS + sq) = b4;
    }
  };

  if (dA_job) {
    const int rb = job / nkb, r0 = rb * RB;
    f32x4 acc[4] = {};
    DzRegs dr;
    float wv[4][4];
    auto load_w = [&](int nc) {
#pragma unroll
      for (int p = 0; p < 4; ++p) load4<VW>(L.W, K, nc + sr + 16 * p, k0 + sq, N, K, wv[p]);
    };
    load_dz(r0, 0, dr);
    load_w(0);
    for (int nc = 0; nc < N; nc += TB) {
      put_dz(r0, nc, dr, LAST && kb == 0);
#pragma unroll
      for (int p = 0; p < 4; ++p) {  // T1[k][n] = W[nc + n][k0 + k]
        const int nl_ = sr + 16 * p;
#pragma unroll
        for (int e = 0; e < 4; ++e) T1[(sq + e) * LS + nl_] = (bf16)wv[p][e];
      }
      __syncthreads();
      if (nc + TB < N) {  // (a load left in flight at the end holds the epilogue's registers)
        load_dz(r0, nc + TB, dr);
        load_w(nc + TB);
      }
#pragma unroll
      for (int ks = 0; ks < TB; ks += 32) {
        const int kk = ks + 8 * (lane >> 4);
        const bf16x8 bw = *reinterpret_cast<const bf16x8*>(T1 + (16 * wid + (lane & 15)) * LS + kk);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const bf16x8 av = *reinterpret_cast<const bf16x8*>(T0 + (16 * mt + (lane & 15)) * LS + kk);
          acc[mt] = mfma16(av, bw, acc[mt]);
        }
      }
      __syncthreads();
    }
    const int k = k0 + 16 * wid + (lane & 15);
    const bool kv = k < K;
    const float pdrop = L.drop;
    const float inv = pdrop > 0.f ? 1.f / (1.f - pdrop) : 1.f;
    const uint64_t seed = pdrop > 0.f ? *reinterpret_cast<const unsigned long long*>(ws) : 0ull;
    if (l == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gr = r0 + 16 * mt + 4 * (lane >> 4) + r;
          float v = acc[mt][r];
          if (pdrop > 0.f && v != 0.f) v = hkeep(seed, 0, gr, k, K, pdrop) ? v * inv : 0.f;
          if (gr < B && kv) dx[(long)gr * lddx + k] = v;
        }
      return;
    }
    const BLayer& P = a.L[l - 1];  // P.out == K
    float mean = 0.f, rstd = 1.f, s = 1.f, t = 0.f;
    if (P.bn && kv) {
      const F2 st = reinterpret_cast<const F2*>(ws + P.stat_off)[k];
      mean = st.x;
      rstd = st.y;
      s = P.gamma[k] * rstd;
      t = P.beta[k] - mean * s;
    }
    const float* Zp = reinterpret_cast<const float*>(ws + P.z_off);
    float* dyp = reinterpret_cast<float*>(ws + P.dy_off);
    bf16* dzp = reinterpret_cast<bf16*>(ws + P.dz_off);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = r0 + 16 * mt + 4 * (lane >> 4) + r;
        const bool ok = gr < B && kv;
        float v = acc[mt][r];
        if (pdrop > 0.f && v != 0.f) v = hkeep(seed, l, gr, k, K, pdrop) ? v * inv : 0.f;
        const float z = Zp[ok ? (long)gr * K + k : 0];
        if (P.relu && s * z + t <= 0.f) v = 0.f;
        v = ok ? v : 0.f;
        if (P.bn) {
          if (ok) dyp[(long)gr * K + k] = v;
          s2 += v * (z - mean) * rstd;
        } else if (gr < B && k < P.S_z) {
          dzp[(long)gr * P.S_z + k] = (bf16)v;
        }
        s1 += v;
      }
    s1 = colsum4(s1);
    if (P.bn) {
      s2 = colsum4(s2);
      if (lane < 16 && kv) reinterpret_cast<F2*>(ws + P.part2_off)[(long)rb * K + k] = F2{s1, s2};
    } else if (lane < 16 && kv) {
      reinterpret_cast<float*>(ws + P.dbp_off)[(long)rb * K + k] = s1;
    }
    return;
  }

  // dW job (tile, split): sum over split `sp`'s rows of dZ_l[b][n] A_l[b][k] for the 64 x 64
  // tile n0.., k0..; one split accumulates into gW directly, several write partials that
  // headb_dw_reduce adds in split order
  const int tile = job / RS, sp = job - tile * RS;
  const int kbw = tile % nkb, k0w = kbw * TB;
  const int n0 = (tile / nkb) * TB;
  const int rb0 = sp * a.nrb / RS, rb1 = (sp + 1) * a.nrb / RS;
  const bf16* aimg = reinterpret_cast<const bf16*>(ws + L.a_off);
  f32x4 acc[4] = {};
  DzRegs dr;
  bf16x4 av4[4];
  auto load_a = [&](int r0) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int gr = r0 + sr + 16 * p, c = k0w + sq;
      const bool ok = gr < B && c < L.S_a;
      const bf16x4 q = *reinterpret_cast<const bf16x4*>(aimg + (ok ? (long)gr * L.S_a + c : 0));
      const bf16x4 zero = {};
      av4[p] = ok ? q : zero;
    }
  };
  load_dz(rb0 * RB, n0, dr);
  load_a(rb0 * RB);
  for (int r0 = rb0 * RB; r0 < rb1 * RB; r0 += RB) {
    put_dz(r0, n0, dr, false);
#pragma unroll
    for (int p = 0; p < 4; ++p) *reinterpret_cast<bf16x4*>(T1 + (sr + 16 * p) * LS + sq) = av4[p];
    __syncthreads();
    if (r0 + RB < rb1 * RB) {
      load_dz(r0 + RB, n0, dr);
      load_a(r0 + RB);
    }
#pragma unroll
    for (int ks = 0; ks < RB; ks += 32) {
      const bf16x8 bf = tr_frag(T1, LS, 16 * wid, ks, lane);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = mfma16(tr_frag(T0, LS, 16 * mt, ks, lane), bf, acc[mt]);
    }
    __syncthreads();
  }
  const int k = k0w + 16 * wid + (lane & 15);
  float* part = reinterpret_cast<float*>(ws + L.dwp_off) + (long)sp * N * K;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 16 * mt + 4 * (lane >> 4) + r;
      if (n < N && k < K) {
        if (RS == 1) L.gW[(long)n * K + k] += acc[mt][r];
        else part[(long)n * K + k] = acc[mt][r];
      }
    }
  if (sp == 0 && kbw == 0 && L.gb && tid < TB && n0 + tid < N) {
    const int n = n0 + tid;
    float db;
    if constexpr (LAST) {
      db = reinterpret_cast<const float*>(ws + a.gs_off)[n] * gscale;
    } else {
      const float* dbp = reinterpret_cast<const float*>(ws + L.dbp_off);
      db = 0.f;
      for (int r8 = 0; r8 < a.nrb; r8 += 16) {  // 16 loads in flight, summed in order
        float qs[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) qs[i] = dbp[(long)min(r8 + i, a.nrb - 1) * N + n];
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (r8 + i < a.nrb) db += qs[i];
      }
    }
    L.gb[n] += db;
  }
}

// the first layer's reduce (nothing of the head runs after it)
__global__ void __launch_bounds__(256)
headb_dw_reduce_kernel(BArgs a, int l, const char* __restrict__ ws, int RS) {
  dw_reduce_body(a, l, ws, RS, blockIdx.x, gridDim.x);
}

struct BPlan {
  BArgs a;
  long ws_bytes;
};

static long al256(long v) { return (v + 255) & ~255L; }

static bool bplan(int nl, const int* dims, const int* flags, const float* drops, const float* bnp,
                  void* const* ptrs, int B, BPlan& p) {
  if (nl < 1 || nl > BMAXL || B < 1) return false;
  if (dims[nl] < 1 || dims[nl] > 16) return false;
  if (flags[nl - 1] != 0) return false;  // the logits come straight out of a Linear
  BArgs& a = p.a;
  a.nl = nl;
  a.B = B;
  a.nrb = (B + RB - 1) / RB;
  long off = 256;  // header: dropout seed
  for (int l = 0; l < nl; ++l) {
    BLayer& L = a.L[l];
    L.in = dims[l];
    L.out = dims[l + 1];
    if (L.in < 1 || L.out < 1 || L.in > MAXD || L.out > MAXD) return false;
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
    L.S_a = rup8(L.in);
    L.S_z = rup8(L.out);
    const long Bl = B, R = a.nrb, N = L.out;
    L.a_off = off;
    off = al256(off + 2 * Bl * L.S_a);
    L.z_off = off;
    off = al256(off + 4 * Bl * N);
    L.part_off = L.stat_off = L.dy_off = L.part2_off = 0;
    if (L.bn) {
      L.part_off = off;
      off = al256(off + 8 * R * N);
      L.stat_off = off;
      off = al256(off + 8 * N);
      L.dy_off = off;
      off = al256(off + 4 * Bl * N);
      L.part2_off = off;
      off = al256(off + 8 * R * N);
    }
    L.dz_off = off;
    off = al256(off + 2 * Bl * L.S_z);
    L.dbp_off = off;
    off = al256(off + 4 * R * N);
  }
  a.g_off = off;
  off = al256(off + 4L * B * dims[nl]);
  a.gs_off = off;
  off = al256(off + 4L * 16);
  for (int l = 0; l < nl; ++l) {
    BLayer& L = a.L[l];
    const int nkb = (L.in + TB - 1) / TB, nW = ((L.out + TB - 1) / TB) * nkb;
    const int rs = dw_splits(nW, a.nrb);
    L.dwp_off = off;
    if (rs > 1) off = al256(off + 4L * rs * L.out * L.in);
  }
  p.ws_bytes = off;
  return true;
}

template <typename Kern>
static void launch_fwd_layer(Kern k, const BPlan& p, int l, const float* x, long ldx,
                             unsigned long long* rng, void* ws, hipStream_t st) {
  const BLayer& L = p.a.L[l];
  const dim3 grid(p.a.nrb, (L.out + TB - 1) / TB);
  const size_t lds = 2 * (RB + TB) * LS + (l > 0 ? 8 * L.in : 0);
  hipLaunchKernelGGL(k, grid, dim3(BNT), lds, st, p.a, l, x, ldx, rng, (char*)ws);
}

}  // namespace

int headb_layout(int nl, const int* dims, const int* flags, int B, long* out) {
  BPlan p;
  if (!bplan(nl, dims, flags, nullptr, nullptr, nullptr, B, p)) return DN_UNSUPPORTED;
  out[0] = p.ws_bytes;
  for (int l = 0; l < nl; ++l) {
    out[1 + 4 * l] = p.a.L[l].a_off;
    out[2 + 4 * l] = p.a.L[l].S_a;
    out[3 + 4 * l] = p.a.L[l].dz_off;
    out[4 + 4 * l] = p.a.L[l].S_z;
  }
  return DN_OK;
}

int headb_fwd(int nl, const int* dims, const int* flags, const float* drops, const float* bnp,
              void* const* ptrs, const float* x, long ldx, int B, const long long* y, float* out,
              float* loss, long long* pred, unsigned long long* rng, void* ws, int train,
              int log_out, hipStream_t st) {
  BPlan p;
  if (!bplan(nl, dims, flags, drops, bnp, ptrs, B, p)) return DN_UNSUPPORTED;
  p.a.train = train;
  p.a.log_out = log_out;
  for (int l = 0; l < nl; ++l) {
    const int K = p.a.L[l].in;
    const bool vw = K % 4 == 0;
    const bool vx = l == 0 ? (K % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0) : vw;
    if (vx && vw) launch_fwd_layer(headb_fwd_kernel<true, true>, p, l, x, ldx, rng, ws, st);
    else if (vw) launch_fwd_layer(headb_fwd_kernel<false, true>, p, l, x, ldx, rng, ws, st);
    else launch_fwd_layer(headb_fwd_kernel<false, false>, p, l, x, ldx, rng, ws, st);
  }
  hipLaunchKernelGGL(headb_loss_kernel, dim3(1), dim3(LOSS_NT), 0, st, p.a, y, out, loss, pred,
                     rng, (char*)ws);
  return dn_launch_status();
}

int headb_bwd(int nl, const int* dims, const int* flags, const float* drops, const float* bnp,
              void* const* ptrs, int B, void* ws, const float* dloss, float* dx, long lddx,
              hipStream_t st) {
  BPlan p;
  if (!bplan(nl, dims, flags, drops, bnp, ptrs, B, p)) return DN_UNSUPPORTED;
  for (int l = 0; l < nl; ++l) {
    const BLayer& L = p.a.L[l];
    if (!L.gW || (L.b && !L.gb) || (L.bn && (!L.ggamma || !L.gbeta))) return DN_BAD_SHAPE;
  }
  p.a.train = 1;
  p.a.log_out = 0;
  RedJob pend{-1, 0, 0};  // the previous layer's reduce, carried by the next launch
  long pend_blocks = 0;
  auto take = [&](int r0, unsigned& grid) {
    RedJob r = pend;
    if (r.rl >= 0) {
      r.r0 = r0;
      grid += (unsigned)pend_blocks;
    }
    pend = RedJob{-1, 0, 0};
    return r;
  };
  for (int l = nl - 1; l >= 0; --l) {
    const BLayer& L = p.a.L[l];
    if (l < nl - 1 && L.bn) {
      unsigned g = (unsigned)p.a.nrb;
      const RedJob rj = take(p.a.nrb, g);
      hipLaunchKernelGGL(headb_bn_bwd_kernel, dim3(g), dim3(BNT), 20 * L.out, st, p.a, l,
                         (char*)ws, rj);
    }
    const int nkb = (L.in + TB - 1) / TB;
    const int nA = (l > 0 || dx) ? p.a.nrb * nkb : 0;
    const int nWt = ((L.out + TB - 1) / TB) * nkb;
    const int RS = dw_splits(nWt, p.a.nrb);
    const int nW = nWt * RS;
    const bool vw = L.in % 4 == 0;
    unsigned g = (unsigned)(nA + nW);
    const RedJob rj = take(nA + nW, g);
    const dim3 grid(g);
    if (l == nl - 1) {
      if (vw) hipLaunchKernelGGL((headb_bwd_kernel<true, true>), grid, dim3(BNT), 0, st, p.a, l, (char*)ws, dloss, dx, lddx, nA, RS, rj);
      else hipLaunchKernelGGL((headb_bwd_kernel<true, false>), grid, dim3(BNT), 0, st, p.a, l, (char*)ws, dloss, dx, lddx, nA, RS, rj);
    } else {
      if (vw) hipLaunchKernelGGL((headb_bwd_kernel<false, true>), grid, dim3(BNT), 0, st, p.a, l, (char*)ws, dloss, dx, lddx, nA, RS, rj);
      else hipLaunchKernelGGL((headb_bwd_kernel<false, false>), grid, dim3(BNT), 0, st, p.a, l, (char*)ws, dloss, dx, lddx, nA, RS, rj);
    }
    if (RS > 1) {
      const long NK = (long)L.out * L.in;
      long blocks = (NK + 255) / 256;
      if (blocks > 1024) blocks = 1024;
      pend = RedJob{l, RS, 0};
      pend_blocks = blocks;
    }
  }
  if (pend.rl >= 0)
    hipLaunchKernelGGL(headb_dw_reduce_kernel, dim3((unsigned)pend_blocks), dim3(BNT), 0, st, p.a,
                       pend.rl, (const char*)ws, pend.rs);
  return dn_launch_status();
}
