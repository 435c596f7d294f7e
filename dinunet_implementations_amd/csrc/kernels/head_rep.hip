// Fused head training step with a REPLICATED forward (gfx950, batch <= 32): forward, loss, the
// output-gradient chain, every head parameter gradient and d input of the ICA classifier
// (reference comps/icalstm/models.py:95-103 + comps/icalstm/__init__.py:59-63) in ONE launch with
// no cross-workgroup hand-off.
//
// The round-4 one-launch head (head_step.hip, folded into this kernel in round 6) split layer 0 by
// output columns over 16 workgroups and ran the narrow layers, the loss and the output-gradient
// chain in one tail workgroup, handing A1 -> tail -> dZ1 -> columns -> dZ0 -> dX between them
// through write-through stores and polled counters: three hops of ~1.2 us plus a single-workgroup
// chain, 33 us of the 311 us B=32 step (profiles/r4_graph_step_timeline_final.txt).  The whole
// head is ~10 M MAC at B = 32 -- ~5000 MFMA cycles on ONE CU -- so here EVERY workgroup computes
// the complete forward and the output-gradient chain down to dZ0 itself (one 16-wave workgroup:
// layer 0 one output tile per wave with its weight rows in registers, the narrow layers' weights
// as LDS images), and the workgroups split only what is written: the dW tiles of every layer (one
// 16 x 16 tile = one MFMA over the batch, read-modify-write into .grad), the dX column tiles (dZ0
// W0, K split in the three-launch head's groups so the sums are bitwise the same), and workgroup 0
// writes the outputs, the loss, the BatchNorm running statistics and the vector gradients.
// Nothing waits on another workgroup (no co-residency requirement, no spin limit): the last
// workgroup to finish (one agent-scope counter) advances the dropout seed for the next launch,
// after every workgroup has read it.
//
// The weights come as bf16 images: the ones the fused Adam keeps current (optim.hip
// adam_pack_kernel, ops.lstm.PersistentPack extra casts), or -- steps without that pack -- the
// head's own images, cast from the fp32 weights by one launch right before
// (ops.head.HeadSpec.own_images, elementwise.hip dn_cast_bf16_group).  The kernel is VALU-issue
// bound (16 waves on 4 SIMDs), and a first version that converted fp32 weights with per-element
// masks and per-lane layer decodes ran ~2850 VALU instructions per wave, 47 us.  Here every
// decode is wave-uniform and every operand copy is a whole 16-byte chunk.
//
// Numerics: the rounding points and reduction orders of mlp_head.hip (bf16 MFMA operands, fp32
// accumulation, layer-0 K in four interleaved k-step groups summed in group order, the same
// counter-hash dropout masks), so the one-launch and three-launch heads agree bitwise.
#include "head_common.h"
#include <stdlib.h>

namespace {

constexpr int RNW = 16;           // waves per workgroup
constexpr int RNT = RNW * 64;
constexpr int RMT = 2;            // 32 batch rows = two 16-row MFMA tiles
constexpr int RMP = 32;
constexpr int RMAXL = 6;
constexpr int RKS0 = 12;          // layer-0 k-steps of 32: layer-0 inputs <= 384
constexpr int RDXT = 2;           // dX 16-column tiles per workgroup
constexpr int RDWJ = 4;           // dW 16 x 16 tiles per wave
constexpr int RWU = 3;            // rounds of wave jobs for the narrow weight images
constexpr int RPU = 3;            // rounds of wave jobs for the parameter vectors
constexpr int RWCS = 24;          // row stride of the dX weight-column image (16 + 8 pad)
constexpr int Y_DONE_REP = 192;   // control-block word of the done counter (own line)

typedef __attribute__((address_space(1))) unsigned gu32r;
// read-only tables the kernel never writes: constant address space, so wave-uniform reads are
// scalar loads (a global load would make every wave wait on vmcnt before its first use)
typedef const __attribute__((address_space(4))) int cint;

struct RLayer {
  const bf16* Wb;  // bf16 image [out][in] of the weight (kept current by the fused Adam)
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
  int in, out, Kp, Np;  // Kp = rup32(in), Np = rup32(out)
  int bn, relu;
  float drop, eps, momentum;
  int SW, SZ;              // image row strides (elements): input / W images Kp + 8, dZ image Np + 8
  int a_lds, w_lds, z_lds, x_lds, r_lds, p_lds;  // LDS byte offsets (see rep_plan)
  int tn, tk, dw0;         // dW tiles (out / 16, in / 16) and the layer's first global dW job
  int kcmag;               // ceil(65536 / (Kp / 8)): lane -> weight-image row without a divide
};

struct RepArgs {
  RLayer L[RMAXL];
  int nl, B, G, ndx, njobs;
  int t_logit, t_dlogit, t_y, t_red, t_wc;
  int log_out;
  // wave jobs of the prologue, decoded on the host (wave-uniform, no divides on the device):
  // weight-image chunks (l << 12 | 64-chunk block) and parameter vectors (l << 12 | field << 8 |
  // 64-column block); -1 = none
  short wjob[RWU * RNW];
  short pjob[RPU * RNW];
  // dW tiles per (workgroup, wave, slot): (l << 16 | n-tile << 8 | k-tile), -1 = none
  // (a device table filled once per geometry, dn_head_rep_jobs)
  const int* jtab;
};

__device__ __forceinline__ void rlds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ void warm_rep_kernargs() {
  constexpr int LINES = (int)((sizeof(RepArgs) + 128 + 63) / 64);
  typedef const __attribute__((address_space(4))) unsigned cu32;
  cu32* kp = (cu32*)__builtin_amdgcn_kernarg_segment_ptr();
  unsigned acc = 0;
#pragma unroll
  for (int i = 0; i < LINES; ++i) acc += kp[16 * i];
  asm volatile("" ::"s"(acc));
}

__global__ void __launch_bounds__(RNT)
head_rep_kernel(RepArgs a, const float* __restrict__ x, long ldx, const long long* __restrict__ y,
                float* __restrict__ out, float* __restrict__ loss, long long* __restrict__ pred,
                unsigned long long* __restrict__ rng, const float* __restrict__ dloss,
                float* __restrict__ dx, long lddx, unsigned* __restrict__ sync,
                unsigned long long* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  warm_rep_kernargs();
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
  const int g = blockIdx.x;
#define RSTAMP(i) do { if (stamps && g == 0 && tid == 0) stamps[(i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
  RSTAMP(0);
  const bool lead = g == 0;  // writes outputs, running statistics and the vector gradients
  const int B = a.B, nl = a.nl;
  const uint64_t seed = *rng;
  const float gs = *dloss;
  const RLayer& L0 = a.L[0];
  const RLayer& L1 = a.L[1];
  const int K0 = L0.in, N0 = L0.out, nks0 = L0.Kp / 32;
  bf16* img0 = reinterpret_cast<bf16*>(smem + L0.a_lds);
  const int q = lane >> 4, ln = lane & 15;

  // ---- 1. every global operand of the prologue in ONE round: input rows, narrow weight-image
  // chunks and parameter vectors (each wave job wave-uniform: one layer, one field), then the
  // layer-0 weight rows (needed only after the barrier; younger, so never waited for here) -------
  const long long yv = (tid < RMP && tid < B) ? y[tid] : 0ll;
  // input rows 2w, 2w + 1; lane -> 8 columns (K0 % 8 == 0: a chunk is all in range or all out)
  f32x4 xv[2][2];
  const int xk = 8 * lane;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int m = 2 * wid + u;
    const bool ok = m < B && xk < K0;
    const float* src = x + (ok ? (long)m * ldx + xk : 0);
    xv[u][0] = *reinterpret_cast<const f32x4*>(src);
    xv[u][1] = *reinterpret_cast<const f32x4*>(src + 4);
  }
  bf16x8 wv[RWU];
#pragma unroll
  for (int u = 0; u < RWU; ++u) {
    const int wd = a.wjob[wid + RNW * u];
    wv[u] = bf16x8{};
    if (wd >= 0) {
      const RLayer& L = a.L[wd >> 12];
      const int c = (wd & 0xfff) * 64 + lane, KC = L.Kp / 8;
      const int nn = (c * L.kcmag) >> 16, kk = 8 * (c - nn * KC);
      if (nn < L.out && kk < L.in)
        wv[u] = *reinterpret_cast<const bf16x8*>(L.Wb + (long)nn * L.in + kk);
    }
  }
  float pv[RPU];
#pragma unroll
  for (int u = 0; u < RPU; ++u) {
    const int pd = a.pjob[wid + RNW * u];
    pv[u] = 0.f;
    if (pd >= 0) {
      const RLayer& L = a.L[pd >> 12];
      const int f = (pd >> 8) & 15, i = (pd & 0xff) * 64 + lane;
      const float* src = f == 0 ? L.b : f == 1 ? L.gamma : f == 2 ? L.beta : f == 3 ? L.rmean
                       : f == 4 ? L.rvar : f == 5 ? (L.b ? L.gb : nullptr)
                       : f == 6 ? L.ggamma : L.gbeta;
      if ((f >= 1 && f <= 2) || f >= 6) src = L.bn ? src : nullptr;
      if (f == 3 || f == 4) src = L.bn == 2 ? src : nullptr;
      pv[u] = (src && i < L.out) ? src[i] : (f == 4 ? 1.f : 0.f);
    }
  }
  // the W0 columns of this workgroup's dX tiles: 16-B row chunks of the bf16 image (the lanes of
  // each row's two 8-column halves), straight into their LDS image
  bf16x8 wcv[RDXT];
#pragma unroll
  for (int i = 0; i < RDXT; ++i) {
    const int t = g + a.G * i, h = q & 1, nr = 16 * wid + ln;
    wcv[i] = bf16x8{};
    if (t < a.ndx && q < 2 && nr < N0 && 16 * t + 8 * h < K0)
      wcv[i] = *reinterpret_cast<const bf16x8*>(L0.Wb + (long)nr * K0 + 16 * t + 8 * h);
  }
  // layer-0 weight rows of this wave's output tile (bf16 image, one 16-B fragment per k-step):
  // k-step groups 0 / 1 now, groups 2 / 3 once the prologue's registers are free again
  const int n = 16 * wid + ln;           // this lane's layer-0 column (tile = wave)
  const bool t0v = wid < L0.Np / 16;     // does this wave own a layer-0 tile (zero columns too)
  const bool cv = n < N0;
  bf16x8 w0f[RKS0];
  auto load_w0 = [&](int g0) {
#pragma unroll
    for (int ks = 0; ks < RKS0; ++ks) {
      if ((ks & 2) != g0) continue;
      w0f[ks] = bf16x8{};
      if (t0v && ks < nks0 && cv && 32 * ks + 8 * q < K0)
        w0f[ks] = *reinterpret_cast<const bf16x8*>(L0.Wb + (long)n * K0 + 32 * ks + 8 * q);
    }
  };
  load_w0(0);
  RSTAMP(1);
  // ---- stores into LDS ----------------------------------------------------------------------
  if (tid < RMP)
    reinterpret_cast<int*>(smem + a.t_y)[tid] = (int)(yv < 0 ? -1 : (yv > 0x7fffffffll ? 0x7fffffff : yv));
  RSTAMP(10);
  {
    const float p0 = L0.drop;
    const float inv = p0 > 0.f ? 1.f / (1.f - p0) : 1.f;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = 2 * wid + u;
      if (xk < L0.Kp) {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float t = xv[u][e >> 2][e & 3];
          if (!(m < B && xk < K0)) t = 0.f;
          if (p0 > 0.f && t != 0.f) t = hkeep(seed, 0, m, xk + e, K0, p0) ? t * inv : 0.f;
          o[e] = (bf16)t;
        }
        *reinterpret_cast<bf16x8*>(img0 + m * L0.SW + xk) = o;
      }
    }
  }
  RSTAMP(11);
#pragma unroll
  for (int u = 0; u < RWU; ++u) {
    const int wd = a.wjob[wid + RNW * u];
    if (wd >= 0) {
      const RLayer& L = a.L[wd >> 12];
      const int c = (wd & 0xfff) * 64 + lane, KC = L.Kp / 8;
      const int nn = (c * L.kcmag) >> 16, kk = 8 * (c - nn * KC);
      if (nn < L.Np)
        *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(smem + L.w_lds) + nn * L.SW + kk) = wv[u];
    }
  }
  RSTAMP(12);
#pragma unroll
  for (int u = 0; u < RPU; ++u) {
    const int pd = a.pjob[wid + RNW * u];
    if (pd >= 0) {
      const RLayer& L = a.L[pd >> 12];
      const int f = (pd >> 8) & 15, i = (pd & 0xff) * 64 + lane;
      if (i < L.Np) reinterpret_cast<float*>(smem + L.p_lds)[f * L.Np + i] = pv[u];
    }
  }
#pragma unroll
  for (int i = 0; i < RDXT; ++i) {
    const int t = g + a.G * i, nr = 16 * wid + ln;
    if (t < a.ndx && q < 2 && nr < L0.Np)
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(smem + a.t_wc) + (i * L0.Np + nr) * RWCS +
                                 8 * q) = wcv[i];
  }
  RSTAMP(13);
  load_w0(2);
  rlds_barrier();
  RSTAMP(2);

  // ---- 2. layer 0: one output tile per wave; K in four interleaved k-step groups ------------
  const float p1 = L1.drop;
  const float inv1 = p1 > 0.f ? 1.f / (1.f - p1) : 1.f;
  float xh[RMT][4];
  float rstd = 0.f;
  unsigned relu_ok = 0xffu;  // bit 4 mt + r: post-ReLU output > 0
  if (t0v) {
    f32x4 acc[RMT], part[RMT];
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      f32x4 (&dst)[RMT] = grp == 0 ? acc : part;
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt) dst[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < RKS0 / 4; ++u) {
        const int ks = grp + 4 * u;
        if (ks < nks0) {
#pragma unroll
          for (int mt = 0; mt < RMT; ++mt) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(img0 + (16 * mt + ln) * L0.SW + 32 * ks + 8 * q);
            dst[mt] = mfma16(af, w0f[ks], dst[mt]);
          }
        }
      }
      if (grp > 0) {
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[mt][r] += part[mt][r];
      }
    }
    const float* pp = reinterpret_cast<const float*>(smem + L0.p_lds);
    const float bias = pp[n];
    float z[RMT][4];
#pragma unroll
    for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) z[mt][r] = acc[mt][r] + bias;
    if (L0.bn) {
      float s = 0.f;
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += (16 * mt + 4 * q + r < B) ? z[mt][r] : 0.f;
      const float mean = colsum4(s) / (float)B;
      float v = 0.f;
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = z[mt][r] - mean;
          v += (16 * mt + 4 * q + r < B) ? d * d : 0.f;
        }
      v = colsum4(v) / (float)B;
      rstd = rsqrtf(v + L0.eps);
      if (lead && L0.bn == 2 && lane < 16 && cv) {
        const float mo = L0.momentum;
        L0.rmean[n] = (1.f - mo) * pp[3 * L0.Np + n] + mo * mean;
        L0.rvar[n] = (1.f - mo) * pp[4 * L0.Np + n] + mo * v * ((float)B / (float)(B > 1 ? B - 1 : 1));
      }
      const float ga = pp[L0.Np + n], be = pp[2 * L0.Np + n];
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * mt + 4 * q + r;
          xh[mt][r] = (row < B && cv) ? (z[mt][r] - mean) * rstd : 0.f;
          z[mt][r] = ga * xh[mt][r] + be;
        }
    } else {
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) xh[mt][r] = 0.f;
    }
    bf16* a1 = reinterpret_cast<bf16*>(smem + L1.a_lds);
#pragma unroll
    for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * mt + 4 * q + r;
        float v = z[mt][r];
        if (L0.relu) {
          v = fmaxf(v, 0.f);
          if (!(v > 0.f)) relu_ok &= ~(1u << (4 * mt + r));
        }
        v = (row < B && cv) ? v : 0.f;
        if (p1 > 0.f && v != 0.f) v = hkeep(seed, 1, row, n, N0, p1) ? v * inv1 : 0.f;
        a1[row * L1.SW + n] = (bf16)v;
      }
  }

  rlds_barrier();  // A1
  RSTAMP(3);

  // ---- 4. forward of layers 1 .. nl-1 (one 16-column tile per wave) ----------------------------
  float* logit = reinterpret_cast<float*>(smem + a.t_logit);
  float* dlogit = reinterpret_cast<float*>(smem + a.t_dlogit);
  for (int l = 1; l < nl; ++l) {
    const RLayer& L = a.L[l];
    const bool last = l == nl - 1;
    const bf16* aimg = reinterpret_cast<const bf16*>(smem + L.a_lds);
    const bf16* wimg = reinterpret_cast<const bf16*>(smem + L.w_lds);
    const float* pp = reinterpret_cast<const float*>(smem + L.p_lds);
    const int ntiles = last ? 1 : L.Np / 16, nks = L.Kp / 32, N = L.out;
    const RLayer& Ln = a.L[last ? l : l + 1];
    bf16* nimg = reinterpret_cast<bf16*>(smem + Ln.a_lds);
    const float pn = last ? 0.f : Ln.drop;
    const float invn = pn > 0.f ? 1.f / (1.f - pn) : 1.f;
    for (int t = wid; t < ntiles; t += RNW) {
      const int nn = 16 * t + ln;
      const bool lv = nn < N;
      f32x4 acc[RMT];
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int ks = 0; ks < nks; ++ks) {
        const bf16x8 bq = *reinterpret_cast<const bf16x8*>(wimg + nn * L.SW + 32 * ks + 8 * q);
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(aimg + (16 * mt + ln) * L.SW + 32 * ks + 8 * q);
          acc[mt] = mfma16(af, bq, acc[mt]);
        }
      }
      float z[RMT][4];
      const float bias = pp[nn];
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) z[mt][r] = acc[mt][r] + bias;
      if (L.bn) {
        float s = 0.f;
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) s += (16 * mt + 4 * q + r < B) ? z[mt][r] : 0.f;
        const float mean = colsum4(s) / (float)B;
        float v = 0.f;
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float dd = z[mt][r] - mean;
            v += (16 * mt + 4 * q + r < B) ? dd * dd : 0.f;
          }
        v = colsum4(v) / (float)B;
        const float rs = rsqrtf(v + L.eps);
        if (lead && L.bn == 2 && lane < 16 && lv) {
          const float mo = L.momentum;
          L.rmean[nn] = (1.f - mo) * pp[3 * L.Np + nn] + mo * mean;
          L.rvar[nn] = (1.f - mo) * pp[4 * L.Np + nn] + mo * v * ((float)B / (float)(B > 1 ? B - 1 : 1));
        }
        float* xhat = reinterpret_cast<float*>(smem + L.x_lds);
        const float gg = pp[L.Np + nn], bb = pp[2 * L.Np + nn];
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + 4 * q + r;
            const float xv2 = (row < B && lv) ? (z[mt][r] - mean) * rs : 0.f;
            xhat[row * L.Np + nn] = xv2;
            z[mt][r] = gg * xv2 + bb;
          }
        if (lane < 16) reinterpret_cast<float*>(smem + L.r_lds)[nn] = lv ? rs : 0.f;
      }
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * mt + 4 * q + r;
          float v = z[mt][r];
          if (L.relu) v = fmaxf(v, 0.f);
          if (last) {
            logit[row * 16 + ln] = v;
          } else {
            v = (row < B && lv) ? v : 0.f;
            if (pn > 0.f && v != 0.f) v = hkeep(seed, l + 1, row, nn, N, pn) ? v * invn : 0.f;
            nimg[row * Ln.SW + nn] = (bf16)v;
          }
        }
    }
    rlds_barrier();
  }
  RSTAMP(4);

  // ---- 5. loss: softmax / log-softmax + CE / NLL, argmax (wave 0, lane = row) ---------------
  const RLayer& LL = a.L[nl - 1];
  const int C = LL.out;
  const int m = lane;
  const bool mv = m < B;
  const float* lr = logit + m * 16;
  float* dr = dlogit + m * 16;
  const int* ylds = reinterpret_cast<const int*>(smem + a.t_y);
  if (wid == 0) {
    // the row's logits in registers (one round of LDS reads, then register-only math: the
    // serial per-class loops of a lane-per-row loss would otherwise wait on LDS every step)
    float lg[16];
    {
      const f32x4* l4 = reinterpret_cast<const f32x4*>(logit + (m & (RMP - 1)) * 16);
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const f32x4 t = l4[j4];
#pragma unroll
        for (int e = 0; e < 4; ++e) lg[4 * j4 + e] = (mv && 4 * j4 + e < C) ? t[e] : 0.f;
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int cc = 0; cc < 16; ++cc)
      if (cc < C) mx = fmaxf(mx, lg[cc]);
    float se = 0.f;
#pragma unroll
    for (int cc = 0; cc < 16; ++cc)
      if (cc < C) se += expf(lg[cc] - mx);
    const float lse = mx + logf(se);
    int yc = mv ? ylds[m & (RMP - 1)] : 0;
    yc = yc < 0 ? 0 : (yc >= C ? C - 1 : yc);
    float pr[16], dv[16];
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) {
      pr[cc] = expf(lg[cc] - lse);
      dv[cc] = (mv && cc < C) ? (pr[cc] - (cc == yc ? 1.f : 0.f)) / (float)B : 0.f;
    }
    if (lane < RMP) {
      f32x4* d4 = reinterpret_cast<f32x4*>(dr);
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4)
        d4[j4] = f32x4{dv[4 * j4], dv[4 * j4 + 1], dv[4 * j4 + 2], dv[4 * j4 + 3]};
    }
    bf16* dz = reinterpret_cast<bf16*>(smem + LL.z_lds);
    bf16x8 z0, z1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      z0[j] = (bf16)(lane < 32 ? gs * dv[j] : 0.f);
      z1[j] = (bf16)(lane < 32 ? gs * dv[8 + j] : 0.f);
    }
    bf16* zr = dz + (lane & 31) * LL.SZ + (lane < 32 ? 0 : 16);
    *reinterpret_cast<bf16x8*>(zr) = z0;
    *reinterpret_cast<bf16x8*>(zr + 8) = z1;
    // outputs, the loss and the last layer's bias gradient (workgroup 0)
    if (lead) {
      float ly = 0.f;
      int am = 0;
      float amx = -INFINITY;
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) {
        if (cc < C) {
          if (lg[cc] > amx) { amx = lg[cc]; am = cc; }
          if (cc == yc) ly = lg[cc];
          if (mv) out[(long)m * C + cc] = a.log_out ? lg[cc] - lse : pr[cc];
        }
      }
      float ls = mv ? lse - ly : 0.f;
      if (mv) pred[m] = am;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) ls += __shfl_xor(ls, off);
      if (lane == 0) {
        *loss = ls / (float)B;
        for (int l = 0; l < nl; ++l)
          if (a.L[l].bn == 2 && a.L[l].nbt)
            __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(a.L[l].nbt), 1ull,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (LL.b) {
        // lane = class: the column of d logits summed over the rows in row order (all reads
        // issued at once; the same serial order as the three-launch head's per-class sum)
        __builtin_amdgcn_wave_barrier();
        if (lane < C) {
          float col[RMP];
#pragma unroll
          for (int mm = 0; mm < RMP; ++mm) col[mm] = dlogit[mm * 16 + lane];
          float v = 0.f;
#pragma unroll
          for (int mm = 0; mm < RMP; ++mm)
            if (mm < B) v += col[mm];
          const float* pb = reinterpret_cast<const float*>(smem + LL.p_lds) + 5 * LL.Np;
          LL.gb[lane] = pb[lane] + gs * v;
        }
      }
    }
  }
  rlds_barrier();
  RSTAMP(5);

  // ---- the old values of this wave's dW tiles: requested now, they land during 6.-7. --------
  float gold[RDWJ][4];
  {
    cint* jt = (cint*)a.jtab + (g * RNW + wid) * RDWJ;
#pragma unroll
    for (int qq = 0; qq < RDWJ; ++qq) {
      const int jd = jt[qq], l = jd >> 16, ta = (jd >> 8) & 0xff, tb = jd & 0xff;
      const bool ok = jd >= 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = 0.f;
        if (ok) {
          const RLayer& L = a.L[l];
          const int nr = 16 * ta + 4 * q + r, k = 16 * tb + ln;
          v = L.gW[(nr < L.out && k < L.in) ? (long)nr * L.in + k : 0];
        }
        gold[qq][r] = v;
      }
    }
  }
  // ---- 6. output-gradient chain dZ_l -> dZ_{l-1}, l = nl-1 .. 2 --------------------------------
  for (int l = nl - 1; l >= 2; --l) {
    const RLayer& L = a.L[l];
    const RLayer& P = a.L[l - 1];
    const bf16* wimg = reinterpret_cast<const bf16*>(smem + L.w_lds);
    const bf16* aimg = reinterpret_cast<const bf16*>(smem + L.a_lds);  // ReLU mask of P
    const bf16* dz = reinterpret_cast<const bf16*>(smem + L.z_lds);
    bf16* dzn = reinterpret_cast<bf16*>(smem + P.z_lds);
    const float* pq = reinterpret_cast<const float*>(smem + P.p_lds);
    const float* xhat = reinterpret_cast<const float*>(smem + P.x_lds);
    const float* rsl = reinterpret_cast<const float*>(smem + P.r_lds);
    const int K = L.in, ntl = L.Kp / 16, nns = L.Np / 32;
    const float inv = L.drop > 0.f ? 1.f / (1.f - L.drop) : 1.f;
    for (int t = wid; t < ntl; t += RNW) {
      const int kk = 16 * t + ln;
      const bool kv = kk < K;
      const int kc = kv ? kk : 0;
      float xhp[RMT][4], rsp = 0.f;
      if (P.bn) {
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) xhp[mt][r] = xhat[(16 * mt + 4 * q + r) * P.Np + kc];
        rsp = rsl[kc];
      }
      f32x4 acc[RMT];
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < nns; ++s) {
        const bf16x8 bq = tr_frag(wimg, L.SW, 16 * t, 32 * s, lane);
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(dz + (16 * mt + ln) * L.SZ + 32 * s + 8 * q);
          acc[mt] = mfma16(af, bq, acc[mt]);
        }
      }
      float d[RMT][4];
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * mt + 4 * q + r;
          float v = (row < B && kv) ? acc[mt][r] : 0.f;
          if (L.drop > 0.f && v != 0.f) v = hkeep(seed, l, row, kk, K, L.drop) ? v * inv : 0.f;
          if (P.relu && !((float)aimg[row * L.SW + kk] > 0.f)) v = 0.f;
          d[mt][r] = v;
        }
      if (P.bn) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s1 += d[mt][r];
            s2 += d[mt][r] * xhp[mt][r];
          }
        s1 = colsum4(s1);
        s2 = colsum4(s2);
        if (lead && lane < 16 && kv) {
          P.ggamma[kk] = pq[6 * P.Np + kk] + s2;
          P.gbeta[kk] = pq[7 * P.Np + kk] + s1;
        }
        const float gg = kv ? pq[P.Np + kk] : 0.f;
        const float m1 = s1 / (float)B, m2 = s2 / (float)B;
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + 4 * q + r;
            d[mt][r] = (row < B && kv) ? gg * rsp * (d[mt][r] - m1 - xhp[mt][r] * m2) : 0.f;
          }
      }
      if (P.b) {
        float sb = 0.f;
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) sb += d[mt][r];
        sb = colsum4(sb);
        if (lead && lane < 16 && kv) P.gb[kk] = pq[5 * P.Np + kk] + sb;
      }
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) dzn[(16 * mt + 4 * q + r) * P.SZ + kk] = (bf16)d[mt][r];
    }
    rlds_barrier();
  }
  RSTAMP(6);

  // ---- 7. dA0 = dZ1 W1 on this wave's layer-0 tile, ReLU / BatchNorm backward -> dZ0 ---------
  if (t0v) {
    const bf16* w1 = reinterpret_cast<const bf16*>(smem + L1.w_lds);
    const bf16* z1 = reinterpret_cast<const bf16*>(smem + L1.z_lds);
    const int n1s = L1.Np / 32;
    f32x4 da[RMT];
#pragma unroll
    for (int mt = 0; mt < RMT; ++mt) da[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < n1s; ++s) {
      const bf16x8 bq = tr_frag(w1, L1.SW, 16 * wid, 32 * s, lane);
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt) {
        const bf16x8 zf = *reinterpret_cast<const bf16x8*>(z1 + (16 * mt + ln) * L1.SZ + 32 * s + 8 * q);
        da[mt] = mfma16(zf, bq, da[mt]);
      }
    }
    const float* pp = reinterpret_cast<const float*>(smem + L0.p_lds);
    float d[RMT][4];
#pragma unroll
    for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * mt + 4 * q + r;
        float t = (row < B && cv) ? da[mt][r] : 0.f;
        if (p1 > 0.f && t != 0.f) t = hkeep(seed, 1, row, n, N0, p1) ? t * inv1 : 0.f;
        if (L0.relu && !((relu_ok >> (4 * mt + r)) & 1u)) t = 0.f;
        d[mt][r] = t;
      }
    if (L0.bn) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1 += d[mt][r];
          s2 += d[mt][r] * xh[mt][r];
        }
      s1 = colsum4(s1);
      s2 = colsum4(s2);
      if (lead && lane < 16 && cv) {
        L0.ggamma[n] = pp[6 * L0.Np + n] + s2;
        L0.gbeta[n] = pp[7 * L0.Np + n] + s1;
      }
      const float ga = cv ? pp[L0.Np + n] : 0.f;
      const float m1 = s1 / (float)B, m2 = s2 / (float)B;
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * mt + 4 * q + r;
          d[mt][r] = (row < B && cv) ? ga * rstd * (d[mt][r] - m1 - xh[mt][r] * m2) : 0.f;
        }
    }
    if (L0.b) {
      float sb = 0.f;
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) sb += d[mt][r];
      sb = colsum4(sb);
      if (lead && lane < 16 && cv) L0.gb[n] = pp[5 * L0.Np + n] + sb;
    }
    bf16* z0 = reinterpret_cast<bf16*>(smem + L0.z_lds);
#pragma unroll
    for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) z0[(16 * mt + 4 * q + r) * L0.SZ + n] = (bf16)d[mt][r];
  }
  rlds_barrier();  // dZ0
  RSTAMP(7);

  // ---- 8. this workgroup's share: the dW tiles of every layer, then its dX tiles ------------
  {
    cint* jt = (cint*)a.jtab + (g * RNW + wid) * RDWJ;
#pragma unroll
    for (int qq = 0; qq < RDWJ; ++qq) {
      const int jd = jt[qq], l = jd >> 16, ta = (jd >> 8) & 0xff, tb = jd & 0xff;
      if (jd < 0) continue;
      const RLayer& L = a.L[l];
      const bf16* zl = reinterpret_cast<const bf16*>(smem + L.z_lds);
      const bf16* al = reinterpret_cast<const bf16*>(smem + L.a_lds);
      f32x4 acc = mfma16(tr_frag(zl, L.SZ, 16 * ta, 0, lane), tr_frag(al, L.SW, 16 * tb, 0, lane),
                         f32x4{0.f, 0.f, 0.f, 0.f});
      const int k = 16 * tb + ln;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nr = 16 * ta + 4 * q + r;
        if (nr < L.out && k < L.in) L.gW[(long)nr * L.in + k] = gold[qq][r] + acc[r];
      }
    }
  }
  RSTAMP(8);
  if (dx) {
    const int dxi = wid >> 2, dxg = wid & 3;   // dX: tile slot of this workgroup, k-step group
    const int nns0 = L0.Np / 32;
    const int dxt = g + a.G * dxi;             // this wave's dX tile (global 16-column index)
    const bool dxw = dxi < RDXT && dxt < a.ndx;
    float* red = reinterpret_cast<float*>(smem + a.t_red);  // [RDXT][3][RMT][4][64]
    const bf16* z0 = reinterpret_cast<const bf16*>(smem + L0.z_lds);
    const bf16* wc = reinterpret_cast<const bf16*>(smem + a.t_wc) + (dxi < RDXT ? dxi : 0) * L0.Np * RWCS;
    f32x4 ax[RMT];
#pragma unroll
    for (int mt = 0; mt < RMT; ++mt) ax[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (dxw) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int s = dxg + 4 * j;
        if (s >= nns0) continue;
        const bf16x8 bq = tr_frag(wc, RWCS, 0, 32 * s, lane);
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt) {
          const bf16x8 zf = *reinterpret_cast<const bf16x8*>(z0 + (16 * mt + ln) * L0.SZ + 32 * s + 8 * q);
          ax[mt] = mfma16(zf, bq, ax[mt]);
        }
      }
      if (dxg > 0) {
#pragma unroll
        for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            red[(((dxi * 3 + dxg - 1) * RMT + mt) * 4 + r) * 64 + lane] = ax[mt][r];
      }
    }
    rlds_barrier();
    if (dxw && dxg == 0) {
      const float p0 = L0.drop;
      const float inv0 = p0 > 0.f ? 1.f / (1.f - p0) : 1.f;
      const int kx = 16 * dxt + ln;
#pragma unroll
      for (int mt = 0; mt < RMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = ax[mt][r];
#pragma unroll
          for (int w = 0; w < 3; ++w) v += red[(((dxi * 3 + w) * RMT + mt) * 4 + r) * 64 + lane];
          const int row = 16 * mt + 4 * q + r;
          if (p0 > 0.f && v != 0.f) v = hkeep(seed, 0, row, kx, K0, p0) ? v * inv0 : 0.f;
          if (row < B && kx < K0) dx[(long)row * lddx + kx] = v;
        }
    }
  }
  RSTAMP(9);
  // ---- 9. the last workgroup to finish advances the dropout seed (every workgroup read it) ----
  rlds_barrier();
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add((gu32r*)(sync + Y_DONE_REP), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (unsigned)a.G - 1u) {
      __hip_atomic_store((gu32r*)(sync + Y_DONE_REP), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *rng = seed + 1ull;
    }
  }
#undef RSTAMP
}

}  // namespace

namespace {

struct RPlan {
  RepArgs a;
  long lds;
};

static int al16r(int v) { return (v + 15) & ~15; }

// LDS layout and work split; false outside the kernel's envelope (the caller then runs
// the three-launch head of mlp_head.hip): batch <= 32, 2..6 layers, layer 0 <= 384 inputs and <= 256 outputs (one
// 16-column tile per wave), narrow layers <= 256 wide, every input width a multiple of 8, <= 16
// classes, everything in 160 KB of LDS, and a bf16 image of every weight.
static bool rep_plan(int nl, const int* dims, const int* flags, const float* drops,
                     const float* bnp, void* const* ptrs, void* const* wbf, int B, RPlan& p) {
  if (nl < 2 || nl > RMAXL || B < 1 || B > RMP) return false;
  if (dims[nl] < 1 || dims[nl] > 16) return false;
  RepArgs& a = p.a;
  a.nl = nl;
  a.B = B;
  int c = 0, jobs = 0, wj = 0, pj = 0;
  for (int i = 0; i < RWU * RNW; ++i) a.wjob[i] = -1;
  for (int i = 0; i < RPU * RNW; ++i) a.pjob[i] = -1;
  a.jtab = nullptr;
  for (int l = 0; l < nl; ++l) {
    RLayer& L = a.L[l];
    L.in = dims[l];
    L.out = dims[l + 1];
    if (L.in < 1 || L.out < 1 || L.in % 8) return false;
    L.Kp = rup32(L.in);
    L.Np = rup32(L.out);
    L.bn = flags[l] & 3;
    L.relu = (flags[l] >> 2) & 1;
    L.drop = drops ? drops[l] : 0.f;
    if (L.drop < 0.f || L.drop >= 1.f) return false;
    L.eps = bnp ? bnp[2 * l] : 1e-5f;
    L.momentum = bnp ? bnp[2 * l + 1] : 0.1f;
    static void* const none[11] = {};
    void* const* q = ptrs ? ptrs + 11 * l : none;
    L.Wb = wbf ? (const bf16*)wbf[l] : nullptr;
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
      if (!L.Wb || (((uintptr_t)L.Wb) & 15) || !L.gW || (L.b && !L.gb)) return false;
      if (L.bn && (!L.gamma || !L.beta || !L.ggamma || !L.gbeta)) return false;
      if (L.bn == 2 && (!L.rmean || !L.rvar)) return false;
    }
    if (l == 0 && (L.in > 32 * RKS0 || L.Np > 16 * RNW)) return false;
    if (l >= 1 && (L.in > 256 || L.Np > 256)) return false;
    L.SW = L.Kp + 8;
    L.SZ = L.Np + 8;
    L.tn = (L.out + 15) / 16;
    L.tk = (L.in + 15) / 16;
    L.dw0 = jobs;
    jobs += L.tn * L.tk;
    L.kcmag = (65536 + L.Kp / 8 - 1) / (L.Kp / 8);
    if (l >= 1) {
      for (int blk = 0; blk < (L.Np * (L.Kp / 8) + 63) / 64; ++blk, ++wj)
        if (wj < RWU * RNW) a.wjob[wj] = (short)(l << 12 | blk);
    }
    for (int f = 0; f < 8; ++f)
      for (int blk = 0; blk < (L.Np + 63) / 64; ++blk, ++pj)
        if (pj < RPU * RNW) a.pjob[pj] = (short)(l << 12 | f << 8 | blk);
    L.a_lds = c;
    c = al16r(c + 2 * RMP * L.SW);
    L.w_lds = 0;
    if (l >= 1) {
      L.w_lds = c;
      c = al16r(c + 2 * L.Np * L.SW);
    }
    L.z_lds = c;
    c = al16r(c + 2 * RMP * L.SZ);
    L.x_lds = L.r_lds = 0;
    if (l >= 1 && L.bn) {  // layer 0's BatchNorm state stays in the owning wave's registers
      L.x_lds = c;
      c = al16r(c + 4 * RMP * L.Np);
      L.r_lds = c;
      c = al16r(c + 4 * L.Np);
    }
    L.p_lds = c;
    c = al16r(c + 4 * 8 * L.Np);
  }
  a.t_logit = c;
  c = al16r(c + 4 * RMP * 16);
  a.t_dlogit = c;
  c = al16r(c + 4 * RMP * 16);
  a.t_y = c;
  c = al16r(c + 4 * RMP);
  a.t_red = c;
  c = al16r(c + 4 * RDXT * 3 * RMT * 4 * 64);
  // the W0 columns of the workgroup's dX tiles (written right after layer 0)
  a.t_wc = c;
  c = al16r(c + 2 * RDXT * a.L[0].Np * RWCS);
  p.lds = c;
  if (c > 160 * 1024) return false;
  a.ndx = (a.L[0].in + 15) / 16;
  a.njobs = jobs;
  if (wj > RWU * RNW || pj > RPU * RNW) return false;
  // workgroups: enough for <= RDXT dX tiles each and <= RDWJ dW tiles per wave, and at least 8
  // (the read-modify-write of the gradients is spread over that many CUs)
  int G = (a.ndx + RDXT - 1) / RDXT;
  const int gj = (jobs + RNW * RDWJ - 1) / (RNW * RDWJ);
  if (gj > G) G = gj;
  if (G < 8) G = 8;
  a.G = G;
  return true;
}

// the dW job table of a plan: entry (g, wave, slot) -> global job g*RNW + wave + slot*G*RNW
// (consecutive jobs on consecutive waves, then workgroups) decoded to (layer, n-tile, k-tile)
static void rep_fill_jobs(const RepArgs& a, int* out) {
  for (int g = 0; g < a.G; ++g)
    for (int w = 0; w < RNW; ++w)
      for (int s = 0; s < RDWJ; ++s) {
        const int j = g * RNW + w + s * a.G * RNW;
        int v = -1;
        if (j < a.njobs) {
          int l = 0;
          for (int i = 1; i < a.nl; ++i)
            if (j >= a.L[i].dw0) l = i;
          const int r = j - a.L[l].dw0, ta = r / a.L[l].tk;
          v = l << 16 | ta << 8 | (r - ta * a.L[l].tk);
        }
        out[(g * RNW + w) * RDWJ + s] = v;
      }
}

static bool g_rep_init = false;
static unsigned long long* g_rep_stamps = nullptr;

}  // namespace

// The whole training step of the head in one launch with a replicated forward (see the top of
// this file); the arguments of the three-launch head's entry points, plus `wbf`: one bf16 [out][in]
// weight image per layer (16-B aligned; ops.lstm.PersistentPack.bf16_of), and `jtab`: the dW job
// table of this geometry in device memory (dn_head_rep_jobs).  sync: the head's
// control block (dn_head_rep_sync_bytes(), zeroed before first use).  DN_UNSUPPORTED outside the
// envelope (rep_plan).
DN_API int dn_head_rep(int nl, const int* dims, const int* flags, const float* drops,
                       const float* bnp, void* const* ptrs, void* const* wbf, const int* jtab,
                       const float* x,
                       long ldx, int B, const long long* y, float* out, float* loss,
                       long long* pred, unsigned long long* rng, void* sync, int log_out,
                       const float* dloss, float* dx, long lddx, hipStream_t st) {
  RPlan p;
  if (!dloss || !sync || !rng || !wbf || !rep_plan(nl, dims, flags, drops, bnp, ptrs, wbf, B, p))
    return DN_UNSUPPORTED;
  if (!jtab) return DN_BAD_SHAPE;
  p.a.jtab = jtab;
  if ((((uintptr_t)x) & 15) || ldx % 4) return DN_UNSUPPORTED;
  if (!g_rep_init) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(head_rep_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    g_rep_init = true;
  }
  p.a.log_out = log_out;
  // probe knob (tools/head_rep_stamps.py): DN_HEAD_REP_G=k launches only k workgroups -- the
  // gradients of the others are then missing (timing of the replicated part only)
  if (const char* e = getenv("DN_HEAD_REP_G")) {
    const int k = atoi(e);
    if (k > 0 && k < p.a.G) p.a.G = k;
  }
  hipLaunchKernelGGL(head_rep_kernel, dim3(p.a.G), dim3(RNT), p.lds, st, p.a, x, ldx, y, out,
                     loss, pred, rng, dloss, dx, lddx, (unsigned*)sync, g_rep_stamps);
  return dn_launch_status();
}

// Phase stamps of workgroup 0 (s_memrealtime, 100 MHz) into p[0..15]; null turns them off
DN_API int dn_head_rep_set_stamps(void* p) {
  g_rep_stamps = (unsigned long long*)p;
  return DN_OK;
}

// The dW job table of this geometry (int32 entries) into host memory `out` of `cap` entries: returns
// the entry count (copy it to the device once and pass it as dn_head_rep's jtab), 0 outside the
// kernel's envelope, -1 when cap is too small.
DN_API int dn_head_rep_jobs(int nl, const int* dims, const int* flags, int B, int* out, int cap) {
  RPlan p;
  if (!rep_plan(nl, dims, flags, nullptr, nullptr, nullptr, nullptr, B, p)) return 0;
  const int n = p.a.G * RNW * RDWJ;
  if (!out || cap < n) return -1;
  rep_fill_jobs(p.a, out);
  return n;
}

// Bytes of the control block (zeroed once by the caller; word Y_DONE_REP on a line of its own)
DN_API long dn_head_rep_sync_bytes() { return 4L * (Y_DONE_REP + 64); }

// Does the replicated head take this geometry (1) or not (0)?
DN_API int dn_head_rep_supported(int nl, const int* dims, const int* flags, int B) {
  RPlan p;
  return rep_plan(nl, dims, flags, nullptr, nullptr, nullptr, nullptr, B, p) ? 1 : 0;
}
