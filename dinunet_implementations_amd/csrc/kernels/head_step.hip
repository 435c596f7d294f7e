// One-launch fused head training step for gfx950 (batch <= 32): forward, loss, the whole backward
// and every head parameter gradient of the ICA classifier (reference
// comps/icalstm/models.py:95-103 + comps/icalstm/__init__.py:59-63) or of the FreeSurfer MSANNet
// (comps/fs/models.py:4-31 + comps/fs/__init__.py:54-57) in ONE kernel, replacing the three
// launches of mlp_head.hip (fwd0 / fwd1+bwd1 / bwd0: 43.6 us of the B=32 ICA step, each phase a
// single-workgroup chain of global round trips).
//
// Work split (G0 = rup32(layer-0 outputs) / 16 "column" workgroups + 1 "tail" workgroup):
//   column wg c: layer 0 for its 16 output columns -- the input image, K split over its four
//       waves, the BatchNorm statistics of its columns (column-local: no cross-workgroup
//       reduction), ReLU, the layer-1 dropout -- and publishes its A1 slice.  After the tail
//       hands back dZ1 it runs dA1 = dZ1 W1[:, cols], the ReLU / BatchNorm backward of its
//       columns (state kept in registers since the forward), dW0[cols, :] from its LDS input
//       image, publishes its dZ0 slice, and finally 1-2 16-column tiles of dX = dZ0 W0.
//   tail wg: converts the narrow layers' weights into LDS while layer 0 runs, then layers
//       1..L-1, softmax-CE / log-softmax-NLL, the output-gradient chain down to dZ1 (published),
//       and the dW of layers 1..L-1.
// Hand-offs (MI355X_MICROARCH "handoff" rows; cdna_hip_programming §6 Guideline 16, first row
// of the sc1 table): payloads are written with 16-B write-through (sc1) buffer stores, the
// storing wave drains (s_waitcnt vmcnt(0)) and ONE lane signals with an agent-scope atomic; the
// consumer polls ONE word with relaxed sc1 loads (s_sleep between polls, bounded: a timeout
// sets an error word instead of hanging), joins a workgroup barrier, and EVERY load of the
// payload is an sc1 buffer load.  Counters are monotonic across launches: each launch reads the
// epoch E that the previous launch's last-finishing workgroup advanced, and waits for targets
// (E+1)*n -- a stale value can only be smaller than the target, never satisfy it.
//
// Numerics are those of mlp_head.hip: bf16 MFMA operands, fp32 accumulation / statistics, the
// same counter-hash dropout masks (a seed word bumped once per launch), BatchNorm running-stat
// update, bias / BatchNorm / weight gradients accumulated into the caller's fp32 .grad buffers.
#include "head_common.h"

namespace {

constexpr int SMAXL = 6;
constexpr int SNT = 256;     // every workgroup: 4 waves
constexpr int SMT = 2;       // 32 batch rows = two 16-row MFMA tiles
constexpr int SMP = 32;
constexpr int KS0_MAX = 4;   // layer-0 k-steps (32) per wave: layer-0 inputs <= 512
constexpr int DXT_MAX = 2;   // dX 16-column tiles per column workgroup
constexpr int DXN_MAX = 2;   // dX reduction steps (32 layer-0 outputs) per wave: outputs <= 256
constexpr int DW0_MAX = 8;   // dW0 16x16 tiles per wave: layer-0 inputs <= 512
constexpr int W1S_MAX = 8;   // dA1 reduction steps over layer-1 outputs: <= 256
constexpr int W1T_MAX = 4;   // dW1 16-row tiles per wave (layer-1 outputs <= 256)
constexpr int SPIN_MAX = 1 << 22;  // ~0.2 s of polling before a hand-off gives up

// sync block (u32 words, one 128-B line each)
constexpr int Y_EPOCH = 0, Y_A1 = 32, Y_DZ1 = 64, Y_DZ0 = 96, Y_DONE = 128, Y_ERR = 160;
constexpr int Y_WORDS = 256;

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

struct SLayer {
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
  int in, out, Kp, Np;  // Kp = rup32(in), Np = rup32(out)
  int bn, relu;
  float drop, eps, momentum;
  // tail LDS (layers >= 1): W image [Np][SW] bf16, input image [SMP][SW] bf16 (SW = Kp + 8),
  // fp32 [Np] x 8: bias, gamma, beta, rmean, rvar, old gb, old ggamma, old gbeta
  int w_lds, a_lds, p_lds, SW;
  int z_lds, SZ;            // output-gradient image dZ [SMP][SZ] bf16 (SZ = Np + 8)
  long xhat_off, rstd_off;  // workspace: BatchNorm xhat [SMP][Np] / rstd [Np] (tail layers)
};

struct StepArgs {
  SLayer L[SMAXL];
  int nl, B, G0, ndx;      // ndx = 16-column tiles of dX
  long a1_off, dz1_off, dz0_off;  // workspace: published images (bf16)
  int SA1, SZ1, SZ0;       // their row strides (elements)
  // column-workgroup LDS: input image, cross-wave reduction, dZ0 slice, A1 slice, dZ1 image
  int c_img, c_red, c_dzs, c_a1s, c_z1s;
  // tail LDS: logits + dlogits fp32 [SMP][16] each, labels [SMP]
  int t_logit, t_dlogit, t_y;
  int log_out;
  int spin;                // poll limit of the hand-off waits (dn_spin_limit)
};

#define YSTAMP(i) do { if (stamps && threadIdx.x == 0) stamps[(i)] = __builtin_amdgcn_s_memrealtime(); } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ws_rsrc(char* ws) {
  return __builtin_amdgcn_make_buffer_rsrc(ws, 0, 0x7fffffff, 0x00020000);
}
// write-through 16-B store / L1-bypassing 16-B load (aux bit 4 = sc1)
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, long off, bf16x8 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, 16);
}
__device__ __forceinline__ bf16x8 ld_sc1(__amdgpu_buffer_rsrc_t r, long off) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16));
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void arrive(unsigned* sync, int w) {
  __hip_atomic_fetch_add((gu32*)(sync + w), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// ONE lane polls; wrap-safe `>=`; bounded (the error word records which wait gave up)
__device__ __forceinline__ void poll_ge(unsigned* sync, int w, unsigned target, unsigned code,
                                        int spin) {
  gu32* p = (gu32*)(sync + w);
  for (int it = 0; it < spin; ++it) {
    const unsigned v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((int)(v - target) >= 0) return;
    __builtin_amdgcn_s_sleep(1);
  }
  __hip_atomic_store((gu32*)(sync + Y_ERR), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// fp32 weight row fragment, lane -> row n, k .. k+7 (clamped index, validity at conversion)
__device__ __forceinline__ void wrow_raw(const float* __restrict__ W, int N, int K, int n, int k,
                                         bool vec, f32x4 (&r)[2]) {
  if (vec) {
    const int idx = (n < N && k < K) ? n * K + k : 0;
    r[0] = *reinterpret_cast<const f32x4*>(W + idx);
    r[1] = *reinterpret_cast<const f32x4*>(W + idx + 4);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e >> 2][e & 3] = W[(n < N && k + e < K) ? n * K + k + e : 0];
  }
}
__device__ __forceinline__ bf16x8 wrow_cvt(const f32x4 (&r)[2], int N, int K, int n, int k) {
  bf16x8 f;
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = (bf16)((n < N && k + e < K) ? r[e >> 2][e & 3] : 0.f);
  return f;
}
// fp32 weight COLUMN fragment, lane -> column kk, rows n .. n+7 (raw; validity at conversion)
__device__ __forceinline__ void wcol_raw(const float* __restrict__ W, int N, int K, int n, int kk,
                                         float (&r)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = W[(n + j < N && kk < K) ? (n + j) * K + kk : 0];
}
__device__ __forceinline__ bf16x8 wcol_cvt(const float (&r)[8], int N, int K, int n, int kk) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (bf16)((n + j < N && kk < K) ? r[j] : 0.f);
  return f;
}

// LDS-only workgroup barrier: orders the waves and their LDS traffic WITHOUT waiting for the
// wave's outstanding global stores (a __syncthreads is also a device-scope fence: every phase
// that ended in a global store then waited a memory round trip at the barrier).  Global data
// shared between waves of a workgroup goes through explicit waits / hand-offs instead.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ============================================================================================
// column workgroup c: layer 0 for output columns 16c .. 16c+15
// ============================================================================================
__device__ __forceinline__ void column_wg(const StepArgs& a, int c, const float* __restrict__ x,
                                          long ldx, const unsigned long long* __restrict__ rng,
                                          float* __restrict__ dx, long lddx, char* __restrict__ ws,
                                          unsigned* __restrict__ sync, char* smem,
                                          unsigned long long* __restrict__ stamps) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const SLayer& L0 = a.L[0];
  const SLayer& L1 = a.L[1];
  const int B = a.B, K = L0.in, N = L0.out, Kp = L0.Kp, S0 = Kp + 8;
  const unsigned E1 = sync[Y_EPOCH] + 1u;
  const uint64_t seed = *rng;
  const __amdgpu_buffer_rsrc_t rw = ws_rsrc(ws);
  bf16* img = reinterpret_cast<bf16*>(smem + a.c_img);
  float* red = reinterpret_cast<float*>(smem + a.c_red);
  bf16* dzs = reinterpret_cast<bf16*>(smem + a.c_dzs);  // [SMP][24] dZ0 slice
  bf16* a1s = reinterpret_cast<bf16*>(smem + a.c_a1s);  // [SMP][24] A1 slice (dW1)
  bf16* z1s = reinterpret_cast<bf16*>(smem + a.c_z1s);  // [SMP][SZ1] dZ1 (dW1)
  const bool st = c == 0 && stamps;
  if (st) YSTAMP(0);

  const int n = 16 * c + (lane & 15);  // this lane's layer-0 column (wave 0 epilogue)
  const bool cv = n < N;
  const int ni = cv ? n : 0;
  const int nks = Kp / 32;
  const bool vec0 = (K % 8) == 0;

  // ---- 1. the input image (layer-0 dropout applied), bf16 in LDS: its loads lead the queue --
  {
    const float p0 = L0.drop;
    const float inv = p0 > 0.f ? 1.f / (1.f - p0) : 1.f;
    constexpr int R = 16;
    const int KC = Kp / 4, nch = SMP * KC;
    const bool vec = (K % 4) == 0 && (ldx % 4) == 0 && ((reinterpret_cast<uintptr_t>(x)) & 15) == 0;
    const int dm = SNT / KC, dk = SNT - (SNT / KC) * KC;
    int cm = tid / KC, ck = tid - (tid / KC) * KC;
    for (int base = tid; base < nch; base += R * SNT) {
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
      if (vec) {
#pragma unroll
        for (int u = 0; u < R; ++u) {
          const int idx = (ms[u] < B && ks[u] < K) ? ms[u] * (int)ldx + ks[u] : 0;
          v[u] = *reinterpret_cast<const f32x4*>(x + idx);
        }
      } else {
#pragma unroll
        for (int u = 0; u < R; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[u][e] = x[(ms[u] < B && ks[u] + e < K) ? ms[u] * (int)ldx + ks[u] + e : 0];
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int m = ms[u], k = ks[u];
        if (m >= SMP) continue;
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = (m < B && k + e < K) ? v[u][e] : 0.f;
          if (p0 > 0.f && t != 0.f) t = hkeep(seed, 0, m, k + e, K, p0) ? t * inv : 0.f;
          o[e] = (bf16)t;
        }
        *reinterpret_cast<bf16x4*>(img + m * S0 + k) = o;
      }
    }
  }

  if (st) YSTAMP(7);
  // ---- 2. W0 rows of this wave's k-steps (the layer-0 GEMM) and the epilogue parameters -----
  f32x4 wr[KS0_MAX][2];
#pragma unroll
  for (int u = 0; u < KS0_MAX; ++u) {
    const int ks = wid + 4 * u;
    wrow_raw(L0.W, N, K, n, 32 * (ks < nks ? ks : 0) + 8 * (lane >> 4), vec0, wr[u]);
  }
  float bias = 0.f, ga = 1.f, be = 0.f, rm = 0.f, rv = 1.f, gbo = 0.f, ggo = 0.f, gbeo = 0.f;
  if (wid == 0) {
    if (L0.b) { bias = L0.b[ni]; gbo = L0.gb[ni]; }
    if (L0.bn) {
      ga = L0.gamma[ni]; be = L0.beta[ni];
      ggo = L0.ggamma[ni]; gbeo = L0.gbeta[ni];
      if (L0.bn == 2) { rm = L0.rmean[ni]; rv = L0.rvar[ni]; }
    }
  }
  const int n1s = L1.Np / 32, nn1 = L1.Np / 16;
  const int nns = L0.Np / 32;
  const int ntk = (K + 15) / 16;
  float w1c[W1S_MAX][8];           // W1 columns of this workgroup (dA1 = dZ1 W1[:, cols]), wave 0
  float w0c[DXT_MAX][DXN_MAX][8];  // W0 columns of this workgroup's dX tiles
  float gold[DW0_MAX][4];          // old dW0 of this wave's tiles: rows 16c + 4(lane>>4) + r
  float g1o[W1T_MAX][4];           // old dW1 of this workgroup's input columns: n1-tiles wid + 4i
  // operands needed only after the dZ1 hand-off: requested once this wave's part of the
  // forward is out (issuing ~100 loads per lane before the layer-0 GEMM delayed it by ~4.7 us)
  auto prefetch_late = [&]() {
    if (wid == 0) {
#pragma unroll
      for (int s = 0; s < W1S_MAX; ++s)
        if (s < n1s) wcol_raw(L1.W, L1.out, L1.in, 32 * s + 8 * (lane >> 4), n, w1c[s]);
    }
#pragma unroll
    for (int i = 0; i < DXT_MAX; ++i) {
      const int t = c + a.G0 * i;
#pragma unroll
      for (int j = 0; j < DXN_MAX; ++j) {
        const int s = wid + 4 * j;
        if (t < a.ndx && s < nns) wcol_raw(L0.W, N, K, 32 * s + 8 * (lane >> 4), 16 * t + (lane & 15), w0c[i][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < DW0_MAX; ++i) {
      const int tk = wid + 4 * i;
      const int k = 16 * tk + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nr = 16 * c + 4 * (lane >> 4) + r;
        gold[i][r] = L0.gW[(tk < ntk && nr < N && k < K) ? (long)nr * K + k : 0];
      }
    }
#pragma unroll
    for (int i = 0; i < W1T_MAX; ++i) {
      const int tn = wid + 4 * i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n1 = 16 * tn + 4 * (lane >> 4) + r;
        g1o[i][r] = L1.gW[(tn < nn1 && n1 < L1.out && n < N) ? (long)n1 * L1.in + n : 0];
      }
    }
  };
  if (st) YSTAMP(15);
  lds_barrier();  // the input image
  if (st) YSTAMP(1);

  // ---- layer 0: K split over the four waves -------------------------------------------------
  f32x4 acc[SMT];
#pragma unroll
  for (int mt = 0; mt < SMT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < KS0_MAX; ++u) {
    const int ks = wid + 4 * u;
    if (ks < nks) {
      const bf16x8 bq = wrow_cvt(wr[u], N, K, n, 32 * ks + 8 * (lane >> 4));
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(img + (16 * mt + (lane & 15)) * S0 + 32 * ks + 8 * (lane >> 4));
        acc[mt] = mfma16(af, bq, acc[mt]);
      }
    }
  }
  if (wid > 0) {
#pragma unroll
    for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((wid - 1) * SMT * 4 + mt * 4 + r) * 64 + lane] = acc[mt][r];
  }
  lds_barrier();
  if (wid > 0) prefetch_late();

  // wave 0: epilogue + publish; keeps xhat / rstd / the ReLU mask for the backward
  const float p1 = L1.drop;
  const float inv1 = p1 > 0.f ? 1.f / (1.f - p1) : 1.f;
  if (wid == 0) {
    float xh[SMT][4];
    float rstd = 0.f;
    unsigned relu_ok = 0xffu;  // bit 4 mt + r: post-ReLU output > 0
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[mt][r] += red[(w * SMT * 4 + mt * 4 + r) * 64 + lane];
    float z[SMT][4];
#pragma unroll
    for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) z[mt][r] = acc[mt][r] + (cv ? bias : 0.f);
    if (L0.bn) {
      float s = 0.f;
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += (16 * mt + 4 * (lane >> 4) + r < B) ? z[mt][r] : 0.f;
      const float mean = colsum4(s) / (float)B;
      float v = 0.f;
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = z[mt][r] - mean;
          v += (16 * mt + 4 * (lane >> 4) + r < B) ? d * d : 0.f;
        }
      v = colsum4(v) / (float)B;
      rstd = rsqrtf(v + L0.eps);
      if (L0.bn == 2 && lane < 16 && cv) {
        const float mo = L0.momentum;
        L0.rmean[n] = (1.f - mo) * rm + mo * mean;
        L0.rvar[n] = (1.f - mo) * rv + mo * v * ((float)B / (float)(B > 1 ? B - 1 : 1));
      }
      const float g = cv ? ga : 0.f, bb = cv ? be : 0.f;
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * mt + 4 * (lane >> 4) + r;
          xh[mt][r] = (row < B && cv) ? (z[mt][r] - mean) * rstd : 0.f;
          z[mt][r] = g * xh[mt][r] + bb;
        }
    } else {
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) xh[mt][r] = 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * mt + 4 * (lane >> 4) + r;
        float v = z[mt][r];
        if (L0.relu) {
          v = fmaxf(v, 0.f);
          if (!(v > 0.f)) relu_ok &= ~(1u << (4 * mt + r));
        }
        v = (row < B && cv) ? v : 0.f;
        if (p1 > 0.f && v != 0.f) v = hkeep(seed, 1, row, n, N, p1) ? v * inv1 : 0.f;
        a1s[row * 24 + (lane & 15)] = (bf16)v;
      }
    // publish: lane -> (row, 8-column half), one 16-B write-through store each
    const int row = lane >> 1, h = lane & 1;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(a1s + row * 24 + 8 * h);
    st_sc1(rw, a.a1_off + 2L * (row * a.SA1 + 16 * c + 8 * h), v);
    drain();
    if (lane == 0) arrive(sync, Y_A1);
    if (st) YSTAMP(2);
    prefetch_late();

    // ---- wait for dZ1, then dA1 = dZ1 W1[:, cols] and the layer-0 backward -----------------
    if (lane == 0) poll_ge(sync, Y_DZ1, E1, 1u, a.spin);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (st) YSTAMP(3);
    bf16x8 zf[W1S_MAX][SMT];
#pragma unroll
    for (int s = 0; s < W1S_MAX; ++s)
      if (s < n1s)
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
          zf[s][mt] = ld_sc1(rw, a.dz1_off + 2L * ((16 * mt + (lane & 15)) * a.SZ1 + 32 * s + 8 * (lane >> 4)));
    f32x4 da[SMT];
#pragma unroll
    for (int mt = 0; mt < SMT; ++mt) da[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < W1S_MAX; ++s)
      if (s < n1s) {
        const bf16x8 bq = wcol_cvt(w1c[s], L1.out, L1.in, 32 * s + 8 * (lane >> 4), n);
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt) {
          da[mt] = mfma16(zf[s][mt], bq, da[mt]);
          // dZ1 also to LDS: the dW1 tiles of this workgroup's columns read it transposed
          *reinterpret_cast<bf16x8*>(z1s + (16 * mt + (lane & 15)) * a.SZ1 + 32 * s + 8 * (lane >> 4)) = zf[s][mt];
        }
      }
    float d[SMT][4];
#pragma unroll
    for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * mt + 4 * (lane >> 4) + r;
        float t = (row < B && cv) ? da[mt][r] : 0.f;
        if (p1 > 0.f && t != 0.f) t = hkeep(seed, 1, row, n, N, p1) ? t * inv1 : 0.f;
        if (L0.relu && !((relu_ok >> (4 * mt + r)) & 1u)) t = 0.f;
        d[mt][r] = t;
      }
    if (L0.bn) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1 += d[mt][r];
          s2 += d[mt][r] * xh[mt][r];
        }
      s1 = colsum4(s1);
      s2 = colsum4(s2);
      if (lane < 16 && cv) {
        L0.ggamma[n] = ggo + s2;
        L0.gbeta[n] = gbeo + s1;
      }
      const float g = cv ? ga : 0.f;
      const float m1 = s1 / (float)B, m2 = s2 / (float)B;
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * mt + 4 * (lane >> 4) + r;
          d[mt][r] = (row < B && cv) ? g * rstd * (d[mt][r] - m1 - xh[mt][r] * m2) : 0.f;
        }
    }
    if (L0.b) {
      float sb = 0.f;
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) sb += d[mt][r];
      sb = colsum4(sb);
      if (lane < 16 && cv) L0.gb[n] = gbo + sb;
    }
#pragma unroll
    for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) dzs[(16 * mt + 4 * (lane >> 4) + r) * 24 + (lane & 15)] = (bf16)d[mt][r];
    const bf16x8 dv = *reinterpret_cast<const bf16x8*>(dzs + row * 24 + 8 * h);
    st_sc1(rw, a.dz0_off + 2L * (row * a.SZ0 + 16 * c + 8 * h), dv);
    drain();
    if (lane == 0) arrive(sync, Y_DZ0);
    if (st) YSTAMP(4);
  }
  lds_barrier();  // dZ0 slice, dZ1 and the A1 slice in LDS

  // ---- dW0[cols, :] += dZ0_slice^T A0 ; dW1[:, cols] += dZ1^T A1_slice ------------------------
  {
    f32x4 dw[DW0_MAX];
#pragma unroll
    for (int i = 0; i < DW0_MAX; ++i) {
      const int tk = wid + 4 * i;
      dw[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (tk < ntk) dw[i] = mfma16(tr_frag(dzs, 24, 0, 0, lane), tr_frag(img, S0, 16 * tk, 0, lane), dw[i]);
    }
    f32x4 d1[W1T_MAX];
#pragma unroll
    for (int i = 0; i < W1T_MAX; ++i) {
      const int tn = wid + 4 * i;
      d1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (tn < nn1) d1[i] = mfma16(tr_frag(z1s, a.SZ1, 16 * tn, 0, lane), tr_frag(a1s, 24, 0, 0, lane), d1[i]);
    }
#pragma unroll
    for (int i = 0; i < DW0_MAX; ++i) {
      const int tk = wid + 4 * i;
      const int k = 16 * tk + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nr = 16 * c + 4 * (lane >> 4) + r;
        if (tk < ntk && nr < N && k < K) L0.gW[(long)nr * K + k] = gold[i][r] + dw[i][r];
      }
    }
#pragma unroll
    for (int i = 0; i < W1T_MAX; ++i) {
      const int tn = wid + 4 * i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n1 = 16 * tn + 4 * (lane >> 4) + r;
        if (tn < nn1 && n1 < L1.out && n < N) L1.gW[(long)n1 * L1.in + n] = g1o[i][r] + d1[i][r];
      }
    }
  }

  // ---- dX tiles: dX[:, t] = dZ0 W0[:, t] (+ the layer-0 dropout) ---------------------------
  if (dx) {
    if (tid == 0) poll_ge(sync, Y_DZ0, E1 * (unsigned)a.G0, 2u, a.spin);
    lds_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (st) YSTAMP(5);
    bf16x8 zf[DXN_MAX][SMT];
#pragma unroll
    for (int j = 0; j < DXN_MAX; ++j) {
      const int s = wid + 4 * j;
      if (s < nns)
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
          zf[j][mt] = ld_sc1(rw, a.dz0_off + 2L * ((16 * mt + (lane & 15)) * a.SZ0 + 32 * s + 8 * (lane >> 4)));
    }
    f32x4 ax[DXT_MAX][SMT];
#pragma unroll
    for (int i = 0; i < DXT_MAX; ++i)
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt) ax[i][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < DXT_MAX; ++i) {
      const int t = c + a.G0 * i;
      if (t >= a.ndx) continue;
#pragma unroll
      for (int j = 0; j < DXN_MAX; ++j) {
        const int s = wid + 4 * j;
        if (s >= nns) continue;
        const bf16x8 bq = wcol_cvt(w0c[i][j], N, K, 32 * s + 8 * (lane >> 4), 16 * t + (lane & 15));
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt) ax[i][mt] = mfma16(zf[j][mt], bq, ax[i][mt]);
      }
    }
    if (wid > 0) {
#pragma unroll
      for (int i = 0; i < DXT_MAX; ++i)
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            red[(((wid - 1) * DXT_MAX + i) * SMT * 4 + mt * 4 + r) * 64 + lane] = ax[i][mt][r];
    }
    lds_barrier();
    if (wid == 0) {
      const float p0 = L0.drop;
      const float inv0 = p0 > 0.f ? 1.f / (1.f - p0) : 1.f;
#pragma unroll
      for (int i = 0; i < DXT_MAX; ++i) {
        const int t = c + a.G0 * i;
        if (t >= a.ndx) continue;
        const int kx = 16 * t + (lane & 15);
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = ax[i][mt][r];
#pragma unroll
            for (int w = 0; w < 3; ++w) v += red[((w * DXT_MAX + i) * SMT * 4 + mt * 4 + r) * 64 + lane];
            const int row = 16 * mt + 4 * (lane >> 4) + r;
            if (p0 > 0.f && v != 0.f) v = hkeep(seed, 0, row, kx, K, p0) ? v * inv0 : 0.f;
            if (row < B && kx < K) dx[(long)row * lddx + kx] = v;
          }
      }
    }
  }
  if (st) YSTAMP(6);
}

// dW_l += dZ_l^T A_l for a tail layer: dZ image `dzl` [SMP][SZ], input image from LDS
__device__ __forceinline__ void tail_dw(const SLayer& L, const bf16* dzl, int SZ, const bf16* aimg,
                                        int lane, int wid) {
  constexpr int G = 4;
  const int K = L.in, N = L.out, tn = (N + 15) / 16, tk = (K + 15) / 16, nt = tn * tk;
  for (int t0 = wid * G; t0 < nt; t0 += 4 * G) {
    float old[G][4];
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const int t = t0 + gi;
      const int a_ = t / tk, b_ = t - (t / tk) * tk;
      const int k = 16 * b_ + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nn = 16 * a_ + 4 * (lane >> 4) + r;
        const bool ok = t < nt && nn < N && k < K;
        old[gi][r] = L.gW[ok ? (long)nn * K + k : 0];
      }
    }
    f32x4 acc[G];
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const int t = t0 + gi;
      const int a_ = t / tk, b_ = t - (t / tk) * tk;
      acc[gi] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t < nt) acc[gi] = mfma16(tr_frag(dzl, SZ, 16 * a_, 0, lane), tr_frag(aimg, L.SW, 16 * b_, 0, lane), acc[gi]);
    }
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const int t = t0 + gi;
      const int a_ = t / tk, b_ = t - (t / tk) * tk;
      const int k = 16 * b_ + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nn = 16 * a_ + 4 * (lane >> 4) + r;
        if (t < nt && nn < N && k < K) L.gW[(long)nn * K + k] = old[gi][r] + acc[gi][r];
      }
    }
  }
}

// ============================================================================================
// tail workgroup: layers 1 .. nl-1, the loss, the output-gradient chain down to dZ1, their dW
// ============================================================================================
__device__ __forceinline__ void tail_wg(const StepArgs& a, const long long* __restrict__ y,
                                        float* __restrict__ out, float* __restrict__ loss,
                                        long long* __restrict__ pred,
                                        unsigned long long* __restrict__ rng,
                                        const float* __restrict__ dloss, char* __restrict__ ws,
                                        unsigned* __restrict__ sync, char* smem,
                                        unsigned long long* __restrict__ stamps) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int B = a.B, nl = a.nl;
  const unsigned E1 = sync[Y_EPOCH] + 1u;
  const uint64_t seed = *rng;
  const float gs = *dloss;
  const __amdgpu_buffer_rsrc_t rw = ws_rsrc(ws);
  float* logit = reinterpret_cast<float*>(smem + a.t_logit);
  float* dlogit = reinterpret_cast<float*>(smem + a.t_dlogit);
  int* ylds = reinterpret_cast<int*>(smem + a.t_y);
  const bool st = stamps != nullptr;
  if (st) YSTAMP(8);
  if (tid < SMP) {
    const long long yv = tid < B ? y[tid] : 0ll;
    ylds[tid] = (int)(yv < 0 ? -1 : (yv > 0x7fffffffll ? 0x7fffffff : yv));
  }
  // narrow layers' weights -> bf16 LDS images (zero padded), parameters -> LDS (fp32)
  for (int l = 1; l < nl; ++l) {
    const SLayer& L = a.L[l];
    bf16* wimg = reinterpret_cast<bf16*>(smem + L.w_lds);
    const int KC = L.Kp / 8, nch = L.Np * KC;
    const bool vec = (L.in % 8) == 0;
    constexpr int R = 8;
    for (int base = tid; base < nch; base += R * SNT) {
      f32x4 v[R][2];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int ch = base + u * SNT < nch ? base + u * SNT : 0;
        const int nn = ch / KC, kk = 8 * (ch - (ch / KC) * KC);
        wrow_raw(L.W, L.out, L.in, nn, kk, vec, v[u]);
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int ch = base + u * SNT;
        if (ch >= nch) continue;
        const int nn = ch / KC, kk = 8 * (ch - (ch / KC) * KC);
        *reinterpret_cast<bf16x8*>(wimg + nn * L.SW + kk) = wrow_cvt(v[u], L.out, L.in, nn, kk);
      }
    }
    float* pp = reinterpret_cast<float*>(smem + L.p_lds);
    for (int i = tid; i < L.Np; i += SNT) {
      const bool ok = i < L.out;
      pp[i] = (ok && L.b) ? L.b[i] : 0.f;
      pp[L.Np + i] = (ok && L.bn) ? L.gamma[i] : 0.f;
      pp[2 * L.Np + i] = (ok && L.bn) ? L.beta[i] : 0.f;
      pp[3 * L.Np + i] = (ok && L.bn == 2) ? L.rmean[i] : 0.f;
      pp[4 * L.Np + i] = (ok && L.bn == 2) ? L.rvar[i] : 1.f;
      pp[5 * L.Np + i] = (ok && L.b) ? L.gb[i] : 0.f;
      pp[6 * L.Np + i] = (ok && L.bn) ? L.ggamma[i] : 0.f;
      pp[7 * L.Np + i] = (ok && L.bn) ? L.gbeta[i] : 0.f;
    }
  }
  // ---- A1 from the column workgroups --------------------------------------------------------
  if (tid == 0) poll_ge(sync, Y_A1, E1 * (unsigned)a.G0, 3u, a.spin);
  lds_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (st) YSTAMP(9);
  {
    const SLayer& L1 = a.L[1];
    bf16* aimg = reinterpret_cast<bf16*>(smem + L1.a_lds);
    const int KC = L1.Kp / 8, nch = SMP * KC;
    constexpr int R = 4;
    for (int base = tid; base < nch; base += R * SNT) {
      bf16x8 v[R];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int ch = base + u * SNT < nch ? base + u * SNT : 0;
        const int m = ch / KC, kk = 8 * (ch - (ch / KC) * KC);
        v[u] = ld_sc1(rw, a.a1_off + 2L * (m * a.SA1 + kk));
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int ch = base + u * SNT;
        if (ch >= nch) continue;
        const int m = ch / KC, kk = 8 * (ch - (ch / KC) * KC);
        *reinterpret_cast<bf16x8*>(aimg + m * L1.SW + kk) = v[u];
      }
    }
  }
  lds_barrier();
  if (st) YSTAMP(10);

  // ---- forward of layers 1 .. nl-1 ---------------------------------------------------------
  for (int l = 1; l < nl; ++l) {
    const SLayer& L = a.L[l];
    const bool last = l == nl - 1;
    const bf16* aimg = reinterpret_cast<const bf16*>(smem + L.a_lds);
    const bf16* wimg = reinterpret_cast<const bf16*>(smem + L.w_lds);
    const float* pp = reinterpret_cast<const float*>(smem + L.p_lds);
    const int ntiles = last ? 1 : L.Np / 16, nks = L.Kp / 32, N = L.out;
    const SLayer& Ln = a.L[last ? l : l + 1];
    bf16* nimg = reinterpret_cast<bf16*>(smem + Ln.a_lds);
    const float pn = last ? 0.f : Ln.drop;
    const float invn = pn > 0.f ? 1.f / (1.f - pn) : 1.f;
    for (int t = wid; t < ntiles; t += 4) {
      const int nn = 16 * t + (lane & 15);
      const bool cv = nn < N;
      f32x4 acc[SMT];
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int ks = 0; ks < nks; ++ks) {
        const bf16x8 bq = *reinterpret_cast<const bf16x8*>(wimg + nn * L.SW + 32 * ks + 8 * (lane >> 4));
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(aimg + (16 * mt + (lane & 15)) * L.SW + 32 * ks + 8 * (lane >> 4));
          acc[mt] = mfma16(af, bq, acc[mt]);
        }
      }
      float z[SMT][4];
      const float bias = pp[nn];
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) z[mt][r] = acc[mt][r] + bias;
      if (L.bn) {
        float s = 0.f;
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) s += (16 * mt + 4 * (lane >> 4) + r < B) ? z[mt][r] : 0.f;
        const float mean = colsum4(s) / (float)B;
        float v = 0.f;
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float dd = z[mt][r] - mean;
            v += (16 * mt + 4 * (lane >> 4) + r < B) ? dd * dd : 0.f;
          }
        v = colsum4(v) / (float)B;
        const float rstd = rsqrtf(v + L.eps);
        if (L.bn == 2 && lane < 16 && cv) {
          const float mo = L.momentum;
          L.rmean[nn] = (1.f - mo) * pp[3 * L.Np + nn] + mo * mean;
          L.rvar[nn] = (1.f - mo) * pp[4 * L.Np + nn] + mo * v * ((float)B / (float)(B > 1 ? B - 1 : 1));
        }
        float* xhat_ws = reinterpret_cast<float*>(ws + L.xhat_off);
        const float g = pp[L.Np + nn], bb = pp[2 * L.Np + nn];
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + 4 * (lane >> 4) + r;
            const float xv = (row < B && cv) ? (z[mt][r] - mean) * rstd : 0.f;
            xhat_ws[row * L.Np + nn] = xv;
            z[mt][r] = g * xv + bb;
          }
        if (lane < 16) reinterpret_cast<float*>(ws + L.rstd_off)[nn] = cv ? rstd : 0.f;
      }
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * mt + 4 * (lane >> 4) + r;
          float v = z[mt][r];
          if (L.relu) v = fmaxf(v, 0.f);
          if (last) {
            logit[row * 16 + (lane & 15)] = v;
          } else {
            v = (row < B && cv) ? v : 0.f;
            if (pn > 0.f && v != 0.f) v = hkeep(seed, l + 1, row, nn, N, pn) ? v * invn : 0.f;
            nimg[row * Ln.SW + nn] = (bf16)v;
          }
        }
    }
    lds_barrier();
  }
  if (st) YSTAMP(11);

  // ---- loss: softmax / log-softmax + CE / NLL, argmax (wave 0, lane = row) -------------------
  // Only d loss / d logits is on the critical path (-> dZ image -> chain -> dZ1 publish); the
  // outputs, the loss reduction, the counters and the last layer's bias gradient are written
  // after the publish (deferred block below).  Rolled loops over the C live classes: an
  // unrolled 16-class register form was if-converted into 16 precise expf per row.
  const SLayer& LL = a.L[nl - 1];
  const int C = LL.out;
  const int m = lane;
  const bool mv = m < B;
  const float* lr = logit + m * 16;
  float* dr = dlogit + m * 16;
  float lse = 0.f, ly = 0.f;
  int am = 0;
  if (wid == 0) {
    float mx = -INFINITY;
    for (int cc = 0; cc < C; ++cc) {
      const float v = mv ? lr[cc] : 0.f;
      if (v > mx) { mx = v; am = cc; }
    }
    float se = 0.f;
    for (int cc = 0; cc < C; ++cc) se += expf((mv ? lr[cc] : 0.f) - mx);
    lse = mx + logf(se);
    if (st) YSTAMP(19);
    int yc = mv ? ylds[m] : 0;
    yc = yc < 0 ? 0 : (yc >= C ? C - 1 : yc);
    for (int cc = 0; cc < C; ++cc) {
      const float lg = mv ? lr[cc] : 0.f;
      const float p = expf(lg - lse);
      dr[cc] = mv ? (p - (cc == yc ? 1.f : 0.f)) / (float)B : 0.f;
      if (cc == yc) ly = lg;
    }
    if (st) YSTAMP(16);
    // dZ of the logits layer (scaled by d out / d loss): lanes 0-31 row m's 16 leading columns,
    // lanes 32-63 the zero pad columns 16..31 of row m - 32 (C <= 16); each lane reads back only
    // the d loss / d logits row it wrote
    bf16* dz = reinterpret_cast<bf16*>(smem + LL.z_lds);
    bf16x8 z0, z1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      z0[j] = (bf16)(lane < 32 && j < C ? gs * dr[j] : 0.f);
      z1[j] = (bf16)(lane < 32 && 8 + j < C ? gs * dr[8 + j] : 0.f);
    }
    bf16* zr = dz + (lane & 31) * LL.SZ + (lane < 32 ? 0 : 16);
    *reinterpret_cast<bf16x8*>(zr) = z0;
    *reinterpret_cast<bf16x8*>(zr + 8) = z1;
    if (st) YSTAMP(17);
  }
  lds_barrier();
  if (st) YSTAMP(12);

  // ---- output-gradient chain: dZ_l -> dZ_{l-1} for l = nl-1 .. 2 ----------------------------
  // (the BatchNorm xhat / rstd of the narrow layers went to the workspace; each wave reads back
  // the columns it wrote itself, so its own stores only need to have completed)
  bool tail_bn = false;
  for (int l = 1; l < nl - 1; ++l) tail_bn = tail_bn || a.L[l].bn != 0;
  if (tail_bn) drain();
  for (int l = nl - 1; l >= 2; --l) {
    const SLayer& L = a.L[l];
    const SLayer& P = a.L[l - 1];
    const bf16* wimg = reinterpret_cast<const bf16*>(smem + L.w_lds);
    const bf16* aimg = reinterpret_cast<const bf16*>(smem + L.a_lds);  // relu mask of P
    const bf16* dz = reinterpret_cast<const bf16*>(smem + L.z_lds);
    bf16* dzn = reinterpret_cast<bf16*>(smem + P.z_lds);
    const float* pq = reinterpret_cast<const float*>(smem + P.p_lds);
    const int K = L.in, ntl = L.Kp / 16, nns = L.Np / 32;
    const float inv = L.drop > 0.f ? 1.f / (1.f - L.drop) : 1.f;
    const float* xhat_ws = reinterpret_cast<const float*>(ws + P.xhat_off);
    const float* rstd_ws = reinterpret_cast<const float*>(ws + P.rstd_off);
    for (int t = wid; t < ntl; t += 4) {
      const int kk = 16 * t + (lane & 15);
      const bool kv = kk < K;
      const int kc = kv ? kk : 0;
      float xhp[SMT][4], rsp = 0.f;
      if (P.bn) {
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) xhp[mt][r] = xhat_ws[(16 * mt + 4 * (lane >> 4) + r) * P.Np + kc];
        rsp = rstd_ws[kc];
      }
      f32x4 acc[SMT];
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < nns; ++s) {
        const bf16x8 bq = tr_frag(wimg, L.SW, 16 * t, 32 * s, lane);
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(dz + (16 * mt + (lane & 15)) * L.SZ + 32 * s + 8 * (lane >> 4));
          acc[mt] = mfma16(af, bq, acc[mt]);
        }
      }
      float d[SMT][4];
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * mt + 4 * (lane >> 4) + r;
          float v = (row < B && kv) ? acc[mt][r] : 0.f;
          if (L.drop > 0.f && v != 0.f) v = hkeep(seed, l, row, kk, K, L.drop) ? v * inv : 0.f;
          if (P.relu && !((float)aimg[row * L.SW + kk] > 0.f)) v = 0.f;
          d[mt][r] = v;
        }
      if (P.bn) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s1 += d[mt][r];
            s2 += d[mt][r] * xhp[mt][r];
          }
        s1 = colsum4(s1);
        s2 = colsum4(s2);
        if (lane < 16 && kv) {
          P.ggamma[kk] = pq[6 * P.Np + kk] + s2;
          P.gbeta[kk] = pq[7 * P.Np + kk] + s1;
        }
        const float g = kv ? pq[P.Np + kk] : 0.f;
        const float m1 = s1 / (float)B, m2 = s2 / (float)B;
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + 4 * (lane >> 4) + r;
            d[mt][r] = (row < B && kv) ? g * rsp * (d[mt][r] - m1 - xhp[mt][r] * m2) : 0.f;
          }
      }
      if (P.b) {
        float sb = 0.f;
#pragma unroll
        for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) sb += d[mt][r];
        sb = colsum4(sb);
        if (lane < 16 && kv) P.gb[kk] = pq[5 * P.Np + kk] + sb;
      }
#pragma unroll
      for (int mt = 0; mt < SMT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) dzn[(16 * mt + 4 * (lane >> 4) + r) * P.SZ + kk] = (bf16)d[mt][r];
    }
    lds_barrier();
  }
  // dZ1 -> the column workgroups
  {
    const SLayer& L1 = a.L[1];
    const bf16* dz1 = reinterpret_cast<const bf16*>(smem + L1.z_lds);
    const int KC = L1.Np / 8, nch = SMP * KC;
    for (int ch = tid; ch < nch; ch += SNT) {
      const int m = ch / KC, kk = 8 * (ch - (ch / KC) * KC);
      st_sc1(rw, a.dz1_off + 2L * (m * a.SZ1 + kk), *reinterpret_cast<const bf16x8*>(dz1 + m * L1.SZ + kk));
    }
    drain();
    lds_barrier();
    if (tid == 0) __hip_atomic_store((gu32*)(sync + Y_DZ1), E1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (st) YSTAMP(13);
  // ---- deferred loss outputs (wave 0, off the critical path) -------------------------------
  if (wid == 0) {
    for (int cc = 0; cc < C; ++cc) {
      const float lp = (mv ? lr[cc] : 0.f) - lse;
      if (mv) out[(long)m * C + cc] = a.log_out ? lp : expf(lp);
    }
    float ls = mv ? lse - ly : 0.f;
    if (mv) pred[m] = am;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) ls += __shfl_xor(ls, off);
    if (lane == 0) {
      *loss = ls / (float)B;
      *rng = seed + 1ull;
      for (int l = 0; l < nl; ++l)
        if (a.L[l].bn == 2 && a.L[l].nbt)
          __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(a.L[l].nbt), 1ull,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // bias gradient: column sums of d loss / d logits over the batch, summed in row order
    // (readlanes; the same order as the three-launch path, so both agree bitwise)
    if (LL.b) {
      const float* pb = reinterpret_cast<const float*>(smem + LL.p_lds) + 5 * LL.Np;
      for (int cc = 0; cc < C; ++cc) {
        const int bits = __float_as_int(dr[cc]);
        float v = 0.f;
        for (int mm = 0; mm < B; ++mm) v += __int_as_float(__builtin_amdgcn_readlane(bits, mm));
        if (lane == 0) LL.gb[cc] = pb[cc] + gs * v;
      }
    }
    if (st) YSTAMP(18);
  }
  // ---- dW of layers 2 .. nl-1 (layer 1's dW runs in the column workgroups) -----------------
  for (int l = 2; l < nl; ++l) {
    const SLayer& L = a.L[l];
    tail_dw(L, reinterpret_cast<const bf16*>(smem + L.z_lds), L.SZ,
            reinterpret_cast<const bf16*>(smem + L.a_lds), lane, wid);
  }
  if (st) YSTAMP(14);
}

// Touch every 64-B line of the kernel arguments with independent scalar loads, so the argument
// lines are in this CU's scalar cache before the phases that read them one dependent field at a
// time (a per-layer loop over StepArgs serialises one cold scalar miss per line it reaches).
__device__ __forceinline__ void warm_kernargs() {
  constexpr int LINES = (int)((sizeof(StepArgs) + 160 + 63) / 64);
  typedef const __attribute__((address_space(4))) unsigned cu32;
  cu32* kp = (cu32*)__builtin_amdgcn_kernarg_segment_ptr();
  unsigned acc = 0;
#pragma unroll
  for (int i = 0; i < LINES; ++i) acc += kp[16 * i];
  asm volatile("" ::"s"(acc));
}

__global__ void __launch_bounds__(SNT)
head_step_kernel(StepArgs a, const float* __restrict__ x, long ldx, const long long* __restrict__ y,
                 float* __restrict__ out, float* __restrict__ loss, long long* __restrict__ pred,
                 unsigned long long* __restrict__ rng, const float* __restrict__ dloss,
                 float* __restrict__ dx, long lddx, char* __restrict__ ws,
                 unsigned* __restrict__ sync, unsigned long long* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  warm_kernargs();
  const unsigned E1 = sync[Y_EPOCH] + 1u;
  if ((int)blockIdx.x < a.G0) {
    column_wg(a, blockIdx.x, x, ldx, rng, dx, lddx, ws, sync, smem, stamps);
  } else {
    tail_wg(a, y, out, loss, pred, rng, dloss, ws, sync, smem, stamps);
  }
  lds_barrier();
  // every wait of this workgroup is behind it: the last one to finish advances the epoch
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add((gu32*)(sync + Y_DONE), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == E1 * (unsigned)(a.G0 + 1) - 1u)
      __hip_atomic_store((gu32*)(sync + Y_EPOCH), E1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

namespace {

struct SPlan {
  StepArgs a;
  long ws_bytes;
  long lds;
};

static long al256s(long v) { return (v + 255) & ~255L; }
static int al16s(int v) { return (v + 15) & ~15; }

// Workspace / LDS layout of the one-launch head; false when the head is outside its envelope
// (the caller then runs the three-launch path of mlp_head.hip).
static bool step_plan(int nl, const int* dims, const int* flags, const float* drops,
                      const float* bnp, void* const* ptrs, int B, SPlan& p) {
  if (nl < 2 || nl > SMAXL || B < 1 || B > SMP) return false;
  if (dims[nl] < 1 || dims[nl] > 16) return false;
  StepArgs& a = p.a;
  a.nl = nl;
  a.B = B;
  for (int l = 0; l < nl; ++l) {
    SLayer& L = a.L[l];
    L.in = dims[l];
    L.out = dims[l + 1];
    if (L.in < 1 || L.out < 1) return false;
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
      if (!L.W || !L.gW || (L.b && !L.gb)) return false;
      if (L.bn && (!L.gamma || !L.beta || !L.ggamma || !L.gbeta)) return false;
      if (L.bn == 2 && (!L.rmean || !L.rvar)) return false;
    }
    if (l >= 1 && (L.in > 256 || L.Np > 256)) return false;
  }
  const SLayer& L0 = a.L[0];
  if (L0.in > 32 * 4 * KS0_MAX || L0.Np > 32 * 4 * DXN_MAX || L0.Np > 32 * W1S_MAX) return false;
  if ((L0.in + 15) / 16 > 4 * DW0_MAX) return false;
  a.G0 = L0.Np / 16;
  a.ndx = (L0.in + 15) / 16;
  if (a.ndx > DXT_MAX * a.G0) return false;
  // workspace: published images, then the tail's BatchNorm state
  long off = 0;
  a.SA1 = a.L[1].Kp + 8;
  a.SZ1 = a.L[1].Np + 8;
  a.SZ0 = L0.Np + 8;
  a.a1_off = off;
  off = al256s(off + 2L * SMP * a.SA1);
  a.dz1_off = off;
  off = al256s(off + 2L * SMP * a.SZ1);
  a.dz0_off = off;
  off = al256s(off + 2L * SMP * a.SZ0);
  for (int l = 1; l < nl; ++l) {
    SLayer& L = a.L[l];
    L.xhat_off = off;
    if (L.bn) off = al256s(off + 4L * SMP * L.Np);
    L.rstd_off = off;
    if (L.bn) off = al256s(off + 4L * L.Np);
  }
  p.ws_bytes = off;
  // column-workgroup LDS
  int c = 0;
  a.c_img = c;
  c = al16s(c + 2 * SMP * (L0.Kp + 8));
  a.c_red = c;
  c = al16s(c + 4 * 3 * DXT_MAX * SMT * 4 * 64);
  a.c_dzs = c;
  c = al16s(c + 2 * SMP * 24);
  a.c_a1s = c;
  c = al16s(c + 2 * SMP * 24);
  a.c_z1s = c;
  c = al16s(c + 2 * SMP * (a.L[1].Np + 8));
  // tail LDS
  int t = 0;
  for (int l = 1; l < nl; ++l) {
    SLayer& L = a.L[l];
    L.SW = L.Kp + 8;
    L.SZ = L.Np + 8;
    L.w_lds = t;
    t = al16s(t + 2 * L.Np * L.SW);
    L.a_lds = t;
    t = al16s(t + 2 * SMP * L.SW);
    L.p_lds = t;
    t = al16s(t + 4 * 8 * L.Np);
    L.z_lds = t;
    t = al16s(t + 2 * SMP * L.SZ);
  }
  a.t_logit = t;
  t = al16s(t + 4 * SMP * 16);
  a.t_dlogit = t;
  t = al16s(t + 4 * SMP * 16);
  a.t_y = t;
  t = al16s(t + 4 * SMP);
  p.lds = c > t ? c : t;
  return p.lds <= 160 * 1024;
}

static bool g_step_init = false;
static unsigned long long* g_step_stamps = nullptr;

}  // namespace

// Bytes of the persistent control block (zeroed once by the caller, then owned by the kernel).
DN_API long dn_head_step_sync_bytes() { return 4L * Y_WORDS; }

// Workspace bytes of the one-launch head for batch B (out[0]); DN_UNSUPPORTED outside its
// envelope (B <= 32, >= 2 layers, layer 0 <= 512 inputs / 256 outputs, narrow layers <= 256).
DN_API int dn_head_step_layout(int nl, const int* dims, const int* flags, int B, long* out) {
  SPlan p;
  if (!step_plan(nl, dims, flags, nullptr, nullptr, nullptr, B, p)) return DN_UNSUPPORTED;
  out[0] = p.ws_bytes;
  return DN_OK;
}

DN_API int dn_head_step_set_stamps(void* p) {
  g_step_stamps = (unsigned long long*)p;
  return DN_OK;
}

// The whole training step of the head in one launch (forward + loss + backward + every head
// parameter gradient); dloss = device d out / d loss (the step's persistent 1 / accum), dx (may
// be null) = d loss / d x with row stride lddx.  Same pointer table as dn_head_fwd (11 per layer,
// gradient buffers required).  `sync`: dn_head_step_sync_bytes() bytes, zeroed before first use.
DN_API int dn_head_step(int nl, const int* dims, const int* flags, const float* drops,
                        const float* bnp, void* const* ptrs, const float* x, long ldx, int B,
                        const long long* y, float* out, float* loss, long long* pred,
                        unsigned long long* rng, void* ws, void* sync, int log_out,
                        const float* dloss, float* dx, long lddx, hipStream_t st) {
  SPlan p;
  if (!dloss || !sync || !rng || !step_plan(nl, dims, flags, drops, bnp, ptrs, B, p))
    return DN_UNSUPPORTED;
  if (!g_step_init) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(head_step_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    g_step_init = true;
  }
  p.a.log_out = log_out;
  p.a.spin = dn_spin_limit(SPIN_MAX);
  // the column workgroups and the tail hand data to each other: all must be resident at once
  if (!dn_fits_resident(reinterpret_cast<const void*>(head_step_kernel), p.a.G0 + 1, SNT, p.lds))
    return DN_UNSUPPORTED;
  hipLaunchKernelGGL(head_step_kernel, dim3(p.a.G0 + 1), dim3(SNT), p.lds, st, p.a, x, ldx, y,
                     out, loss, pred, rng, dloss, dx, lddx, (char*)ws, (unsigned*)sync,
                     g_step_stamps);
  return dn_launch_status();
}
