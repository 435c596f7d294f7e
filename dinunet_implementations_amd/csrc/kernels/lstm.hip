// Persistent bidirectional LSTM recurrence for gfx950 (MI355X).
//
// Replaces the reference's per-time-step Python loop (comps/icalstm/models.py:30-41, ~12 kernel
// launches per step and direction) with ONE launch per pass:
//
//   grid  = (ceil(B/16) batch chunks, ndir directions)        -> independent workgroups
//   block = HD/16 waves; wave w owns hidden units [16w, 16w+16)
//
// * The recurrent weights W_hh of a direction (4*HD x HD bf16, 295 KB at HD=192) stay RESIDENT in
//   VGPRs for all S steps as MFMA A-fragments (96 VGPRs per lane at HD=192, 12 waves): nothing is
//   re-read from L2 inside the time loop.
// * Gate rows are permuted to m = 4*u + g (g = i,f,o,g) so one 16x16x32 MFMA output tile holds,
//   per lane, all four gate pre-activations of ONE (unit, batch-row): the cell update is entirely
//   lane-local, no shuffles, no LDS round trip for gates.
// * h_t (bf16) is exchanged between waves through a double-buffered, bank-conflict-free LDS tile:
//   exactly one workgroup barrier per time step.
// * The input projection x_t W_ih^T (time-parallel) is hoisted into one large GEMM before the
//   kernel; its per-step loads are issued before the step's MFMAs so their latency hides under
//   the recurrent GEMM.
// * Reference numerics: i,f,o = sigmoid(sigmoid(pre)), g = tanh(pre),
//   reverse direction consumes x[S-1-t]; its outputs stay in processing order.
//
// The backward kernel runs the reverse-time recurrence dh_{t-1} = W_hh^T dpre_t with W_hh^T
// resident the same way (one unit-quad per lane), recomputes the gates from the saved
// pre-activations, and writes dpre (bf16, original time order) for the weight-gradient GEMMs
// dW_ih = dpre^T x, dW_hh = dpre^T h_{t-1} that run after it on the full chip.
#include "common.h"
#include "prologue.h"
#include <stdlib.h>

#ifdef DN_STAMPS
// diagnostic build only (tools/lstm_stamps.py): per-wave phase cycle sums
__device__ unsigned long long* dn_stamp_buf;
DN_API int dn_set_stamp_buf(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(dn_stamp_buf), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
#define STAMP(v) do { __builtin_amdgcn_sched_barrier(0); \
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) :: "memory"); \
  __builtin_amdgcn_sched_barrier(0); } while (0)
#endif

namespace {

template <typename XT> struct Gate4Raw;
template <> struct Gate4Raw<float> { typedef f32x4 type; };
template <> struct Gate4Raw<bf16> { typedef bf16x4 type; };

typedef __attribute__((ext_vector_type(2))) unsigned dn_u32x2;
__device__ __forceinline__ f32x4 to_f32x4(const f32x4& v) { return v; }
__device__ __forceinline__ f32x4 to_f32x4(const bf16x4& v) {
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}

// raw (unconverted) 4-gate load: keeps bf16 inputs packed in 2 VGPRs across the MFMA phase
template <typename XT>
__device__ __forceinline__ typename Gate4Raw<XT>::type load_raw4(const XT* p, bool ok) {
  typedef typename Gate4Raw<XT>::type R;
  if (ok) return *reinterpret_cast<const R*>(p);
  R z;
  z[0] = z[1] = z[2] = z[3] = (XT)0.f;
  return z;
}

// 16-B weight fragment through a buffer descriptor: per-lane offset in one VGPR, the
// fragment's constant part as the scalar offset -- no per-fragment 64-bit address held live
// across the time loop (the streamed-weight variants re-read W every step)
__device__ __forceinline__ bf16x8 load_wfrag(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, soff, 0));
}

__device__ __forceinline__ void load_gate4(const float* p, bool ok, float (&v)[4]) {
  f32x4 x = load_raw4<float>(p, ok);
  v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}

// Cross-lane redistribution of the MFMA output without LDS: lane n of a 16-lane row receives
// register v[n / BR] of lane n % BR of the same row.  DPP row shifts (VALU, a few cycles) instead
// of ds_bpermute (an LDS round trip each): BR=4 -> 3 moves, BR=8 -> 1, BR=16 -> none.
template <int SHR, int BANK>
__device__ __forceinline__ float dpp_row_shr(float old, float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
      __builtin_bit_cast(int, old), __builtin_bit_cast(int, v), 0x110 + SHR, 0xF, BANK, false));
}

template <int BR>
__device__ __forceinline__ float row_gather(const float (&v)[16 / BR]) {
  if constexpr (BR == 4) {
    float o = v[0];
    o = dpp_row_shr<4, 0x2>(o, v[1]);
    o = dpp_row_shr<8, 0x4>(o, v[2]);
    o = dpp_row_shr<12, 0x8>(o, v[3]);
    return o;
  } else if constexpr (BR == 8) {
    return dpp_row_shr<8, 0xC>(v[0], v[1]);
  } else {
    return v[0];
  }
}

// In-workgroup step hand-off without a barrier (LDS only).  A producer wave writes its h (or
// dpre) tile to LDS, makes those writes complete (LDS-only release: s_waitcnt lgkmcnt(0)) and
// adds 1 to its group's counter (4 producer waves per group, so after step t the counter is
// 4 (t + 1)); a consumer polls that ONE word (relaxed atomic LDS load, wave-uniform) until it
// reaches the step it needs, then reads the tile.  LDS services a wave's requests in order, so
// a consumer that has seen the count reads the published data.  (A `volatile` poll would make
// hipcc wait for every outstanding global load and store at each poll.)
__device__ __forceinline__ void publish_count(int* ctr, bool leader) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (leader) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void wait_count(int* ctr, int need) {
  while (__builtin_amdgcn_readfirstlane(
             __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < need)
    __builtin_amdgcn_s_sleep(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ---------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------
// m-tiles (of 4 per wave) whose W fragments live in LDS instead of VGPRs (fwd), and k-steps
// (of 4*HD/32) of W^T kept in LDS (bwd): sized so HD=192 fits 168 VGPRs (3 waves/SIMD) spill-free.
// At BR = 4 / 8 a lane owns 1-2 gate slots, which leaves room for all of W_hh in VGPRs in the
// forward and all but 4 k-steps of W_hh^T in the backward (whose exchange-tile reads run ahead
// of the MFMA chain and need the registers): spill-free at 168.
#ifndef BWD_CHAINS
#define BWD_CHAINS 2
#endif
// k-steps per group of exchange-tile reads in the backward's resident-weight K loop
#ifndef BWD_RG
#define BWD_RG 4
#endif
// LSTM_FLAGS: forward step hand-off through LDS counters (1; 2: with each producer group's h
// fragments read in one round) or a workgroup barrier (0);
// LSTM_PRIO: wave priority raised over the gate phase (the step's critical path) when > 0
#ifndef LSTM_FLAGS
#define LSTM_FLAGS 0
#endif
#ifndef LSTM_PRIO
#define LSTM_PRIO 0
#endif
// LSTM_POLY: the outer sigmoid of the reference's double sigmoid, sigmoid(s) for s = sigmoid(x)
// in (0, 1), as a degree-5 polynomial (max abs error 6.2e-7 on [0, 1]: 5 FMAs instead of
// mul + exp + add + rcp)
#ifndef LSTM_POLY
#define LSTM_POLY 0
#endif
__device__ __forceinline__ float sigmoid_unit(float s) {
  if constexpr (LSTM_POLY) {
    float v = 0.0011067962041124701f;
    v = __builtin_fmaf(v, s, 0.0014183232560753822f);
    v = __builtin_fmaf(v, s, -0.021660439670085907f);
    v = __builtin_fmaf(v, s, 0.00021609874966088682f);
    v = __builtin_fmaf(v, s, 0.24997784197330475f);
    return __builtin_fmaf(v, s, 0.500000536441803f);
  } else {
    return dn_sigmoid(s);
  }
}
template <int HD, int BR> struct LdsSplit { static constexpr int FWD_MT = 0, BWD_KS = 0; };
// (192, 4): all of W_hh^T in VGPRs, exchange-tile reads in groups of 2 k-steps (BWD_RG_192):
// 111.3 vs 117.0 us with 4 k-steps of W^T in LDS and groups of 4 (tools/lstm_time.py) -- the
// LDS-resident weights cost 48 extra wave-wide LDS reads per step on an LDS-bound loop
#ifndef LSTM_BWD_KS_192_4
#define LSTM_BWD_KS_192_4 0
#endif
#ifndef BWD_RG_192
#define BWD_RG_192 2
#endif
template <> struct LdsSplit<192, 4> { static constexpr int FWD_MT = 0, BWD_KS = LSTM_BWD_KS_192_4; };
template <> struct LdsSplit<192, 8> { static constexpr int FWD_MT = 0, BWD_KS = 6; };
template <> struct LdsSplit<192, 16> { static constexpr int FWD_MT = 1, BWD_KS = 9; };

// MFMA columns >= BR (padded batch columns of the 16-wide B operand) are never consumed: the
// row_gather / slot redistribution only takes columns < BR.  Their lanes therefore read row
// n % BR -- the same 16 B as a valid lane, an LDS broadcast -- so every lane group of a
// ds_read_b128 touches only BR distinct addresses on disjoint banks (rows are 4 banks apart).
// The former all-zero slot (row BR, column 64) shared banks with valid rows at some k-steps:
// rocprofv3 SQ_LDS_BANK_CONFLICT was ~90% of SQ_ACTIVE_INST_LDS in the backward.

// BR = batch rows per workgroup (4, 8 or 16).  The recurrent MFMA always computes 16 columns;
// columns >= BR are zero.  For the gate phase the BR valid columns are redistributed over all
// 64 lanes (ds_bpermute), so each lane owns BR/4 (unit, row) slots instead of 4: the VALU-bound
// gate work per CU shrinks by 16/BR while batch rows stay independent (no cross-CU traffic).
// Lane map: q = lane>>4, n = lane&15, r = n / BR (lane group), b = n % BR (row in chunk);
// slot s holds m-tile mt = r + s*(16/BR) -> unit u = 16w + 4*mt + q.
//
// All per-step global traffic is UNCONDITIONAL (internal buffers padded to Bp rows and HD
// units; loads of padded rows clamp to row B-1): no divergent branches around memory ops, so
// hipcc emits counted s_waitcnt vmcnt(N) and a step never waits for the previous step's stores.
// UG = unit groups (16 units = 4 m-tiles each) per wave: UG = 1 is 3 waves per SIMD at HD=192;
// UG = 3 is ONE wave per SIMD owning 12 m-tiles -- the 72 MFMAs of a SIMD come from 12
// independent accumulator chains of one wave (no issue arbitration between waves) and the h
// tile is read once per k-step for 12 MFMAs instead of 4.
// PT: element type of the stored gate pre-activations (float, or bf16 with
// DINUNET_LSTM_PRE_BF16: half the bytes the forward writes and the backward reads per step)
template <int HD, int BR, bool SEQ, int UG, typename PT = float>
__device__ __forceinline__ void
fwd_recur(const bf16* xp,                  // [B*S][ndir][4*HD] permuted cols, no bias (bf16)
          const float* __restrict__ bias,  // [ndir][4*HD] permuted + padded, b_ih + b_hh
          const bf16* __restrict__ whh,    // [ndir][4*HD][HD] permuted rows, zero padded
          int B, int S, int Hd, int ndir,
          float* __restrict__ c_save,      // [ndir][Bp][S][HD]   c_t at original time idx
          bf16* __restrict__ hprev,        // [ndir][Bp][S][HD]   h_{t-1} at original time idx
          float* __restrict__ hseq,        // SEQ: [Bp][S][ndir*HD] (processing order)
          float* __restrict__ hmean, float mean_scale,  // [B][ndir*Hd]
          float* __restrict__ hT, float* __restrict__ cT,  // [B][ndir*Hd]
          PT* __restrict__ pre,  // [B*S][ndir][4*HD] gate pre-activations (+ bias), or null
          int bsplit,  // > 0: bias holds b_ih at [0] and b_hh at [bsplit], summed here
          const int bx, const int dir, const int gx) {
  constexpr int NW = HD / (16 * UG);
  constexpr int NT = NW * 64;
  constexpr int MT = 4 * UG;   // m-tiles per wave
  constexpr int KS = HD / 32;
  // row stride = 16 or 48 dwords mod 64 banks (HD % 64 == 0): the 4 rows x 4 k-quads of a
  // ds_read_b128 lane group land on 16 distinct bank quads (HD + 8 left rows 4 banks apart,
  // colliding with the k-quad offsets)
  constexpr int LDH = HD + 32;
  // HD > 192: W_hh (>= 512 KB per direction) exceeds the register file, so it is streamed from
  // L2 every step (k-step ks+1's fragments requested before ks's MFMAs) instead of resident
  constexpr bool STREAM = HD > 192;
  constexpr int NLM = (UG == 1 && !STREAM) ? LdsSplit<HD, BR>::FWD_MT : 0, NRM = MT - NLM;
  constexpr int G16 = 16 / BR, NSL1 = BR / 4, NSL = UG * NSL1;
  __shared__ __attribute__((aligned(16))) bf16 hbuf[2][16][LDH];
  // hcnt[g] = h_t tiles published by producer group g (4 waves): 4 (t + 1) after step t
  __shared__ __attribute__((aligned(16))) int hcnt[NW / 4];
  __shared__ __attribute__((aligned(16))) float bias_s[4 * HD];
  // lane-linear fragment image: one 1 KiB row per (wave, m-tile, k-step) -> conflict-free b128
  __shared__ __attribute__((aligned(16))) bf16x8 wlds[NLM > 0 ? NW : 1][NLM > 0 ? NLM : 1][NLM > 0 ? KS : 1][64];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q = lane >> 4, n = lane & 15, r = n / BR, bl = n % BR;
  const int Bp = gx * BR;
  const int b = bx * BR + bl;                   // padded row (always < Bp)
  const int bc = b < B ? b : B - 1;             // clamped row for loads
  const long rowX = (long)ndir * 4 * HD;

  // this direction's W_hh (streamed variant: re-read every step, L2-resident) and the lane's
  // byte offset into it
  const __amdgpu_buffer_rsrc_t w_rs = dn_rsrc(whh + (long)dir * 4 * HD * HD, (uint32_t)(4 * HD * HD * 2));
  // fragment-linear image (lstm_pack_kernel): this wave's tiles start at tile MT*w, lane-linear
  const uint32_t wvo = (uint32_t)((MT * w * KS * 64 + lane) * 16);
  bf16x8 wf[STREAM ? 1 : NRM][STREAM ? 1 : KS];
  // streamed variant: a ring of RS k-steps of fragments, PD = RS - 1 k-steps requested ahead of
  // the MFMAs and continuing across time steps (W does not change), so the next step's first
  // fragments fly during this step's gate math and hand-off.  RS divides KS, so a k-step's slot
  // is the same every time step.
  constexpr int RS = !STREAM ? 1 : (HD == 256 ? 4 : 2);  // 3 at HD = 384 spills (SEQ)
  static_assert(KS % RS == 0, "weight ring");
  bf16x8 wring[RS][MT];
  if constexpr (STREAM) {
#pragma unroll
    for (int ks = 0; ks + 1 < RS; ++ks)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) wring[ks][mt] = load_wfrag(w_rs, wvo, (mt * KS + ks) * 1024);
  }
  if constexpr (!STREAM) {
    const bf16* wlane = whh + (long)dir * 4 * HD * HD + (long)(16 * MT * w + n) * HD + 8 * q;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(wlane + (long)16 * mt * HD + 32 * ks);
        if (mt < NRM) wf[mt < NRM ? mt : 0][ks] = v;
        else wlds[w][mt - NRM][ks][lane] = v;
      }
  }
  for (int i = tid; i < 4 * HD; i += NT)
    bias_s[i] = bsplit ? bias[dir * 4 * HD + i] + bias[bsplit + dir * 4 * HD + i]
                       : bias[dir * 4 * HD + i];
  for (int i = tid; i < 2 * 16 * LDH; i += NT) (&hbuf[0][0][0])[i] = (bf16)0.f;
  if (tid < NW / 4) hcnt[tid] = 0;
  __syncthreads();

  int uu[NSL];  // slot (group gu, s1) -> unit of m-tile 4*gu + r + s1*G16 of this wave
#pragma unroll
  for (int s = 0; s < NSL; ++s)
    uu[s] = 16 * (UG * w + s / NSL1) + 4 * (r + (s % NSL1) * G16) + q;
  // Every per-step global access goes through a buffer descriptor with a 32-bit per-lane byte
  // offset: the step part of an address is one scalar multiply, no 64-bit address math per
  // access.  The descriptors are based at THIS workgroup's first batch row (64-bit base), so an
  // offset spans only its BR rows -- any batch size fits (a global base capped the recurrence
  // at B * S * ndir * 4 * HD * 4 < 2 GiB, B ~ 3,500 at the headline geometry).  Gate
  // pre-activation stores of padded rows (b >= B) get an out-of-range offset and are dropped (no
  // branch, see common.h); without a backward the descriptor has no records and every such store
  // is dropped.
  const int rowXi = ndir * 4 * HD;
  const int b0 = bx * BR;                         // first batch row of this workgroup (< B)
  const int nrow = B - b0 < BR ? B - b0 : BR;     // its valid rows
  const __amdgpu_buffer_rsrc_t x_rs = dn_rsrc(xp + (long)b0 * S * rowXi, (uint32_t)(nrow * S * rowXi * 2));
  const __amdgpu_buffer_rsrc_t pre_rs =
      dn_rsrc(pre ? pre + (long)b0 * S * rowXi : pre,
              pre ? (uint32_t)(nrow * S * rowXi * (int)sizeof(PT)) : 0u);
  const long cb0 = ((long)dir * Bp + b0) * S * HD;  // [ndir][Bp][S][HD] images
  const __amdgpu_buffer_rsrc_t c_rs = dn_rsrc(c_save + cb0, (uint32_t)(BR * S * HD * 4));
  const __amdgpu_buffer_rsrc_t hp_rs = dn_rsrc(hprev + cb0, (uint32_t)(BR * S * HD * 2));
  uint32_t xo[NSL], po[NSL], co[NSL], ho[NSL];  // per-lane byte offsets at time index 0
#pragma unroll
  for (int s = 0; s < NSL; ++s) {
    xo[s] = (uint32_t)(((bc - b0) * S * rowXi + dir * 4 * HD + 4 * uu[s]) * 2);
    po[s] = b < B ? (uint32_t)(((b - b0) * S * rowXi + dir * 4 * HD + 4 * uu[s]) * (int)sizeof(PT))
                  : DN_OOB;
    co[s] = (uint32_t)((((b - b0) * S) * HD + uu[s]) * 4);
    ho[s] = (uint32_t)((((b - b0) * S) * HD + uu[s]) * 2);
  }
  const uint32_t xstep = (uint32_t)(rowXi * 2);  // bytes per time index (bf16 projection)
  const uint32_t pstep = (uint32_t)(rowXi * (int)sizeof(PT));  // (pre-activations)
  // the 4 gate inputs of a slot stay packed (2 VGPRs, unconverted) while the load is in flight
  auto load_x = [&](int s, int tau) {  // time index -1 / S wraps out of range: reads 0
    return __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(
        x_rs, (int)(xo[s] + (uint32_t)tau * xstep), 0, 0));
  };
  // h_{t-1} for the weight-gradient GEMMs: each lane stores the h it produces into step t+1's
  // slot (the last step's h has no slot: out-of-range offset, dropped); slot 0 holds h_{-1} = 0
  {
    const int tau0 = dir == 0 ? 0 : S - 1;
#pragma unroll
    for (int s = 0; s < NSL; ++s)
      __builtin_amdgcn_raw_buffer_store_b16((unsigned short)0, hp_rs,
                                            (int)(ho[s] + (uint32_t)(tau0 * HD * 2)), 0, 0);
  }

  float c[NSL], hs[NSL], hl[NSL];
  // xa / xb: the input projection of the current / next step, ping-ponged over a 2-step
  // unrolled loop so that no register copy (and no vmcnt wait) sits between a prefetch and its
  // use one step later
  bf16x4 xa[NSL], xb[NSL];
  f32x4 bbr[NSL];
#pragma unroll
  for (int s = 0; s < NSL; ++s) {
    c[s] = hs[s] = hl[s] = 0.f;
    if constexpr (NSL == 1 || (NSL == 2 && HD != 512)) bbr[s] = *reinterpret_cast<const f32x4*>(&bias_s[4 * uu[s]]);
    xa[s] = load_x(s, dir == 0 ? 0 : S - 1);
  }
  int cur = 0;
  // the resident-weight loads have all landed before the time loop: without this the loop's
  // waitcnt bookkeeping (merged over the loop entry) keeps waiting on the previous step's stores
  // in the MFMA phase
  __builtin_amdgcn_s_waitcnt(DN_VMCNT0);
#ifdef DN_STAMPS
  unsigned long long st_a = 0, st_b = 0, st_c = 0, ts0, ts1, ts2, ts3;
#endif
  // step t+1's projection is requested before this step's MFMAs (up to two gate slots per lane:
  // the bf16 projection keeps a slot's prefetch in 2 VGPRs; 4 slots, and 2 at HD = 512, spill
  // and re-load in place after the use instead).  The bias registers bbr follow the same rule.
  constexpr bool EARLY = NSL == 1 || (NSL == 2 && HD != 512);
  auto step = [&](const int t, bf16x4 (&xn)[NSL], bf16x4 (&xnn)[NSL]) {
    __builtin_amdgcn_sched_barrier(0);  // step boundary for the scheduler (see the backward)
#ifdef DN_STAMPS
    STAMP(ts0);
#endif
    const int tau = dir == 0 ? t : S - 1 - t;
    const int tau1 = dir == 0 ? t + 1 : S - 2 - t;  // past the end at the last step: reads 0
    if constexpr (EARLY) {
#pragma unroll
      for (int s = 0; s < NSL; ++s) xnn[s] = load_x(s, tau1);
    }
    // recurrent GEMM  pre^T[m][b] = sum_k W[m][k] h[b][k]  (W resident).  No workgroup
    // barrier: before the k-steps of a group of 4 producer waves (64*UG units of h_{t-1}) the
    // wave polls that group's counter, so its MFMAs start on the units already published
    // while the slower waves still run the gate math of step t-1
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (STREAM) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        // bounded look-ahead: unbounded hoisting of the loads spills
        __builtin_amdgcn_sched_barrier(0);
        constexpr int PD = RS - 1;
        const int kl = (ks + PD) % KS;  // past the last k-step: the next time step's
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          wring[(ks + PD) % RS][mt] = load_wfrag(w_rs, wvo, (mt * KS + kl) * 1024);
        const bf16x8 hb = *reinterpret_cast<const bf16x8*>(&hbuf[cur][n % BR][32 * ks + 8 * q]);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma16(wring[ks % RS][mt], hb, acc[mt]);
      }
    }
    // every k-step's h fragment requested up front (4-row layout, resident weights, barrier
    // hand-off): hipcc otherwise issued them two at a time right before their MFMAs and exposed
    // the LDS latency three times per step
    constexpr bool HB_ALL = !STREAM && !LSTM_FLAGS && BR == 4 && UG == 1 && NLM == 0;
    bf16x8 hball[HB_ALL ? KS : 1];
    if constexpr (HB_ALL) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        hball[ks] = *reinterpret_cast<const bf16x8*>(&hbuf[cur][n % BR][32 * ks + 8 * q]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // LSTM_FLAGS == 2: the flag hand-off with each producer group's h fragments read together
    // right after its counter is seen (2 k-steps per read round instead of one read per k-step)
    constexpr bool GRP = LSTM_FLAGS == 2 && !STREAM && UG == 1 && NLM == 0;
    bf16x8 hg[2];
#pragma unroll
    for (int ks = 0; ks < (STREAM ? 0 : KS); ++ks) {
      if constexpr (LSTM_FLAGS) {
        if (ks % (2 * UG) == 0) {
          wait_count(&hcnt[ks / (2 * UG)], 4 * t);
          if constexpr (GRP) {
            hg[0] = *reinterpret_cast<const bf16x8*>(&hbuf[cur][n % BR][32 * ks + 8 * q]);
            hg[1] = *reinterpret_cast<const bf16x8*>(&hbuf[cur][n % BR][32 * (ks + 1) + 8 * q]);
          }
        }
      }
      // unmasked (exec-masking made the compiler branch and drain lgkmcnt before every MFMA):
      // lanes of padded columns re-read a valid row, see above
      const bf16x8 hb = HB_ALL ? hball[HB_ALL ? ks : 0]
                      : GRP ? hg[ks & 1]
                            : *reinterpret_cast<const bf16x8*>(&hbuf[cur][n % BR][32 * ks + 8 * q]);
#pragma unroll
      for (int mt = 0; mt < NRM; ++mt) acc[mt] = mfma16(wf[mt][ks], hb, acc[mt]);
#pragma unroll
      for (int mt = NRM; mt < MT; ++mt) acc[mt] = mfma16(wlds[w][mt - NRM][ks][lane], hb, acc[mt]);
    }
    // redistribute the BR valid columns over all lanes (identity when BR == 16)
    f32x4 pa[NSL];
    if constexpr (BR == 16) {
#pragma unroll
      for (int s = 0; s < NSL; ++s) pa[s] = acc[s];
    } else {
      // slot (gu, s1) of lane (q, r, bl) = m-tile 4*gu + r + s1*G16 of column bl (held by
      // lane (q, bl))
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v[G16];
#pragma unroll
          for (int g = 0; g < G16; ++g) v[g] = acc[4 * (sl / NSL1) + g + (sl % NSL1) * G16][j];
          pa[sl][j] = row_gather<BR>(v);
        }
    }
#ifdef DN_STAMPS
    { float z = pa[0][0]; asm volatile("" :: "v"(z)); }
    STAMP(ts1);
#endif
    if constexpr (LSTM_PRIO > 0) __builtin_amdgcn_s_setprio(LSTM_PRIO);
    const int nxt = cur ^ 1;
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      const int u = uu[s];
      const f32x4 bb = EARLY ? bbr[s] : *reinterpret_cast<const f32x4*>(&bias_s[4 * u]);
      const float p0 = pa[s][0] + (float)xn[s][0] + bb[0];
      const float p1 = pa[s][1] + (float)xn[s][1] + bb[1];
      const float p2 = pa[s][2] + (float)xn[s][2] + bb[2];
      const float p3 = pa[s][3] + (float)xn[s][3] + bb[3];
      // the gate pre-activations x W_ih^T + h W_hh^T + b, in place of the projection they were
      // built from: the backward reads them instead of re-running a time-parallel GEMM
      if constexpr (sizeof(PT) == 4) {
        dn_store_f32x4(pre_rs, po[s] + (uint32_t)tau * pstep, f32x4{p0, p1, p2, p3});
      } else {
        const bf16x4 pe = bf16x4{(bf16)p0, (bf16)p1, (bf16)p2, (bf16)p3};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(dn_u32x2, pe), pre_rs,
                                              (int)(po[s] + (uint32_t)tau * pstep), 0, 0);
      }
      if constexpr (!EARLY) xn[s] = load_x(s, tau1);
      const float gi = sigmoid_unit(dn_sigmoid(p0));
      const float gf = sigmoid_unit(dn_sigmoid(p1));
      const float go = sigmoid_unit(dn_sigmoid(p2));
      const float gg = dn_tanh(p3);
      c[s] = gf * c[s] + gi * gg;
      const float h = go * dn_tanh(c[s]);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, c[s]), c_rs,
                                            (int)(co[s] + (uint32_t)(tau * HD * 4)), 0, 0);
      if constexpr (SEQ) hseq[((long)b * S + t) * ndir * HD + dir * HD + u] = h;
      hs[s] += h;
      hl[s] = h;
      const bf16 hb16 = (bf16)h;
      hbuf[nxt][bl][u] = hb16;
      __builtin_amdgcn_raw_buffer_store_b16(
          __builtin_bit_cast(unsigned short, hb16), hp_rs,
          (int)(t + 1 < S ? ho[s] + (uint32_t)(tau1 * HD * 2) : DN_OOB), 0, 0);
    }
#ifdef DN_STAMPS
    STAMP(ts2);
#endif
    if constexpr (LSTM_FLAGS) publish_count(&hcnt[w / 4], lane == 0);
    else __syncthreads();
    if constexpr (LSTM_PRIO > 0) __builtin_amdgcn_s_setprio(0);
#ifdef DN_STAMPS
    STAMP(ts3);
    st_a += ts1 - ts0; st_b += ts2 - ts1; st_c += ts3 - ts2;
#endif
    cur = nxt;
  };
  int t = 0;
  if constexpr (EARLY) {
    for (; t + 1 < S; t += 2) {
      step(t, xa, xb);
      step(t + 1, xb, xa);
    }
  } else {
    for (; t < S; ++t) step(t, xa, xa);
  }
  if (t < S) step(t, xa, xb);
#ifdef DN_STAMPS
  if (lane == 0 && bx == 0) {
    unsigned long long* o = dn_stamp_buf + (dir * 64 + w) * 4;
    o[0] = st_a; o[1] = st_b; o[2] = st_c; o[3] = S;
  }
#endif
#pragma unroll
  for (int s = 0; s < NSL; ++s) {
    const int u = uu[s];
    if (b < B && u < Hd) {
      const long o = (long)b * ndir * Hd + dir * Hd + u;
      if (hmean) hmean[o] = hs[s] * mean_scale;
      if (hT) hT[o] = hl[s];
      if (cT) cT[o] = c[s];
    }
  }
}

template <int HD, int BR, bool SEQ, int UG, typename PT = float>
__global__ void __launch_bounds__(HD / (16 * UG) * 64)
lstm_fwd_kernel(const bf16* xp, const float* __restrict__ bias, const bf16* __restrict__ whh,
                int B, int S, int Hd, int ndir, float* __restrict__ c_save,
                bf16* __restrict__ hprev, float* __restrict__ hseq, float* __restrict__ hmean,
                float mean_scale, float* __restrict__ hT, float* __restrict__ cT,
                PT* __restrict__ pre, int bsplit) {
  fwd_recur<HD, BR, SEQ, UG, PT>(xp, bias, whh, B, S, Hd, ndir, c_save, hprev, hseq, hmean,
                                 mean_scale, hT, cT, pre, bsplit, (int)blockIdx.x,
                                 (int)blockIdx.y, (int)gridDim.x);
}

// ---------------------------------------------------------------------------------------------
// backward (reverse-time recurrence)
// ---------------------------------------------------------------------------------------------
// pre: the gate pre-activations, recomputed time-parallel after the forward by one GEMM
// (pre = x W_ih^T + h_{t-1} W_hh^T + b) instead of being stored per step by the forward kernel.
// MFMA output: lane (q, n) holds dh for units u0 + j (u0 = 16w + 4q, j = 0..3) of column n; as in
// the forward, the BR valid columns are redistributed: lane (q, r, b) owns units u0 + r + s*(16/BR).
template <int HD, int BR, bool DSEQ, int UG, typename PT = float>
__device__ __forceinline__ void
bwd_recur(const PT* __restrict__ pre,        // [B*S][ndir][4*HD] original time order
          const float* __restrict__ c_save,  // [ndir][Bp][S][HD]
          const bf16* __restrict__ whhT,     // [ndir][HD][4*HD]
          const float* __restrict__ dh_ext, long dh_sb, long dh_st, float dh_scale,
          const float* __restrict__ dhT, const float* __restrict__ dcT,  // optional [B][ndir*Hd]
          int B, int S, int Hd, int ndir,
          bf16* __restrict__ dpre,            // [Bp*S][ndir][4*HD] permuted, original time
          const int Bp,                       // rows of the forward's padded buffers (c_save)
          const int bx, const int dir) {
  constexpr int KS = 4 * HD / 32;
  constexpr int LDD = 4 * HD + 32;  // 16 dwords mod 64 banks: see LDH in the forward
  constexpr bool STREAM = HD > 192;  // W_hh^T streamed from L2 every step (see the forward)
  constexpr int NLK = (UG == 1 && !STREAM) ? LdsSplit<HD, BR>::BWD_KS : 0, NRK = KS - NLK;
  constexpr int NW = HD / (16 * UG);
  constexpr int NT = NW * 64;
  constexpr int G16 = 16 / BR, NSL1 = BR / 4, NSL = UG * NSL1;
  __shared__ __attribute__((aligned(16))) bf16 dbuf[2][16][LDD];
  __shared__ __attribute__((aligned(16))) bf16x8 wlds[NLK > 0 ? NW : 1][NLK > 0 ? NLK : 1][64];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q = lane >> 4, n = lane & 15, r = n / BR, bl = n % BR;
  const int b = bx * BR + bl;
  const bool vb = b < B;
  const int bc = vb ? b : B - 1;
  const long rowX = (long)ndir * 4 * HD;

  const __amdgpu_buffer_rsrc_t w_rs = dn_rsrc(whhT + (long)dir * HD * 4 * HD, (uint32_t)(4 * HD * HD * 2));
  const uint32_t wvo = (uint32_t)((UG * w * KS * 64 + lane) * 16);  // fragment-linear
  bf16x8 af[STREAM ? 1 : UG][STREAM ? 1 : NRK];
  constexpr int RS = !STREAM ? 1 : (UG == 1 ? 8 : (HD == 512 ? 2 : 4));  // weight ring (see the forward)
  static_assert(KS % RS == 0, "weight ring");
  bf16x8 wring[RS][UG];
  if constexpr (STREAM) {
#pragma unroll
    for (int ks = 0; ks + 1 < RS; ++ks)
#pragma unroll
      for (int g = 0; g < UG; ++g) wring[ks][g] = load_wfrag(w_rs, wvo, (g * KS + ks) * 1024);
  }
  if constexpr (!STREAM) {
    const bf16* wtl = whhT + (long)dir * HD * 4 * HD + (long)(16 * UG * w + n) * 4 * HD + 8 * q;
#pragma unroll
    for (int g = 0; g < UG; ++g)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(wtl + (long)16 * g * 4 * HD + 32 * ks);
        if (ks < NRK) af[g][ks < NRK ? ks : 0] = v;
        else wlds[w][ks - NRK][lane] = v;
      }
  }
  for (int i = tid; i < 2 * 16 * LDD; i += NT) (&dbuf[0][0][0])[i] = (bf16)0.f;

  int uu[NSL];
  float msk[NSL], dhx[NSL], dcc[NSL];
#pragma unroll
  for (int s = 0; s < NSL; ++s) {
    // slot (group s / NSL1, s1 = s % NSL1): unit offset r + s1*G16 of the group's lane quad
    const int u = 16 * (UG * w + s / NSL1) + 4 * q + r + (s % NSL1) * G16;
    uu[s] = u;
    msk[s] = (vb && u < Hd) ? 1.f : 0.f;
    const int uc = u < Hd ? u : Hd - 1;
    dhx[s] = DSEQ ? 0.f : dh_ext[(long)bc * dh_sb + dir * Hd + uc] * dh_scale * msk[s];
    dcc[s] = dcT ? dcT[(long)bc * ndir * Hd + dir * Hd + uc] * msk[s] : 0.f;
  }
  const PT* prow = pre + (long)bc * S * rowX + (long)dir * 4 * HD;
  const float* crow = c_save + (long)dir * Bp * S * HD + (long)b * S * HD;
  bf16* drow = dpre + (long)b * S * rowX + (long)dir * 4 * HD;
  const float* dhrow = dh_ext + (long)bc * dh_sb + dir * Hd;
  const int tauL = dir == 0 ? S - 1 : 0;
  const int tp0 = S >= 2 ? S - 2 : 0;
  const int tauP = dir == 0 ? tp0 : S - 1 - tp0;
  // pn: step t's gate pre-activations; ca / cb: c_t and c_{t-1}, alternating roles over a 2-step
  // unrolled loop.  Each step turns pn and c_t into gate activations FIRST (they need no MFMA
  // result), then reloads the same registers with step t-1's pre-activations and c_{t-2}: the
  // loads fly during this step's MFMAs and gate phase, and nothing copies a register that a load
  // is still filling (such a copy is a vmcnt wait at the end of the step)
  float ca[NSL], cb[NSL], dTl[NSL];
  typename Gate4Raw<PT>::type pn[NSL];  // (bf16 pre-activations stay packed until used)
#pragma unroll
  for (int s = 0; s < NSL; ++s) {
    const int uc = uu[s] < Hd ? uu[s] : Hd - 1;
    dTl[s] = dhT ? dhT[(long)bc * ndir * Hd + dir * Hd + uc] * msk[s] : 0.f;  // dL/dh_T
    ca[s] = crow[(long)tauL * HD + uu[s]];
    cb[s] = crow[(long)tauP * HD + uu[s]];
    pn[s] = load_raw4<PT>(prow + (long)tauL * rowX + 4 * uu[s], true);
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(DN_VMCNT0);  // resident weights landed (see the forward)

  int cur = 0;
#ifdef DN_STAMPS
  unsigned long long st_a = 0, st_b = 0, st_c = 0, ts0, ts1, ts2, ts3;
#endif
  auto step = [&](const int t, float (&ccur)[NSL], float (&cprv)[NSL]) {
    // nothing of a later step is scheduled above this point: hipcc otherwise hoists the next
    // step's gate math (which needs only the loads issued here) into this step's MFMA phase
    // and waits there for a load it has just issued
    __builtin_amdgcn_sched_barrier(0);
#ifdef DN_STAMPS
    STAMP(ts0);
#endif
    const int tau = dir == 0 ? t : S - 1 - t;
    const int t1 = t > 0 ? t - 1 : 0;
    const int tau1 = dir == 0 ? t1 : S - 1 - t1;
    const int t2 = t > 1 ? t - 2 : 0;
    const int tau2 = dir == 0 ? t2 : S - 1 - t2;
    float si[NSL], sf[NSL], so[NSL], gi[NSL], gf[NSL], go[NSL], gg[NSL], tc[NSL], cp[NSL];
    auto activations = [&]() {
#pragma unroll
      for (int s = 0; s < NSL; ++s) {
        const f32x4 pc = to_f32x4(pn[s]);
        cp[s] = t > 0 ? cprv[s] : 0.f;
        si[s] = dn_sigmoid(pc[0]); sf[s] = dn_sigmoid(pc[1]); so[s] = dn_sigmoid(pc[2]);
        gi[s] = sigmoid_unit(si[s]); gf[s] = sigmoid_unit(sf[s]); go[s] = sigmoid_unit(so[s]);
        gg[s] = dn_tanh(pc[3]);
        tc[s] = dn_tanh(ccur[s]);
        pn[s] = load_raw4<PT>(prow + (long)tau1 * rowX + 4 * uu[s], true);
        ccur[s] = crow[(long)tau2 * HD + uu[s]];
      }
    };
    // up to 2 gate slots per lane the activations are live across the MFMAs; at 4 (BR = 16)
    // they would spill, so they follow the MFMAs there
    constexpr bool HOIST = NSL <= 2;
    if constexpr (HOIST) activations();
    float dx[NSL];
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      dx[s] = dhx[s];
      if constexpr (DSEQ) {
        const int uc = uu[s] < Hd ? uu[s] : Hd - 1;
        dx[s] = dhrow[(long)t * dh_st + uc] * dh_scale * msk[s];
      }
      dx[s] += t == S - 1 ? dTl[s] : 0.f;  // select: no load in the loop
    }
    // K = 4*HD runs as BWD_CHAINS independent accumulator chains per unit group (summed after
    // the loop): one chain of 24 dependent MFMAs left the SIMD waiting on its own results
    constexpr int RG = BR != 4 ? 1 : ((DSEQ || HD == 192) ? (HD == 192 ? BWD_RG_192 : 2) : BWD_RG);
    // with the exchange-tile reads grouped ahead (RG > 1) one chain is fastest (192 / 4 rows:
    // 109.3 us vs 111.0 at 2 chains, 112.9 at 3, 114.8 at 4; tools/lstm_time.py)
    constexpr int NCH = (RG > 1 && !STREAM) ? 1 : BWD_CHAINS;
    f32x4 acc[UG], accp[UG][NCH];
#pragma unroll
    for (int g = 0; g < UG; ++g)
#pragma unroll
      for (int c = 0; c < NCH; ++c) accp[g][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (STREAM) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        __builtin_amdgcn_sched_barrier(0);
        constexpr int PD = RS - 1;
        const int kl = (ks + PD) % KS;
#pragma unroll
        for (int g = 0; g < UG; ++g)
          wring[(ks + PD) % RS][g] = load_wfrag(w_rs, wvo, (g * KS + kl) * 1024);
        const bf16x8 db = *reinterpret_cast<const bf16x8*>(&dbuf[cur][n % BR][32 * ks + 8 * q]);
#pragma unroll
        for (int g = 0; g < UG; ++g) accp[g][ks % NCH] = mfma16(wring[ks % RS][g], db, accp[g][ks % NCH]);
      }
    }
    // Resident weights: the exchange-tile (and LDS-resident weight) reads go in groups of RG
    // k-steps, group g+1 requested before group g's MFMAs (scheduling barriers pin the order).
    // Left to itself hipcc kept ONE read in flight -- ds_read, wait, MFMA for each of the 24
    // k-steps -- so the LDS latency, not the MFMA pipe, paced the step.
    // (4-row layout only: at 8 / 16 rows per workgroup the second register set spills; the
    // per-step output-gradient variant takes groups of 2 for the same reason)
    if constexpr (!STREAM && RG == 1) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        // see the forward: padded columns read (broadcast) a valid row; never consumed
        const bf16x8 db = *reinterpret_cast<const bf16x8*>(&dbuf[cur][n % BR][32 * ks + 8 * q]);
#pragma unroll
        for (int g = 0; g < UG; ++g)
          accp[g][ks % NCH] = mfma16(
              ks < NRK ? af[g][ks < NRK ? ks : 0] : wlds[w][ks < NRK ? 0 : ks - NRK][lane], db,
              accp[g][ks % NCH]);
      }
    }
    if constexpr (!STREAM && RG > 1) {
      static_assert(KS % RG == 0, "read groups");
      bf16x8 dg[2][RG], wg[2][RG];
      auto issue = [&](int k0, bf16x8 (&d)[RG], bf16x8 (&wv)[RG]) {
#pragma unroll
        for (int j = 0; j < RG; ++j) {
          // see the forward: padded columns read (broadcast) a valid row; never consumed
          d[j] = *reinterpret_cast<const bf16x8*>(&dbuf[cur][n % BR][32 * (k0 + j) + 8 * q]);
          if (k0 + j >= NRK) wv[j] = wlds[w][k0 + j >= NRK ? k0 + j - NRK : 0][lane];
        }
      };
      issue(0, dg[0], wg[0]);
#pragma unroll
      for (int k0 = 0; k0 < KS; k0 += RG) {
        const int cb = (k0 / RG) & 1;
        if (k0 + RG < KS) issue(k0 + RG, dg[cb ^ 1], wg[cb ^ 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < RG; ++j) {
          const int ks = k0 + j;
#pragma unroll
          for (int g = 0; g < UG; ++g)
            accp[g][ks % NCH] = mfma16(ks < NRK ? af[g][ks < NRK ? ks : 0] : wg[cb][j], dg[cb][j],
                                       accp[g][ks % NCH]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int g = 0; g < UG; ++g) {
      acc[g] = accp[g][0];
#pragma unroll
      for (int c = 1; c < NCH; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[g][j] += accp[g][c][j];
    }
    float dhr[NSL];
    if constexpr (BR == 16) {
#pragma unroll
      for (int s = 0; s < NSL; ++s) dhr[s] = acc[s / 4][s % 4];
    } else {
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl) {
        float v[G16];
#pragma unroll
        for (int g = 0; g < G16; ++g) v[g] = acc[sl / NSL1][g + (sl % NSL1) * G16];
        dhr[sl] = row_gather<BR>(v);
      }
    }
#ifdef DN_STAMPS
    { float z = dhr[0]; asm volatile("" :: "v"(z)); }
    STAMP(ts1);
#endif
    if constexpr (!HOIST) activations();
    const int nxt = cur ^ 1;
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      const float dh = dhr[s] + dx[s];
      const float dc = dcc[s] + dh * go[s] * (1.f - tc[s] * tc[s]);
      const float d_o = dh * tc[s];
      const float d_i = dc * gg[s], d_g = dc * gi[s], d_f = dc * cp[s];
      const float m = msk[s];
      dcc[s] = dc * gf[s] * m;
      bf16x4 e;
      e[0] = (bf16)(m * d_i * gi[s] * (1.f - gi[s]) * si[s] * (1.f - si[s]));
      e[1] = (bf16)(m * d_f * gf[s] * (1.f - gf[s]) * sf[s] * (1.f - sf[s]));
      e[2] = (bf16)(m * d_o * go[s] * (1.f - go[s]) * so[s] * (1.f - so[s]));
      e[3] = (bf16)(m * d_g * (1.f - gg[s] * gg[s]));
      *reinterpret_cast<bf16x4*>(&dbuf[nxt][bl][4 * uu[s]]) = e;
      *reinterpret_cast<bf16x4*>(drow + (long)tau * rowX + 4 * uu[s]) = e;
    }
#ifdef DN_STAMPS
    STAMP(ts2);
#endif
    __syncthreads();
#ifdef DN_STAMPS
    STAMP(ts3);
    st_a += ts1 - ts0; st_b += ts2 - ts1; st_c += ts3 - ts2;
#endif
    cur = nxt;
  };
  int t = S - 1;
  for (; t >= 1; t -= 2) {
    step(t, ca, cb);
    step(t - 1, cb, ca);
  }
  if (t >= 0) step(t, ca, cb);
#ifdef DN_STAMPS
  if (lane == 0 && bx == 0) {
    unsigned long long* o = dn_stamp_buf + (256 + dir * 64 + w) * 4;
    o[0] = st_a; o[1] = st_b; o[2] = st_c; o[3] = S;
  }
#endif
}

template <int HD, int BR, bool DSEQ, int UG, typename PT = float>
__global__ void __launch_bounds__(HD / (16 * UG) * 64)
lstm_bwd_kernel(const PT* __restrict__ pre, const float* __restrict__ c_save,
                const bf16* __restrict__ whhT, const float* __restrict__ dh_ext, long dh_sb,
                long dh_st, float dh_scale, const float* __restrict__ dhT,
                const float* __restrict__ dcT, int B, int S, int Hd, int ndir,
                bf16* __restrict__ dpre, int Bp) {
  bwd_recur<HD, BR, DSEQ, UG, PT>(pre, c_save, whhT, dh_ext, dh_sb, dh_st, dh_scale, dhT, dcT,
                                  B, S, Hd, ndir, dpre, Bp, (int)blockIdx.x, (int)blockIdx.y);
}

// ---------------------------------------------------------------------------------------------
// weight pack: reference layout ([i|f|o|g] rows, fp32) -> kernel layouts (bf16, m = 4u+g,
// units zero-padded to HD)
// ---------------------------------------------------------------------------------------------
struct LstmParams {
  const float* wih[2];
  const float* bih[2];
  const float* whh[2];
  const float* bhh[2];
};

// extra fp32 -> bf16 casts riding in the pack launch (e.g. the encoder weights, whose GEMM
// goes to hipBLASLt with bf16 operands): saves a launch at the head of every step
constexpr int PACK_CASTS = 4;
struct CastJobs {
  const float* src[PACK_CASTS];
  bf16* dst[PACK_CASTS];
  int n[PACK_CASTS];
  int cnt;
};

// Fragment-linear image of a row-major [rows][KS*32] bf16 matrix (the streamed-weight kernels,
// HD > 192): element f sits at ((T*KS + ks)*64 + lane)*8 + e for MFMA A-fragment lane
// (q = lane/16, n = lane%16) of 16-row tile T and k-step ks, i.e. row 16T + n, column
// 32ks + 8q + e -- every wave-wide 16-B fragment load reads 1 KiB contiguous.
__device__ __forceinline__ void frag_rc(int f, int KS, int& row, int& col) {
  const int e = f & 7, lane = (f >> 3) & 63, rest = f >> 9;
  const int ks = rest % KS, T = rest / KS;
  row = 16 * T + (lane & 15);
  col = 32 * ks + 8 * (lane >> 4) + e;
}

__global__ void lstm_pack_kernel(LstmParams p, int I, int Hd, int HD, int ndir,
                                 bf16* __restrict__ wih_p,    // [ndir*4HD][I]
                                 float* __restrict__ bias_p,  // [ndir*4HD]
                                 bf16* __restrict__ whh_p,    // [ndir][4HD][HD]
                                 bf16* __restrict__ whhT_p,   // [ndir][HD][4HD]
                                 CastJobs cj, StepPrologue sp) {
  if (sp.bump && blockIdx.x == 0 && threadIdx.x == 0) *sp.bump += 1;
  // 32-bit index math throughout (every extent < 2^31): 64-bit div/mod per element made this
  // ~1M-element repack a 6 us kernel at the head of every step
  const int GP = 4 * HD;
  const int n_wih = ndir * GP * I, n_b = ndir * GP, n_whh = ndir * GP * HD;
  const int n_pack = n_wih + n_b + 2 * n_whh;
  int n_pc = n_pack;
  for (int j = 0; j < cj.cnt; ++j) n_pc += cj.n[j];
  const long total = n_pc + sp.ux + sp.ug + sp.ny;
  const long cur = prologue_cursor(sp);
  for (long li = blockIdx.x * (long)blockDim.x + threadIdx.x; li < total;
       li += (long)gridDim.x * blockDim.x) {
    if (li >= n_pc) {  // step prologue
      prologue_item(sp, li - n_pc, cur);
      continue;
    }
    const int idx = (int)li;
    if (idx >= n_pack) {
      int r = idx - n_pack, j = 0;
      while (j + 1 < cj.cnt && r >= cj.n[j]) r -= cj.n[j++];
      cj.dst[j][r] = (bf16)cj.src[j][r];
    } else if (idx < n_wih) {
      const int r = idx / I, k = idx - r * I;
      const int d = r / GP, m = r - d * GP, u = m >> 2, g = m & 3;
      wih_p[idx] = (bf16)(u < Hd ? p.wih[d][(g * Hd + u) * I + k] : 0.f);
    } else if (idx < n_wih + n_b) {
      const int r = idx - n_wih;
      const int d = r / GP, m = r - d * GP, u = m >> 2, g = m & 3;
      float v = 0.f;
      if (u < Hd) {
        if (p.bih[d]) v += p.bih[d][g * Hd + u];
        if (p.bhh[d]) v += p.bhh[d][g * Hd + u];
      }
      bias_p[r] = v;
    } else if (idx < n_wih + n_b + n_whh) {
      const int r = idx - n_wih - n_b;  // [d][m][k], or fragment-linear (see frag_rc)
      int d, m, k;
      if (HD > 192) {
        d = r / (GP * HD);
        frag_rc(r - d * GP * HD, HD / 32, m, k);
      } else {
        const int dm = r / HD;
        k = r - dm * HD;
        d = dm / GP;
        m = dm - d * GP;
      }
      const int u = m >> 2, g = m & 3;
      whh_p[r] = (bf16)((u < Hd && k < Hd) ? p.whh[d][(g * Hd + u) * Hd + k] : 0.f);
    } else {
      const int r = idx - n_wih - n_b - n_whh;  // [d][k][m], or fragment-linear
      int d, m, k;
      if (HD > 192) {
        d = r / (GP * HD);
        frag_rc(r - d * GP * HD, GP / 32, k, m);
      } else {
        const int dk = r / GP;
        m = r - dk * GP;
        d = dk / HD;
        k = dk - d * HD;
      }
      const int u = m >> 2, g = m & 3;
      whhT_p[r] = (bf16)((u < Hd && k < Hd) ? p.whh[d][(g * Hd + u) * Hd + k] : 0.f);
    }
  }
}

// rows per workgroup: spread small batches over more CUs (the gate phase is VALU-bound per CU)
static inline int pick_br(int B, int HD) {
  // streamed-weight variants (HD > 192): 4 rows per workgroup keeps them spill-free at every
  // HD (8 / 16 rows spill above 256), and their step time is bound by the per-CU W stream,
  // which more rows per workgroup would not shorten
  if (HD > 192) return 4;
  if (const char* e = getenv("DN_LSTM_BR")) {
    const int v = atoi(e);
    if (v == 4 || v == 8 || v == 16) return v;
  }
  // measured per step (bench.py, MI355X, round 4 with bf16 stored pre-activations from 512 rows,
  // profiles/r4_lstm_rows_per_wg_ab.jsonl): B = 512: 4 rows 0.838 ms vs 8 rows 1.029; B = 1024:
  // 1.506 vs 1.522; B = 2048: 2.726 vs 2.784 / 2.807 (16 rows 2.907); B = 4096: 5.31 / 5.34 vs
  // 5.37 / 5.51; B = 8192: 10.61 vs 10.52 (both recurrences at one size).  With the backward at
  // 8 rows from B = 2048 (pick_br_bwd), a 4-row forward also wins at B = 8192: 10.21 / 10.20 vs
  // 10.41 / 10.44 ms (profiles/r4_lstm_bwd_rows_ab.jsonl)
  if (HD == 192) return 4;
  return B <= 4096 ? 4 : 8;
}

// rows per workgroup of the BACKWARD recurrence: the forward's, except at large batches of the
// resident 192-unit geometry, where 8 rows win for the backward alone (B = 2048 kernel trace:
// backward 462 us at 8 rows vs 513 at 4, forward 606 vs 450; profiles/r4_b2048_timeline.txt;
// step A/B in profiles/r4_lstm_bwd_rows_ab.jsonl: from B = 1024 on, 1.404 vs 1.433 ms there,
// while B = 512 loses, 0.869 vs 0.802, and B = 128 0.554 vs 0.466).
// The buffers are row-major over the batch, so the two launches may tile the rows differently
// as long as both tilings cover the padded batch exactly (B % 8 == 0).
static inline int pick_br_bwd(int B, int HD) {
  const int br = pick_br(B, HD);
  if (getenv("DN_LSTM_BR") || getenv("DN_LSTM_BR_BWD_SAME")) return br;
  static const int minb = [] {  // probe knob: smallest batch with the 8-row backward
    const char* e = getenv("DN_LSTM_BWD8_MINB");
    return e ? atoi(e) : 1024;
  }();
  return (HD == 192 && br == 4 && B >= minb && B % 8 == 0) ? 8 : br;
}

// unit groups per wave for (HD, BR) = (192, 4): 1 (12 waves, 3 per SIMD) unless
// DINUNET_LSTM_UG=3 asks for one wave per SIMD.  Measured on MI355X (tools/lstm_stamps.py): the
// one-wave layout runs 2.06 us/step fwd and bwd vs 1.19 / 1.46 -- a lone wave issues its 72
// MFMAs at ~2700 cycles (not 1152) and its 3 gate slots serialise (1400 cycles): the 3-wave
// layout's inter-wave overlap of MFMA, LDS and VALU work is worth more than the 3x fewer
// exchange-tile reads.
static int lstm_ug() {
  static const int ug = [] {
    const char* e = getenv("DINUNET_LSTM_UG");
    return (e && e[0] == '3') ? 3 : 1;
  }();
  return ug;
}

// bias layout of the current dn_lstm_fwd call (0: fused b_ih + b_hh; > 0: split, see the kernel),
// set by dn_lstm_fwd for the launchers below (host launches are issued from one thread)
int g_bias_split = 0;

template <int HD, int BR, int UG>
int launch_fwd_ug(const bf16* xp, const float* bias, const bf16* whh, int B, int S, int Hd, int ndir,
                  float* c_save, bf16* hprev, float* hseq, float* hmean, float mean_scale, float* hT,
                  float* cT, float* pre, int pre_bf16, hipStream_t st) {
  dim3 grid((B + BR - 1) / BR, ndir), block(HD / (16 * UG) * 64);
  if constexpr (HD == 192 && UG == 1) {
    if (pre_bf16 && !hseq) {  // bf16 pre-activations (dn_lstm_pre_bf16_used)
      hipLaunchKernelGGL((lstm_fwd_kernel<HD, BR, false, UG, bf16>), grid, block, 0, st, xp, bias,
                         whh, B, S, Hd, ndir, c_save, hprev, hseq, hmean, mean_scale, hT, cT,
                         reinterpret_cast<bf16*>(pre), g_bias_split);
      return dn_launch_status();
    }
  }
  if (hseq)
    hipLaunchKernelGGL((lstm_fwd_kernel<HD, BR, true, UG>), grid, block, 0, st, xp, bias, whh, B, S,
                       Hd, ndir, c_save, hprev, hseq, hmean, mean_scale, hT, cT, pre, g_bias_split);
  else
    hipLaunchKernelGGL((lstm_fwd_kernel<HD, BR, false, UG>), grid, block, 0, st, xp, bias, whh, B,
                       S, Hd, ndir, c_save, hprev, hseq, hmean, mean_scale, hT, cT, pre,
                       g_bias_split);
  return dn_launch_status();
}

template <int HD, int BR>
int launch_fwd_br(const bf16* xp, const float* bias, const bf16* whh, int B, int S, int Hd, int ndir,
                  float* c_save, bf16* hprev, float* hseq, float* hmean, float mean_scale, float* hT,
                  float* cT, float* pre, int pre_bf16, hipStream_t st) {
  if constexpr (HD == 192 && BR == 4) {
    if (lstm_ug() == 3)
      return launch_fwd_ug<HD, BR, 3>(xp, bias, whh, B, S, Hd, ndir, c_save, hprev, hseq, hmean,
                                      mean_scale, hT, cT, pre, pre_bf16, st);
  }
  if constexpr (HD > 256)  // streamed weights: 2 unit groups per wave keep the block <= 16 waves
    return launch_fwd_ug<HD, BR, 2>(xp, bias, whh, B, S, Hd, ndir, c_save, hprev, hseq, hmean,
                                    mean_scale, hT, cT, pre, pre_bf16, st);
  else return launch_fwd_ug<HD, BR, 1>(xp, bias, whh, B, S, Hd, ndir, c_save, hprev, hseq, hmean,
                                  mean_scale, hT, cT, pre, pre_bf16, st);
}

template <int HD>
int launch_fwd(int BR, const bf16* xp, const float* bias, const bf16* whh, int B, int S, int Hd,
               int ndir, float* c_save, bf16* hprev, float* hseq, float* hmean, float mean_scale,
               float* hT, float* cT, float* pre, int pre_bf16, hipStream_t st) {
  if (BR == 4) return launch_fwd_br<HD, 4>(xp, bias, whh, B, S, Hd, ndir, c_save, hprev, hseq, hmean, mean_scale, hT, cT, pre, pre_bf16, st);
  if constexpr (HD > 192) return DN_UNSUPPORTED;  // streamed variants: 4 rows only (pick_br)
  else {
  if (BR == 8) return launch_fwd_br<HD, 8>(xp, bias, whh, B, S, Hd, ndir, c_save, hprev, hseq, hmean, mean_scale, hT, cT, pre, pre_bf16, st);
  return launch_fwd_br<HD, 16>(xp, bias, whh, B, S, Hd, ndir, c_save, hprev, hseq, hmean, mean_scale, hT, cT, pre, pre_bf16, st);
  }
}

template <int HD, int BR, int UG>
int launch_bwd_ug(const float* pre, const float* c_save, const bf16* whhT, const float* dh_ext,
                  long sb, long st_, float scale, const float* dhT, const float* dcT, int B, int S,
                  int Hd, int ndir, bf16* dpre, int Bp, int pre_bf16, hipStream_t st) {
  dim3 grid((B + BR - 1) / BR, ndir), block(HD / (16 * UG) * 64);
  if constexpr (HD == 192 && UG == 1) {
    if (pre_bf16 && st_ == 0) {  // bf16 pre-activations (dn_lstm_pre_bf16_used)
      hipLaunchKernelGGL((lstm_bwd_kernel<HD, BR, false, UG, bf16>), grid, block, 0, st,
                         reinterpret_cast<const bf16*>(pre), c_save, whhT, dh_ext, sb, st_, scale,
                         dhT, dcT, B, S, Hd, ndir, dpre, Bp);
      return dn_launch_status();
    }
  }
  if (st_ != 0)
    hipLaunchKernelGGL((lstm_bwd_kernel<HD, BR, true, UG>), grid, block, 0, st, pre, c_save, whhT,
                       dh_ext, sb, st_, scale, dhT, dcT, B, S, Hd, ndir, dpre, Bp);
  else
    hipLaunchKernelGGL((lstm_bwd_kernel<HD, BR, false, UG>), grid, block, 0, st, pre, c_save, whhT,
                       dh_ext, sb, st_, scale, dhT, dcT, B, S, Hd, ndir, dpre, Bp);
  return dn_launch_status();
}

template <int HD, int BR>
int launch_bwd_br(const float* pre, const float* c_save, const bf16* whhT, const float* dh_ext,
                  long sb, long st_, float scale, const float* dhT, const float* dcT, int B, int S,
                  int Hd, int ndir, bf16* dpre, int Bp, int pre_bf16, hipStream_t st) {
  if constexpr (HD == 192 && BR == 4) {
    if (lstm_ug() == 3)
      return launch_bwd_ug<HD, BR, 3>(pre, c_save, whhT, dh_ext, sb, st_, scale, dhT, dcT, B, S,
                                      Hd, ndir, dpre, Bp, pre_bf16, st);
  }
  if constexpr (HD > 256)
    return launch_bwd_ug<HD, BR, 2>(pre, c_save, whhT, dh_ext, sb, st_, scale, dhT, dcT, B, S, Hd,
                                    ndir, dpre, Bp, pre_bf16, st);
  else return launch_bwd_ug<HD, BR, 1>(pre, c_save, whhT, dh_ext, sb, st_, scale, dhT, dcT, B, S, Hd,
                                  ndir, dpre, Bp, pre_bf16, st);
}

template <int HD>
int launch_bwd(int BR, const float* pre, const float* c_save, const bf16* whhT, const float* dh_ext,
               long sb, long st_, float scale, const float* dhT, const float* dcT, int B, int S,
               int Hd, int ndir, bf16* dpre, int Bp, int pre_bf16, hipStream_t st) {
  if (BR == 4) return launch_bwd_br<HD, 4>(pre, c_save, whhT, dh_ext, sb, st_, scale, dhT, dcT, B, S, Hd, ndir, dpre, Bp, pre_bf16, st);
  if constexpr (HD > 192) return DN_UNSUPPORTED;
  else {
  if (BR == 8) return launch_bwd_br<HD, 8>(pre, c_save, whhT, dh_ext, sb, st_, scale, dhT, dcT, B, S, Hd, ndir, dpre, Bp, pre_bf16, st);
  return launch_bwd_br<HD, 16>(pre, c_save, whhT, dh_ext, sb, st_, scale, dhT, dcT, B, S, Hd, ndir, dpre, Bp, pre_bf16, st);
  }
}

}  // namespace

// padded per-direction hidden the kernels are instantiated for
DN_API int dn_lstm_padded_hidden(int Hd) {
  if (Hd <= 0) return 0;
  if (Hd <= 64) return 64;
  if (Hd <= 128) return 128;
  if (Hd <= 192) return 192;
  // above 192 the recurrent weights no longer fit the register file: streamed variants
  if (Hd <= 256) return 256;
  if (Hd <= 384) return 384;
  if (Hd <= 512) return 512;
  return 0;
}

static int lstm_pack_launch(const float* wih0, const float* bih0, const float* whh0,
                            const float* bhh0, const float* wih1, const float* bih1,
                            const float* whh1, const float* bhh1, int I, int Hd, int ndir,
                            void* wih_p, float* bias_p, void* whh_p, void* whhT_p, int ncast,
                            const float* const* cast_src, void* const* cast_dst,
                            const int* cast_n, const StepPrologue& sp, hipStream_t st) {
  const int HD = dn_lstm_padded_hidden(Hd);
  if (!HD || ndir < 1 || ndir > 2 || ncast < 0 || ncast > PACK_CASTS) return DN_BAD_SHAPE;
  LstmParams p{{wih0, wih1}, {bih0, bih1}, {whh0, whh1}, {bhh0, bhh1}};
  CastJobs cj{};
  cj.cnt = ncast;
  long total = ndir * 4L * HD * I + ndir * 4L * HD + 2L * ndir * 4 * HD * HD;
  for (int j = 0; j < ncast; ++j) {
    if (cast_n[j] <= 0) return DN_BAD_SHAPE;
    cj.src[j] = cast_src[j];
    cj.dst[j] = (bf16*)cast_dst[j];
    cj.n[j] = cast_n[j];
    total += cast_n[j];
  }
  if (total >= (1L << 31)) return DN_BAD_SHAPE;
  total += sp.ux + sp.ug + sp.ny;
  // the batch conversion is HBM-bound: as many workgroups as the standalone prologue had
  const long cap = sp.ux ? 4096 : 2048;
  const int blocks = (int)((total + 255) / 256 < cap ? (total + 255) / 256 : cap);
  hipLaunchKernelGGL(lstm_pack_kernel, dim3(blocks), dim3(256), 0, st, p, I, Hd, HD, ndir,
                     (bf16*)wih_p, bias_p, (bf16*)whh_p, (bf16*)whhT_p, cj, sp);
  return dn_launch_status();
}

DN_API int dn_lstm_pack(const float* wih0, const float* bih0, const float* whh0, const float* bhh0,
                        const float* wih1, const float* bih1, const float* whh1, const float* bhh1,
                        int I, int Hd, int ndir, void* wih_p, float* bias_p, void* whh_p,
                        void* whhT_p, int ncast, const float* const* cast_src,
                        void* const* cast_dst, const int* cast_n, hipStream_t st) {
  const StepPrologue sp{};
  return lstm_pack_launch(wih0, bih0, whh0, bhh0, wih1, bih1, whh1, bhh1, I, Hd, ndir, wih_p,
                          bias_p, whh_p, whhT_p, ncast, cast_src, cast_dst, cast_n, sp, st);
}

// dn_lstm_pack + dn_step_prologue in ONE launch (x: nx fp32 -> xb bf16, nx % 8 == 0; y: ny int64
// -> yd; g: ng floats zeroed, ng % 4 == 0; 16-B aligned x, xb, g; bump: Adam's device step
// counter advanced once, or null)
DN_API int dn_lstm_pack_prologue(const float* wih0, const float* bih0, const float* whh0,
                                 const float* bhh0, const float* wih1, const float* bih1,
                                 const float* whh1, const float* bhh1, int I, int Hd, int ndir,
                                 void* wih_p, float* bias_p, void* whh_p, void* whhT_p, int ncast,
                                 const float* const* cast_src, void* const* cast_dst,
                                 const int* cast_n, const float* x, long nx, void* xb,
                                 const long long* y, long ny, long long* yd, float* g, long ng,
                                 int* bump, hipStream_t st) {
  if (nx % 8 || ng % 4 || (((uintptr_t)x | (uintptr_t)xb | (uintptr_t)g) & 15)) return DN_BAD_SHAPE;
  StepPrologue sp{};
  sp.x = x;
  sp.xb = (bf16*)xb;
  sp.y = y;
  sp.yd = yd;
  sp.g = g;
  sp.ux = nx / 8;
  sp.ug = ng / 4;
  sp.ny = ny;
  sp.bump = bump;
  return lstm_pack_launch(wih0, bih0, whh0, bhh0, wih1, bih1, whh1, bhh1, I, Hd, ndir, wih_p,
                          bias_p, whh_p, whhT_p, ncast, cast_src, cast_dst, cast_n, sp, st);
}

// dn_lstm_pack + the DEVICE-FED step prologue (prologue.h) in one launch: batch rows gathered
// from the HBM-resident dataset gx ([N][row_elems], bf16 if gx_bf16 else fp32) at the device
// cursor, labels from gy, gradient zeroed, Adam's counter advanced
DN_API int dn_lstm_pack_gather(const float* wih0, const float* bih0, const float* whh0,
                               const float* bhh0, const float* wih1, const float* bih1,
                               const float* whh1, const float* bhh1, int I, int Hd, int ndir,
                               void* wih_p, float* bias_p, void* whh_p, void* whhT_p, int ncast,
                               const float* const* cast_src, void* const* cast_dst,
                               const int* cast_n, const void* gx, int gx_bf16, long row_elems,
                               const long long* gy, const long long* order, long nb,
                               const long long* cursor, int B, void* xb, long long* yd, float* g,
                               long ng, int* bump, hipStream_t st) {
  StepPrologue sp;
  const int rc = prologue_gather(sp, gx, gx_bf16, row_elems, gy, order, nb, cursor, B, xb, yd, g,
                                 ng, bump);
  if (rc != DN_OK) return rc;
  return lstm_pack_launch(wih0, bih0, whh0, bhh0, wih1, bih1, whh1, bhh1, I, Hd, ndir, wih_p,
                          bias_p, whh_p, whhT_p, ncast, cast_src, cast_dst, cast_n, sp, st);
}


// the forward's per-workgroup buffer descriptors span BR rows (32-bit offsets); the backward
// addresses with 64-bit pointers.  Only a single sequence longer than the descriptors can hold
// (BR * S * ndir * 4 * HD * 4 >= 2 GiB, S in the millions) is refused.
static bool lstm_fits_32bit(int B, int S, int HD, int ndir, int BR) {
  (void)B;
  return (long)BR * S * ndir * 4 * HD * 4 < (1L << 31);
}

// Can dn_lstm_fwd / dn_lstm_bwd keep the gate pre-activations in bf16 (their pre_bf16 argument)?
// Where the kernels offer it: per-direction hidden padded to 192 units, one unit group per wave,
// temporal-mean output.  The caller allocates the pre buffer accordingly.
DN_API int dn_lstm_pre_bf16_used(int Hd, int seq) {
  return dn_lstm_padded_hidden(Hd) == 192 && lstm_ug() == 1 && !seq;
}

// rows per workgroup the kernels use for batch B; internal buffers need Bp = ceil(B/BR)*BR rows
DN_API int dn_lstm_rows_per_wg(int B, int Hd) { return pick_br(B, dn_lstm_padded_hidden(Hd)); }
// rows per workgroup of the backward recurrence (pick_br_bwd; the buffers are padded to the
// forward's dn_lstm_rows_per_wg)
DN_API int dn_lstm_rows_per_wg_bwd(int B, int Hd) {
  return pick_br_bwd(B, dn_lstm_padded_hidden(Hd));
}

// xp: the bf16 input projection [B*S][ndir][4*HD]; pre (fp32, same layout, or null when no
// backward follows) receives the gate pre-activations (+ bias) the backward consumes
// bias_split > 0: `bias` is [2][ndir*4HD] (b_ih image, then b_hh image at offset bias_split, the
// form the fused Adam keeps packed: optim.hip adam_pack_kernel); 0: the fused sum of dn_lstm_pack
DN_API int dn_lstm_fwd(const void* xp, const float* bias, const void* whh_p, int B, int S, int Hd,
                       int ndir, float* c_save, void* hprev, float* hseq, float* hmean,
                       float mean_scale, float* hT, float* cT, float* pre, int bias_split,
                       int pre_bf16, hipStream_t st) {
  const int HD = dn_lstm_padded_hidden(Hd);
  if (!HD || B <= 0 || S <= 0 || ndir < 1 || ndir > 2) return DN_BAD_SHAPE;
  if (bias_split != 0 && bias_split != ndir * 4 * HD) return DN_BAD_SHAPE;
  // pre_bf16: `pre` is bf16 -- allowed only where dn_lstm_pre_bf16_used (a bf16 buffer the kernel
  // would fill in fp32 is refused, not overrun)
  if (pre_bf16 && !dn_lstm_pre_bf16_used(Hd, hseq != nullptr)) return DN_BAD_SHAPE;
  g_bias_split = bias_split;
  const int BR = pick_br(B, HD);
  if (!lstm_fits_32bit(B, S, HD, ndir, BR)) return DN_BAD_SHAPE;
  switch (HD) {
    case 64: return launch_fwd<64>(BR, (const bf16*)xp, bias, (const bf16*)whh_p, B, S, Hd, ndir, c_save, (bf16*)hprev, hseq, hmean, mean_scale, hT, cT, pre, pre_bf16, st);
    case 128: return launch_fwd<128>(BR, (const bf16*)xp, bias, (const bf16*)whh_p, B, S, Hd, ndir, c_save, (bf16*)hprev, hseq, hmean, mean_scale, hT, cT, pre, pre_bf16, st);
    case 192: return launch_fwd<192>(BR, (const bf16*)xp, bias, (const bf16*)whh_p, B, S, Hd, ndir, c_save, (bf16*)hprev, hseq, hmean, mean_scale, hT, cT, pre, pre_bf16, st);
    case 256: return launch_fwd<256>(BR, (const bf16*)xp, bias, (const bf16*)whh_p, B, S, Hd, ndir, c_save, (bf16*)hprev, hseq, hmean, mean_scale, hT, cT, pre, pre_bf16, st);
    case 384: return launch_fwd<384>(BR, (const bf16*)xp, bias, (const bf16*)whh_p, B, S, Hd, ndir, c_save, (bf16*)hprev, hseq, hmean, mean_scale, hT, cT, pre, pre_bf16, st);
    case 512: return launch_fwd<512>(BR, (const bf16*)xp, bias, (const bf16*)whh_p, B, S, Hd, ndir, c_save, (bf16*)hprev, hseq, hmean, mean_scale, hT, cT, pre, pre_bf16, st);
  }
  return DN_UNSUPPORTED;
}

DN_API int dn_lstm_bwd(const float* pre, const float* c_save, const void* whhT_p,
                       const float* dh_ext, long dh_sb, long dh_st, float dh_scale,
                       const float* dhT, const float* dcT, int B, int S, int Hd, int ndir,
                       void* dpre, int Bp, int pre_bf16, hipStream_t st) {
  // Bp: padded rows of the FORWARD's buffers (c_save [ndir][Bp][S][HD], dpre [Bp*S][...]): the
  // backward may tile the batch with other rows per workgroup (pick_br_bwd) but addresses the
  // forward's layout; pre_bf16 as in dn_lstm_fwd
  const int HD = dn_lstm_padded_hidden(Hd);
  if (!HD || B <= 0 || S <= 0 || ndir < 1 || ndir > 2 || Bp < B) return DN_BAD_SHAPE;
  if (pre_bf16 && !dn_lstm_pre_bf16_used(Hd, dh_st != 0)) return DN_BAD_SHAPE;
  int BR = pick_br_bwd(B, HD);
  if ((B + BR - 1) / BR * BR > Bp) BR = pick_br(B, HD);  // past the buffers: the forward's tiling
  if ((B + BR - 1) / BR * BR > Bp) return DN_BAD_SHAPE;
  if (!lstm_fits_32bit(B, S, HD, ndir, BR)) return DN_BAD_SHAPE;
  switch (HD) {
    case 64: return launch_bwd<64>(BR, pre, c_save, (const bf16*)whhT_p, dh_ext, dh_sb, dh_st, dh_scale, dhT, dcT, B, S, Hd, ndir, (bf16*)dpre, Bp, pre_bf16, st);
    case 128: return launch_bwd<128>(BR, pre, c_save, (const bf16*)whhT_p, dh_ext, dh_sb, dh_st, dh_scale, dhT, dcT, B, S, Hd, ndir, (bf16*)dpre, Bp, pre_bf16, st);
    case 192: return launch_bwd<192>(BR, pre, c_save, (const bf16*)whhT_p, dh_ext, dh_sb, dh_st, dh_scale, dhT, dcT, B, S, Hd, ndir, (bf16*)dpre, Bp, pre_bf16, st);
    case 256: return launch_bwd<256>(BR, pre, c_save, (const bf16*)whhT_p, dh_ext, dh_sb, dh_st, dh_scale, dhT, dcT, B, S, Hd, ndir, (bf16*)dpre, Bp, pre_bf16, st);
    case 384: return launch_bwd<384>(BR, pre, c_save, (const bf16*)whhT_p, dh_ext, dh_sb, dh_st, dh_scale, dhT, dcT, B, S, Hd, ndir, (bf16*)dpre, Bp, pre_bf16, st);
    case 512: return launch_bwd<512>(BR, pre, c_save, (const bf16*)whhT_p, dh_ext, dh_sb, dh_st, dh_scale, dhT, dcT, B, S, Hd, ndir, (bf16*)dpre, Bp, pre_bf16, st);
  }
  return DN_UNSUPPORTED;
}

