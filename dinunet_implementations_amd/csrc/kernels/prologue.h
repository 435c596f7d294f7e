// The training step's prologue (runtime.step.TrainStep): batch -> the graph's bf16 static input,
// labels -> the static label buffer, the flat gradient zeroed, Adam's device step counter
// advanced.  It rides in the first launch of a step (the LSTM weight pack, lstm.hip) or runs as a
// launch of its own (elementwise.hip).
//
// Two batch sources:
//   host-fed  (gx == null): x fp32 [ux * 8] -> xb, y [ny] -> yd (the caller's batch tensors);
//   device-fed (gx != null): the batch is gathered from a dataset RESIDENT in HBM, gx [N][f8 * 8]
//       (bf16, or fp32 when gx_bf16 == 0; gx_bf16 == 2: fp32 copied to an fp32 static input
//       unrounded -- the FS features), labels gy [N]; sample b of this step is row
//       order[c * B + b] (or c * B + b without an order) where c = *cursor mod nb.  Nothing in
//       the step reads the host, so K steps can be captured in one HIP graph.  The cursor is
//       advanced by the step's Adam launch (optim.hip), never here: every workgroup of this
//       launch reads it.  With `sd` the step's dataset row (subject) indices go there too, and
//       xb may be null: the GEMMs then read the batch rows from the dataset through them
//       (gemm.hip GemmProb::gx, the Adam-emitted pack at large batch: no batch copy).
#pragma once
#include "common.h"

struct StepPrologue {
  const float* x;
  bf16* xb;
  const long long* y;
  long long* yd;
  float* g;
  long ux, ug, ny;  // 8-element batch units, 4-element gradient units, labels
  int* bump;        // Adam's device step counter (graph-captured update), advanced once; null: none
  const void* gx;   // device-fed dataset (null: host-fed)
  const long long* gy;
  const long long* order;
  const long long* cursor;
  long nb;          // batches per pass over `order` (the cursor wraps)
  int f8, B, gx_bf16;
  long long* sd;    // optional [B]: the batch's dataset rows (device-fed only)
};

// the dataset row of sample b at cursor batch c
__device__ __forceinline__ long prologue_row(const StepPrologue& sp, long c, int b) {
  const long j = c * sp.B + b;
  return sp.order ? sp.order[j] : j;
}

// work item i of the prologue (i < ux + ug + ny); c = *cursor % nb (device-fed only)
__device__ __forceinline__ void prologue_item(const StepPrologue& sp, long i, long c) {
  if (i < sp.ux) {
    bf16x8 o;
    if (sp.gx) {
      const int ii = (int)i, b = ii / sp.f8, e = ii - b * sp.f8;  // ux < 2^31 (host-checked)
      const long r = prologue_row(sp, c, b);
      if (sp.gx_bf16 == 2) {
        const f32x4* s = reinterpret_cast<const f32x4*>(sp.gx) + 2 * (r * sp.f8 + e);
        f32x4* d = reinterpret_cast<f32x4*>(sp.xb) + 2 * i;
        d[0] = s[0];
        d[1] = s[1];
        return;
      }
      if (sp.gx_bf16) {
        o = reinterpret_cast<const bf16x8*>(sp.gx)[r * sp.f8 + e];
      } else {
        const f32x4* s = reinterpret_cast<const f32x4*>(sp.gx) + 2 * (r * sp.f8 + e);
        const f32x4 a = s[0], bq = s[1];
#pragma unroll
        for (int k = 0; k < 4; ++k) { o[k] = (bf16)a[k]; o[4 + k] = (bf16)bq[k]; }
      }
    } else {
      const f32x4 a = reinterpret_cast<const f32x4*>(sp.x)[2 * i];
      const f32x4 bq = reinterpret_cast<const f32x4*>(sp.x)[2 * i + 1];
#pragma unroll
      for (int k = 0; k < 4; ++k) { o[k] = (bf16)a[k]; o[4 + k] = (bf16)bq[k]; }
    }
    reinterpret_cast<bf16x8*>(sp.xb)[i] = o;
  } else if ((i -= sp.ux) < sp.ug) {
    reinterpret_cast<f32x4*>(sp.g)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
    i -= sp.ug;
    const long r = sp.gx ? prologue_row(sp, c, (int)i) : 0;
    sp.yd[i] = sp.gx ? sp.gy[r] : sp.y[i];
    if (sp.sd) sp.sd[i] = r;
  }
}

__device__ __forceinline__ long prologue_cursor(const StepPrologue& sp) {
  return sp.gx ? (*sp.cursor % sp.nb) : 0;
}

// host-side checks + packing of a device-fed prologue (0 = ok)
static inline int prologue_gather(StepPrologue& sp, const void* gx, int gx_bf16, long row_elems,
                                  const long long* gy, const long long* order, long nb,
                                  const long long* cursor, int B, void* xb, long long* yd, float* g,
                                  long ng, int* bump, long long* sd = nullptr) {
  if (!gx || !gy || !cursor || !(xb || sd) || !yd || B <= 0 || nb <= 0 || row_elems <= 0)
    return DN_BAD_SHAPE;
  if (row_elems % 8 || ng % 4) return DN_BAD_SHAPE;
  if (((uintptr_t)gx | (uintptr_t)xb | (uintptr_t)g) & 15) return DN_BAD_SHAPE;
  if ((long)B * (row_elems / 8) >= (1L << 31)) return DN_BAD_SHAPE;
  sp = StepPrologue{};
  sp.xb = (bf16*)xb;
  sp.yd = yd;
  sp.g = g;
  sp.ux = xb ? (long)B * (row_elems / 8) : 0;  // no xb: the rows only (sd)
  sp.sd = sd;
  sp.ug = ng / 4;
  sp.ny = B;
  sp.bump = bump;
  sp.gx = gx;
  sp.gy = gy;
  sp.order = order;
  sp.cursor = cursor;
  sp.nb = nb;
  sp.f8 = (int)(row_elems / 8);
  sp.B = B;
  sp.gx_bf16 = gx_bf16;
  return DN_OK;
}
