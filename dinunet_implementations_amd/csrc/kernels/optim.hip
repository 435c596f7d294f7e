// Fused optimizer kernels over ONE flat fp32 parameter buffer (all of a model's tensors are views
// into it), so a whole optimizer step is a single launch regardless of the parameter count.
#include "common.h"
#include "prologue.h"

namespace {

// torch.optim.Adam semantics (L2 weight decay, no amsgrad):
//   g += wd * p;  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2
//   p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
// grad_scale folds the dSGD mean (1/world) or loss scaling into the same pass.
__global__ void __launch_bounds__(256)
adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
            float* __restrict__ v, long n, float lr, float b1, float b2, float eps, float wd,
            float bc1, float inv_sqrt_bc2, float grad_scale, const int* __restrict__ tdev,
            double b1d, double b2d, int tofs, long long* __restrict__ cursor) {
  // the device-fed batch cursor (prologue.h) advances once per update; no workgroup of this
  // launch reads it
  if (cursor && blockIdx.x == 0 && threadIdx.x == 0) *cursor += 1;
  if (tdev) {  // graph-replayable form: the step number lives on the device (adam_bump_kernel);
               // double math as on the host, so both forms round to the same fp32 corrections
    const double t = (double)(*tdev + tofs);  // tofs 0: the step prologue advanced it
    bc1 = (float)(1.0 - pow(b1d, t));
    inv_sqrt_bc2 = (float)(1.0 / sqrt(1.0 - pow(b2d, t)));
  }
  const long n4 = n >> 2;
  const float step = lr / bc1;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float gr = gg[e] * grad_scale + wd * pp[e];
      mm[e] = b1 * mm[e] + (1.f - b1) * gr;
      vv[e] = b2 * vv[e] + (1.f - b2) * gr * gr;
      pp[e] -= step * mm[e] / (sqrtf(vv[e]) * inv_sqrt_bc2 + eps);
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
  }
  // scalar tail
  const long t = (n4 << 2) + blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) {
    float gr = g[t] * grad_scale + wd * p[t];
    m[t] = b1 * m[t] + (1.f - b1) * gr;
    v[t] = b2 * v[t] + (1.f - b2) * gr * gr;
    p[t] -= step * m[t] / (sqrtf(v[t]) * inv_sqrt_bc2 + eps);
  }
}


// ---------------------------------------------------------------------------------------------
// Fused Adam that also emits the NEXT step's operands: every updated
// parameter element is written, rounded to bf16, straight into the packed images the step's
// kernels read (the LSTM W_ih / W_hh / W_hh^T kernel layouts, the encoder's bf16 weight copy) and
// the split LSTM bias images (b_ih, b_hh: dn_lstm_fwd bias_split); the gradient is zeroed as it is
// consumed; and the next step's batch is gathered from the HBM-resident dataset at cursor + gofs
// (prologue.h).  The step then starts at its encoder GEMM, which advances the step counter and the
// cursor (gemm.hip group_bump): this launch READS both, so it cannot advance them itself.
// update = 0: pack + gather only (priming the persistent images before the first such step).
enum PackKind { PK_NONE = 0, PK_CAST = 1, PK_WIH = 2, PK_WHH = 3, PK_BIAS = 4 };
constexpr int PACK_SEGS = 16;
struct PackSeg {
  long off;    // flat offset, multiple of 4
  int n;       // elements (reference layout)
  int kind, d; // PackKind, LSTM direction
  void* dst;   // bf16 image (CAST / WIH / WHH), fp32 image (BIAS)
  void* dst2;  // WHH: the W_hh^T image
};
struct PackPlan {
  PackSeg s[PACK_SEGS];
  int cnt;
  int I, Hd, HD;  // LSTM input size, hidden, padded hidden
};

// fragment-linear position of (row, col) in a [rows][KS*32] image (lstm.hip frag_rc inverse)
__device__ __forceinline__ int frag_index(int row, int col, int KS) {
  const int T = row >> 4, n = row & 15, ks = col >> 5, q = (col >> 3) & 3, e = col & 7;
  return ((T * KS + ks) * 64 + q * 16 + n) * 8 + e;
}

__device__ __forceinline__ void pack_store(const PackPlan& pl, const PackSeg& sg, int j, float v) {
  const int GP = 4 * pl.HD;
  switch (sg.kind) {
    case PK_CAST:
      reinterpret_cast<bf16*>(sg.dst)[j] = (bf16)v;
      break;
    case PK_WIH: {
      const int row = j / pl.I, k = j - row * pl.I;
      const int g = row / pl.Hd, u = row - g * pl.Hd;
      reinterpret_cast<bf16*>(sg.dst)[(sg.d * GP + 4 * u + g) * pl.I + k] = (bf16)v;
      break;
    }
    case PK_WHH: {
      const int row = j / pl.Hd, k = j - row * pl.Hd;
      const int g = row / pl.Hd, u = row - g * pl.Hd, m = 4 * u + g;
      const int base = sg.d * GP * pl.HD;
      int a, b;
      if (pl.HD > 192) {
        a = frag_index(m, k, pl.HD / 32);
        b = frag_index(k, m, GP / 32);
      } else {
        a = m * pl.HD + k;
        b = k * GP + m;
      }
      reinterpret_cast<bf16*>(sg.dst)[base + a] = (bf16)v;
      reinterpret_cast<bf16*>(sg.dst2)[base + b] = (bf16)v;
      break;
    }
    case PK_BIAS: {
      const int g = j / pl.Hd, u = j - g * pl.Hd;
      reinterpret_cast<float*>(sg.dst)[sg.d * GP + 4 * u + g] = v;
      break;
    }
    default: break;
  }
}

// 4 consecutive elements j0 .. j0 + 3 of one segment (j0 % 4 == 0, j0 + 3 < sg.n): one index
// decode per thread and one 8-byte store wherever the destination keeps them consecutive (the
// cast images, W_ih rows, the W_hh row image; the transposed W_hh image stays per element) --
// per element, each with its integer divisions and a 2-byte store, the packing was ~6.4 of the
// launch's 14.5 us at B = 32 (profiles/r6_adam_pack_probe.txt).  Same values as pack_store.
__device__ __forceinline__ void pack_store4(const PackPlan& pl, const PackSeg& sg, int j0,
                                            const f32x4& v) {
  const int GP = 4 * pl.HD;
  bf16x4 h;
#pragma unroll
  for (int e = 0; e < 4; ++e) h[e] = (bf16)v[e];
  const bool a8 = (((uintptr_t)sg.dst) & 7) == 0;
  switch (sg.kind) {
    case PK_CAST:
      if (a8) {
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(sg.dst) + j0) = h;
        return;
      }
      break;
    case PK_WIH:
      if (a8 && (pl.I & 3) == 0) {
        const int row = j0 / pl.I, k = j0 - row * pl.I;
        const int g = row / pl.Hd, u = row - g * pl.Hd;
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(sg.dst) +
                                   (long)(sg.d * GP + 4 * u + g) * pl.I + k) = h;
        return;
      }
      break;
    case PK_WHH:
      if (a8 && pl.HD <= 192 && (pl.Hd & 3) == 0 && (pl.HD & 3) == 0) {
        const int row = j0 / pl.Hd, k = j0 - row * pl.Hd;
        const int g = row / pl.Hd, u = row - g * pl.Hd, m = 4 * u + g;
        const int base = sg.d * GP * pl.HD;
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(sg.dst) + base + m * pl.HD + k) = h;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          reinterpret_cast<bf16*>(sg.dst2)[base + (k + e) * GP + m] = h[e];
        return;
      }
      break;
    default:
      break;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) pack_store(pl, sg, j0 + e, v[e]);
}

// Per-step train-metric record of a device-fed epoch (runtime.feed.DeviceFeed): the step's score
// column out[b][col] (ICA: prob[:, 1], reference comps/icalstm/__init__.py:64-65) and its loss
// land in rings indexed by the batch cursor, so an epoch of K-step graph replays yields the exact
// per-sample (score, label) pairs for the train AUC and the per-step losses for the train average
// with no host work between steps.  Slot c = (*cursor + cofs) mod n.
struct StepRecord {
  const float* out;
  long ld;
  int col, B;
  const float* loss;
  float* rs;  // [n][B] scores
  float* rl;  // [n] losses
  long n;
  const long long* cursor;
  const long long* pred;  // col < 0: the score is the predicted class (FS: hard labels)
};

__device__ __forceinline__ void record_step(const StepRecord& r, int cofs) {
  long c = (*r.cursor + cofs) % r.n;
  if (c < 0) c += r.n;
  for (int b = threadIdx.x; b < r.B; b += blockDim.x)
    r.rs[c * r.B + b] = r.col < 0 ? (float)r.pred[b] : r.out[b * r.ld + r.col];
  if (threadIdx.x == 0) r.rl[c] = *r.loss;
}

__global__ void __launch_bounds__(256) record_kernel(StepRecord r, int cofs) { record_step(r, cofs); }

__global__ void __launch_bounds__(256)
adam_pack_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                 float* __restrict__ v, long n, float lr, float b1, float b2, float eps, float wd,
                 float grad_scale, const int* __restrict__ tdev, double b1d, double b2d, int update,
                 int zero_grad, PackPlan pl, StepPrologue sp, int gofs, int ublocks, StepRecord rec) {
  // the step's train record (rec.out set): the LAST workgroup; the cursor was advanced by this
  // step's encoder GEMM, so it names the batch this step trained on
  if (rec.out && blockIdx.x == gridDim.x - 1) {
    record_step(rec, 0);
    return;
  }
  // blocks [0, ublocks) update the parameters (one float4 per thread and round), the rest gather
  // the next batch: no divergent work mix inside a wave, every load of a round issued at once
  if ((int)blockIdx.x >= ublocks) {
    const long c = (*sp.cursor + gofs) % sp.nb;
    const long ng = sp.ux + sp.ny;
    const long stride = (long)(gridDim.x - ublocks - (rec.out ? 1 : 0)) * blockDim.x;
    for (long i = (blockIdx.x - ublocks) * (long)blockDim.x + threadIdx.x; i < ng; i += stride)
      prologue_item(sp, i, c);  // sp.ug == 0: the zeroing rides in the update below
    return;
  }
  float bc1 = 1.f, inv_sqrt_bc2 = 1.f;
  if (update) {  // the encoder GEMM of this step advanced *tdev (prebumped form)
    const double t = (double)(*tdev);
    bc1 = (float)(1.0 - pow(b1d, t));
    inv_sqrt_bc2 = (float)(1.0 / sqrt(1.0 - pow(b2d, t)));
  }
  const float step = lr / bc1;
  const long n4 = n >> 2, stride = (long)ublocks * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    if (update) {
      const f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
      f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
      f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float gr = gg[e] * grad_scale + wd * pp[e];
        mm[e] = b1 * mm[e] + (1.f - b1) * gr;
        vv[e] = b2 * vv[e] + (1.f - b2) * gr * gr;
        pp[e] -= step * mm[e] / (sqrtf(vv[e]) * inv_sqrt_bc2 + eps);
      }
      reinterpret_cast<f32x4*>(p)[i] = pp;
      reinterpret_cast<f32x4*>(m)[i] = mm;
      reinterpret_cast<f32x4*>(v)[i] = vv;
    }
    if (zero_grad) reinterpret_cast<f32x4*>(g)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const long e0 = i << 2;
    int s = 0;
    while (s < pl.cnt && e0 >= pl.s[s].off + pl.s[s].n) ++s;
    if (s < pl.cnt && e0 >= pl.s[s].off) {
      const PackSeg& sg = pl.s[s];
      const int j0 = (int)(e0 - sg.off);
      if (j0 + 4 <= sg.n) {
        pack_store4(pl, sg, j0, pp);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (j0 + e < sg.n) pack_store(pl, sg, j0 + e, pp[e]);
      }
    }
  }
}

__global__ void adam_bump_kernel(int* __restrict__ tdev) { *tdev += 1; }

// plain SGD with momentum (torch.optim.SGD semantics, dampening 0, no nesterov)
__global__ void __launch_bounds__(256)
sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf, long n,
           float lr, float momentum, float wd, float grad_scale, int first) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float d = g[i] * grad_scale + wd * p[i];
    if (momentum != 0.f) {
      float b = first ? d : momentum * buf[i] + d;
      buf[i] = b;
      d = b;
    }
    p[i] -= lr * d;
  }
}

// out = in * scale, fp32 -> bf16 (grad payload compression for precision_bits = 16)
__global__ void cast_scale_bf16_kernel(const float* __restrict__ in, bf16* __restrict__ out, long n,
                                       float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (bf16)(in[i] * scale);
}

__global__ void cast_scale_f32_kernel(const bf16* __restrict__ in, float* __restrict__ out, long n,
                                      float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (float)in[i] * scale;
}

int grid_for(long n) {
  long b = (n + 255) / 256;
  return (int)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

}  // namespace

DN_API int dn_adam(float* p, const float* g, float* m, float* v, long n, float lr, float b1,
                   float b2, float eps, float wd, float bc1, float inv_sqrt_bc2, float grad_scale,
                   long long* cursor, hipStream_t st) {
  if (n <= 0) return DN_OK;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return DN_BAD_SHAPE;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, st, p, g, m, v, n, lr,
                     b1, b2, eps, wd, bc1, inv_sqrt_bc2, grad_scale, (const int*)nullptr, 0.0, 0.0, 1, cursor);
  return dn_launch_status();
}

// Adam whose step number t is read from (and then advanced in) device memory: capturable in a
// HIP graph and replayed every step with the right bias corrections.  *tdev = completed steps.
DN_API int dn_adam_dev(float* p, const float* g, float* m, float* v, long n, float lr, double b1,
                       double b2, float eps, float wd, float grad_scale, int* tdev, int prebumped,
                       long long* cursor, hipStream_t st) {
  if (n <= 0) return DN_OK;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return DN_BAD_SHAPE;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, st, p, g, m, v, n, lr,
                     (float)b1, (float)b2, eps, wd, 0.f, 0.f, grad_scale, (const int*)tdev, b1, b2, prebumped ? 0 : 1,
                     cursor);
  if (!prebumped) hipLaunchKernelGGL(adam_bump_kernel, dim3(1), dim3(1), 0, st, tdev);
  return dn_launch_status();
}

// adam_pack_kernel launch.  segs: host PackSeg-compatible rows {off, n, kind, d, dst, dst2} sorted
// by offset (cnt <= 16); the device-fed gather (gx ... yd) is optional (gx null: none).
DN_API long dn_pack_seg_size() { return (long)sizeof(PackSeg); }
DN_API int dn_adam_pack(float* p, float* g, float* m, float* v, long n, float lr, double b1,
                        double b2, float eps, float wd, float grad_scale, const int* tdev,
                        int update, int zero_grad, const void* segs, int cnt, int I, int Hd,
                        int HD, const void* gx, int gx_bf16, long row_elems, const long long* gy,
                        const long long* order, long nb, const long long* cursor, int B,
                        void* xb, long long* yd, long long* sd, int gofs, const void* record,
                        hipStream_t st) {
  if (n <= 0 || n % 4 || cnt < 0 || cnt > PACK_SEGS) return DN_BAD_SHAPE;
  StepRecord rec{};
  if (record && update) {
    rec = *reinterpret_cast<const StepRecord*>(record);
    if (!rec.out || !rec.loss || !rec.rs || !rec.rl || !rec.cursor || rec.n <= 0 || rec.B <= 0 ||
        (rec.col < 0 ? !rec.pred : rec.ld <= rec.col))
      return DN_BAD_SHAPE;
  }
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return DN_BAD_SHAPE;
  if (update && !tdev) return DN_BAD_SHAPE;
  PackPlan pl{};
  pl.cnt = cnt;
  pl.I = I;
  pl.Hd = Hd;
  pl.HD = HD;
  const PackSeg* hs = reinterpret_cast<const PackSeg*>(segs);
  for (int k = 0; k < cnt; ++k) {
    pl.s[k] = hs[k];
    const PackSeg& s = pl.s[k];
    if (s.off % 4 || s.n <= 0 || s.off + s.n > n || !s.dst) return DN_BAD_SHAPE;
    if (k && s.off < pl.s[k - 1].off + pl.s[k - 1].n) return DN_BAD_SHAPE;  // sorted, disjoint
    if ((s.kind == PK_WIH || s.kind == PK_WHH || s.kind == PK_BIAS) && (Hd <= 0 || HD < Hd || I <= 0))
      return DN_BAD_SHAPE;
    if (s.kind == PK_WHH && !s.dst2) return DN_BAD_SHAPE;
  }
  StepPrologue sp{};
  if (gx) {
    const int rc = prologue_gather(sp, gx, gx_bf16, row_elems, gy, order, nb, cursor, B, xb, yd,
                                   g, 0, nullptr, sd);
    if (rc != DN_OK) return rc;
  }
  // one item per thread up to 4096 workgroups per part (the chip holds ~2048 at a time; the
  // rest start as the first retire)
  auto parts = [](long items) { return (int)((items + 255) / 256 < 4096 ? (items + 255) / 256 : 4096); };
  const int ub = parts(n / 4), gb = sp.gx ? parts(sp.ux + sp.ny) : 0;
  hipLaunchKernelGGL(adam_pack_kernel, dim3(ub + gb + (rec.out ? 1 : 0)), dim3(256), 0, st, p, g,
                     m, v, n, lr, (float)b1, (float)b2, eps, wd, grad_scale, tdev, b1, b2, update,
                     zero_grad, pl, sp, gofs, ub, rec);
  return dn_launch_status();
}

// the standalone record (eager steps, and steps whose update is not the packing Adam): slot
// (*cursor + cofs) mod n, cofs = -1 after an update that advanced the cursor
DN_API long dn_step_record_size() { return (long)sizeof(StepRecord); }
DN_API int dn_step_record(const void* record, int cofs, hipStream_t st) {
  if (!record) return DN_BAD_SHAPE;
  const StepRecord r = *reinterpret_cast<const StepRecord*>(record);
  if (!r.out || !r.loss || !r.rs || !r.rl || !r.cursor || r.n <= 0 || r.B <= 0 ||
      (r.col < 0 ? !r.pred : r.ld <= r.col))
    return DN_BAD_SHAPE;
  hipLaunchKernelGGL(record_kernel, dim3(1), dim3(256), 0, st, r, cofs);
  return dn_launch_status();
}

DN_API int dn_sgd(float* p, const float* g, float* buf, long n, float lr, float momentum, float wd,
                  float grad_scale, int first, hipStream_t st) {
  if (n <= 0) return DN_OK;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, g, buf, n, lr, momentum,
                     wd, grad_scale, first);
  return dn_launch_status();
}

DN_API int dn_cast_f32_bf16(const float* in, void* out, long n, float scale, hipStream_t st) {
  if (n <= 0) return DN_OK;
  hipLaunchKernelGGL(cast_scale_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, st, in, (bf16*)out, n,
                     scale);
  return dn_launch_status();
}

DN_API int dn_cast_bf16_f32(const void* in, float* out, long n, float scale, hipStream_t st) {
  if (n <= 0) return DN_OK;
  hipLaunchKernelGGL(cast_scale_f32_kernel, dim3(grid_for(n)), dim3(256), 0, st, (const bf16*)in,
                     out, n, scale);
  return dn_launch_status();
}
