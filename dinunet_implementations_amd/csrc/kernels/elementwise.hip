// Small fused memory-bound kernels (vectorised 16 B per lane, deterministic reductions).
#include "common.h"
#include "prologue.h"

namespace {

constexpr int RB_SLABS = 64;  // row slabs for column reductions (>= 64 workgroups in flight)

// dym = dy * (y > 0) and per-slab column sums of dym.  y = ReLU output, all bf16 [N][O].
// block = 256 threads = 8 rows x 32 column-groups of 8 (16 B vectors); grid = (col strips, slabs)
__global__ void __launch_bounds__(256)
relu_bwd_colsum_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ y,
                       bf16* __restrict__ dym, float* __restrict__ part, int N, int O) {
  const int cg = blockIdx.x * 32 + (threadIdx.x & 31);  // column group
  const int rl = threadIdx.x >> 5;                       // 0..7
  const int c0 = cg * 8;
  const int rows_per = (N + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows_per, r1 = min(N, r0 + rows_per);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool vec = (O & 7) == 0 && c0 + 8 <= O;
  for (int r = r0 + rl; r < r1; r += 8) {
    const long i = (long)r * O + c0;
    if (vec) {
      const bf16x8 g = *reinterpret_cast<const bf16x8*>(dy + i);
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(y + i);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = (float)a[e] > 0.f ? g[e] : (bf16)0.f;
        s[e] += (float)o[e];
      }
      *reinterpret_cast<bf16x8*>(dym + i) = o;
    } else {
      for (int e = 0; e < 8 && c0 + e < O; ++e) {
        const bf16 o = (float)y[i + e] > 0.f ? dy[i + e] : (bf16)0.f;
        dym[i + e] = o;
        s[e] += (float)o;
      }
    }
  }
  __shared__ float red[8][32 * 8 + 4];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][(threadIdx.x & 31) * 8 + e] = s[e];
  __syncthreads();
  // 256 threads: each finalises one column of this strip
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col < O) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) t += red[r][threadIdx.x];
    part[(long)blockIdx.y * O + col] = t;
  }
}

// dym = dy * (y > 0), elementwise over n bf16 values (n % 8 == 0, 16-B aligned): the encoder
// backward's mask when its bias gradient rides in the weight-gradient GEMM (dym^T @ ones)
__global__ void __launch_bounds__(256)
relu_bwd_kernel(const bf16x8* __restrict__ dy, const bf16x8* __restrict__ y,
                bf16x8* __restrict__ dym, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    const bf16x8 g = dy[i], a = y[i];
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (float)a[e] > 0.f ? g[e] : (bf16)0.f;
    dym[i] = o;
  }
}

// out[c] = sum_s part[s][c]  (fixed order -> bit-reproducible)
__global__ void colsum_slabs_kernel(const float* __restrict__ part, int slabs, int O,
                                    float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= O) return;
  // 8 independent partial chains: the slab loads are issued back to back
  float t[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 8 <= slabs; s += 8)
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] += part[(long)(s + k) * O + c];
  for (; s < slabs; ++s) t[0] += part[(long)s * O + c];
  const float v = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
  out[c] = accumulate ? out[c] + v : v;
}

// Training-step prologue in ONE launch (prologue.h; it replaces three: two copies into the HIP
// graph's static inputs and the gradient zeroing).  Grid-stride over 8-element batch units,
// 4-element gradient units and single labels.
__global__ void __launch_bounds__(256)
step_prologue_kernel(StepPrologue sp) {
  if (sp.bump && blockIdx.x == 0 && threadIdx.x == 0) *sp.bump += 1;  // Adam's device step counter
  const long total = sp.ux + sp.ug + sp.ny;
  const long cur = prologue_cursor(sp);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x)
    prologue_item(sp, i, cur);
}

static int prologue_launch(const StepPrologue& sp, hipStream_t st) {
  const long total = sp.ux + sp.ug + sp.ny;
  if (total <= 0) return DN_OK;
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(step_prologue_kernel, dim3((unsigned)blocks), dim3(256), 0, st, sp);
  return dn_launch_status();
}

}  // namespace

// bump: the graph-captured Adam's device step counter, advanced once by this launch (null: none)
DN_API int dn_step_prologue(const float* x, long nx, void* xb, const long long* y, long ny,
                            long long* yd, float* g, long ng, int* bump, hipStream_t st) {
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
  return prologue_launch(sp, st);
}

// the device-fed prologue as a launch of its own (models whose first launch is not the LSTM pack)
DN_API int dn_step_gather(const void* gx, int gx_bf16, long row_elems, const long long* gy,
                          const long long* order, long nb, const long long* cursor, int B, void* xb,
                          long long* yd, float* g, long ng, int* bump, hipStream_t st) {
  StepPrologue sp;
  const int rc = prologue_gather(sp, gx, gx_bf16, row_elems, gy, order, nb, cursor, B, xb, yd, g,
                                 ng, bump);
  if (rc != DN_OK) return rc;
  return prologue_launch(sp, st);
}

DN_API int dn_relu_bwd(const void* dy, const void* y, void* dym, long n, hipStream_t st) {
  if (n <= 0 || n % 8) return DN_BAD_SHAPE;
  if ((((uintptr_t)dy) | ((uintptr_t)y) | ((uintptr_t)dym)) & 15) return DN_BAD_SHAPE;
  const long n8 = n / 8;
  const long blocks = (n8 + 255) / 256 < 2048 ? (n8 + 255) / 256 : 2048;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const bf16x8*)dy, (const bf16x8*)y, (bf16x8*)dym, n8);
  return dn_launch_status();
}

DN_API long dn_relu_bwd_colsum_workspace(int N, int O) { return (long)RB_SLABS * O; }

DN_API int dn_relu_bwd_colsum(const void* dy, const void* y, void* dym, float* db, float* ws,
                              int N, int O, int accumulate, hipStream_t st) {
  if (N <= 0 || O <= 0) return DN_BAD_SHAPE;
  const int slabs = N < RB_SLABS ? N : RB_SLABS;
  hipLaunchKernelGGL(relu_bwd_colsum_kernel, dim3((O + 255) / 256, slabs), dim3(256), 0, st,
                     (const bf16*)dy, (const bf16*)y, (bf16*)dym, ws, N, O);
  hipLaunchKernelGGL(colsum_slabs_kernel, dim3((O + 255) / 256), dim3(256), 0, st, ws, slabs, O, db,
                     accumulate);
  return dn_launch_status();
}

// in-kernel wait limit (common.h): < 0 restores every kernel's default
// fp32 -> bf16 images of up to 8 tensors in one launch (the replicated head's weight images when
// no Adam-emitted operand pack keeps them current: ops.head.HeadSpec.own_images)
constexpr int CAST_MAX = 8;
struct CastGroup {
  const float* src[CAST_MAX];
  bf16* dst[CAST_MAX];
  long n[CAST_MAX];
  long off[CAST_MAX + 1];  // prefix of n (elements)
  int count;
};

__global__ void __launch_bounds__(256) cast_group_kernel(CastGroup g) {
  const long total = g.off[g.count];
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    int t = 0;
#pragma unroll
    for (int k = 1; k < CAST_MAX; ++k)
      if (k < g.count && i >= g.off[k]) t = k;
    const long j = i - g.off[t];
    g.dst[t][j] = (bf16)g.src[t][j];
  }
}

DN_API int dn_cast_bf16_group(const float* const* src, bf16* const* dst, const long* n, int count,
                              hipStream_t st) {
  if (count < 1 || count > CAST_MAX || !src || !dst || !n) return DN_BAD_SHAPE;
  CastGroup g{};
  g.count = count;
  for (int k = 0; k < count; ++k) {
    if (!src[k] || !dst[k] || n[k] < 0) return DN_BAD_SHAPE;
    g.src[k] = src[k], g.dst[k] = dst[k], g.n[k] = n[k];
    g.off[k + 1] = g.off[k] + n[k];
  }
  const long total = g.off[count];
  if (total == 0) return DN_OK;
  const long blocks = (total + 255) / 256;
  hipLaunchKernelGGL(cast_group_kernel, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(256),
                     0, st, g);
  return dn_launch_status();
}

int g_dn_spin_limit = -1;
DN_API int dn_set_spin_limit(int polls) {
  g_dn_spin_limit = polls < 0 ? -1 : polls;
  return DN_OK;
}

// CU-occupancy probe for tests of the persistent kernels beside collectives: `blocks` workgroups
// of `threads` that each spin (s_sleep between polls) until `us` microseconds have passed on the
// 100 MHz real-time counter -- the footprint of RCCL's channel kernels while a collective is in
// flight (one workgroup per channel, resident for the whole transfer).  Bounded to 100 ms.
__global__ void busy_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

DN_API int dn_busy(int blocks, int threads, int us, hipStream_t st) {
  if (blocks < 1 || blocks > 4096 || threads < 64 || threads > 1024 || us < 0 || us > 100000)
    return DN_BAD_SHAPE;
  hipLaunchKernelGGL(busy_kernel, dim3(blocks), dim3(threads), 0, st, (unsigned long long)us * 100);
  return dn_launch_status();
}
