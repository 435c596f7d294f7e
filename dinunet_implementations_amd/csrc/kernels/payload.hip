// Collective payload kernels for the site-mean reductions (parallel/collective.py).
//
// The reference ships 16-bit site gradients as IEEE half (compspec.json:161-176 "precision_bits")
// and averages them on the remote.  Here the mean is a direct two-phase exchange over the
// fully-connected xGMI mesh (each rank talks to each peer over its own link, instead of a
// ring whose every step is bound by one link):
//
//   pack     fp32 gradient range -> W blocks of [8-element header | chunk] in the payload type
//            (fp16, bf16 or fp32), zero-padded;
//   all_to_all (RCCL): rank r receives block r of every site;
//   rowsum   the W blocks summed in FP32, times 1/world, rounded once to the payload type;
//   all_gather (RCCL) of the mean blocks;
//   unpack   payload -> fp32 gradient range.
//
// A 16-bit payload is rounded exactly twice (site value, mean) and never accumulated in 16 bits,
// unlike an all-reduce on a 16-bit buffer, whose partial sums round at every hop.
//
// fp16 blocks carry a power-of-two scale 2^e (header element 0 = e): a site scales its range so
// that max|g| * 2^e < 2^15 (amax kernel; no host sync), which keeps gradients that are tiny
// against fp16's fixed range (|g| < 2^-14 would be subnormal, < 2^-24 zero) at full 11-bit
// precision.  The mean block uses the smallest of the W exponents (|mean| <= max |g_w|, so it
// cannot overflow).  bf16 / fp32 blocks carry e = 0 (their exponent range is fp32's).
//
// fp16 data carry power-of-two scales 2^e PER SUB-BLOCK of SB = 2,048 elements (an 8-element
// header ahead of every sub-block, element 0 = e): the pack launch computes each sub-block's
// max |x| in the workgroup that packs it (one workgroup = one sub-block, 8 elements per lane) and
// scales it so that max|g| * 2^e < 2^15, which keeps gradients that are tiny against fp16's fixed
// range (|g| < 2^-14 would be subnormal, < 2^-24 zero) at full 11-bit precision -- with no
// separate max launch, no atomic and no host sync (a per-site scale needed a grid-wide max
// first: amax launch + pack, 40 us of local kernels against 16 for bf16, profiles/r4_comm_model).
// The mean sub-block uses the smallest of its W exponents (|mean| <= max |g_w|, so it cannot
// overflow).  bf16 / fp32 sub-blocks carry e = 0 (their exponent range is fp32's).
//
// Layout: a rank-block of `chunk` elements (a multiple of SB) is chunk / SB sub-blocks of
// [HDR | SB]; the payload of W ranks is W rank-blocks back to back.
//
// Element type codes: 0 = bf16, 1 = fp16 (IEEE binary16), 2 = fp32.  Every kernel moves 8
// elements (16/32 bytes) per lane; chunk is a multiple of 8 (host-checked), the fp32 gradient
// range need not be (a scalar tail).
#include "common.h"

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int PT_BF16 = 0, PT_F16 = 1, PT_F32 = 2;

template <int T> struct Pay;
template <> struct Pay<PT_BF16> { typedef bf16x8 v8; typedef bf16 s; };
template <> struct Pay<PT_F16> { typedef f16x8 v8; typedef f16 s; };

template <int T>
__device__ __forceinline__ void load8(const void* p, long i8, float (&o)[8]) {
  if constexpr (T == PT_F32) {
    const f32x4* q = reinterpret_cast<const f32x4*>(p) + 2 * i8;
    const f32x4 a = q[0], b = q[1];
#pragma unroll
    for (int k = 0; k < 4; ++k) { o[k] = a[k]; o[4 + k] = b[k]; }
  } else {
    const typename Pay<T>::v8 v = reinterpret_cast<const typename Pay<T>::v8*>(p)[i8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (float)v[k];
  }
}

template <int T>
__device__ __forceinline__ void store8(void* p, long i8, const float (&o)[8]) {
  if constexpr (T == PT_F32) {
    f32x4* q = reinterpret_cast<f32x4*>(p) + 2 * i8;
    q[0] = f32x4{o[0], o[1], o[2], o[3]};
    q[1] = f32x4{o[4], o[5], o[6], o[7]};
  } else {
    typename Pay<T>::v8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (typename Pay<T>::s)o[k];
    reinterpret_cast<typename Pay<T>::v8*>(p)[i8] = v;
  }
}

template <int T>
__device__ __forceinline__ float load1(const void* p, long i) {
  if constexpr (T == PT_F32) return reinterpret_cast<const float*>(p)[i];
  else return (float)reinterpret_cast<const typename Pay<T>::s*>(p)[i];
}

constexpr int HDR = 8;     // header elements per sub-block (16 B at 16 bits)
constexpr int SB = 2048;   // elements per scaled sub-block: 256 lanes x 8
constexpr int SBS = HDR + SB;

// block exponent of a range with max |x| = amax: max |x| * 2^e < 2^15
__device__ __forceinline__ int scale_exp(float amax) {
  if (!(amax > 0.f) || !__builtin_isfinite(amax)) return 0;  // zero / inf / nan: unscaled
  int k;
  (void)__builtin_frexpf(amax, &k);  // amax = m * 2^k, m in [0.5, 1)
  const int e = 15 - k;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}

__device__ __forceinline__ float exp2i(int e) { return __builtin_ldexpf(1.f, e); }

// max |v| over the workgroup (256 lanes); a NaN wins (and disables scaling)
__device__ __forceinline__ float wg_amax(float m, float* wm) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float t = __shfl_xor(m, o, 64);
    m = t > m || t != t ? t : m;
  }
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  m = wm[0];
#pragma unroll
  for (int w = 1; w < 4; ++w) m = wm[w] > m || wm[w] != wm[w] ? wm[w] : m;
  return m;
}

// src fp32 [n] -> dst T: nsb_total sub-blocks of [HDR | SB] (zeros past n), each scaled by
// scale * 2^e with its own e (fp16: from the sub-block's max |x|, `scaled`)
template <int T>
__global__ void __launch_bounds__(256) pack_kernel(const float* __restrict__ src, void* __restrict__ dst,
                                                   long n, long nsb, float scale, int scaled) {
  __shared__ float wm[4];
  for (long g = blockIdx.x; g < nsb; g += gridDim.x) {
    const long e0 = g * SB + 8 * threadIdx.x;
    float o[8];
    if (e0 + 8 <= n) {
      load8<PT_F32>(src, e0 / 8, o);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = e0 + k < n ? src[e0 + k] : 0.f;
    }
    int e = 0;
    if (T == PT_F16 && scaled) {
      float m = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float a = __builtin_fabsf(o[k]);
        m = a > m || a != a ? a : m;
      }
      e = scale_exp(wg_amax(m, wm));
    }
    const float sc = scale * exp2i(e);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] *= sc;
    const long base8 = g * (SBS / 8);
    store8<T>(dst, base8 + 1 + threadIdx.x, o);
    if (threadIdx.x == 0) {
      float h[8] = {(float)e, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      store8<T>(dst, base8, h);
    }
    if (T == PT_F16 && scaled) __syncthreads();  // wm is reused by the next sub-block
  }
}

// src T: sub-blocks of [HDR | SB] -> dst fp32 [n], each unscaled by its 2^-e, * scale
template <int T>
__global__ void __launch_bounds__(256) unpack_kernel(const void* __restrict__ src, float* __restrict__ dst,
                                                     long n, long nsb, float scale) {
  for (long g = blockIdx.x; g < nsb; g += gridDim.x) {
    const long base8 = g * (SBS / 8);
    const float e = load1<T>(src, g * SBS);
    const float sc = scale * exp2i(-(int)e);
    const long e0 = g * SB + 8 * threadIdx.x;
    if (e0 >= n) continue;
    float o[8];
    load8<T>(src, base8 + 1 + threadIdx.x, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] *= sc;
    if (e0 + 8 <= n) {
      store8<PT_F32>(dst, e0 / 8, o);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (e0 + k < n) dst[e0 + k] = o[k];
    }
  }
}

// src T: W rank-blocks of nsb sub-blocks -> dst T one rank-block: sub-block s = scale * sum_w
// unscaled src[w][s] (fp32 accumulation in rank order), rescaled by the smallest exponent
template <int T>
__global__ void __launch_bounds__(256) rowsum_kernel(const void* __restrict__ src, void* __restrict__ dst,
                                                     int W, long nsb, float scale) {
  for (long s = blockIdx.x; s < nsb; s += gridDim.x) {
    int emin = 1 << 20;
    for (int w = 0; w < W; ++w) emin = min(emin, (int)load1<T>(src, (w * nsb + s) * SBS));
    const float out_sc = scale * exp2i(emin);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, v[8];
    for (int w = 0; w < W; ++w) {
      const long base8 = (w * nsb + s) * (SBS / 8);
      const float un = exp2i(-(int)load1<T>(src, (w * nsb + s) * SBS));
      load8<T>(src, base8 + 1 + threadIdx.x, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k] * un;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= out_sc;
    store8<T>(dst, s * (SBS / 8) + 1 + threadIdx.x, acc);
    if (threadIdx.x == 0) {
      float h[8] = {(float)emin, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      store8<T>(dst, s * (SBS / 8), h);
    }
  }
}


bool aligned(const void* a, const void* b) { return (((uintptr_t)a | (uintptr_t)b) & 15) == 0; }

}  // namespace

#define DN_PAYLOAD_DISPATCH(T, KERNEL, ...)                                                        \
  switch (T) {                                                                                     \
    case PT_BF16: hipLaunchKernelGGL(KERNEL<PT_BF16>, __VA_ARGS__); break;                         \
    case PT_F16: hipLaunchKernelGGL(KERNEL<PT_F16>, __VA_ARGS__); break;                           \
    case PT_F32: hipLaunchKernelGGL(KERNEL<PT_F32>, __VA_ARGS__); break;                           \
    default: return DN_BAD_SHAPE;                                                                  \
  }

static int grid_sb(long nsb) { return (int)(nsb < 8192 ? (nsb > 0 ? nsb : 1) : 8192); }

// fp32 src [n] -> world * chunk elements of payload (chunk % SB == 0, world * chunk >= n)
DN_API int dn_payload_pack(const float* src, void* dst, long n, int world, long chunk, float scale,
                           int scaled, int type, hipStream_t st) {
  if (n < 0 || world < 1 || chunk <= 0 || chunk % SB || world * chunk < n || !aligned(src, dst))
    return DN_BAD_SHAPE;
  const long nsb = world * chunk / SB;
  DN_PAYLOAD_DISPATCH(type, pack_kernel, dim3(grid_sb(nsb)), dim3(256), 0, st, src, dst, n, nsb,
                      scale, scaled);
  return dn_launch_status();
}

// the first n elements of a payload of sub-blocks -> fp32 dst
DN_API int dn_payload_unpack(const void* src, float* dst, long n, float scale, int type,
                             hipStream_t st) {
  if (n < 0 || !aligned(src, dst)) return DN_BAD_SHAPE;
  if (n == 0) return DN_OK;
  const long nsb = (n + SB - 1) / SB;
  DN_PAYLOAD_DISPATCH(type, unpack_kernel, dim3(grid_sb(nsb)), dim3(256), 0, st, src, dst, n, nsb,
                      scale);
  return dn_launch_status();
}

// W rank-blocks of `chunk` elements -> their scaled fp32 sum as one rank-block
DN_API int dn_payload_rowsum(const void* src, void* dst, int world, long chunk, float scale, int type,
                             hipStream_t st) {
  if (world < 1 || chunk <= 0 || chunk % SB || !aligned(src, dst)) return DN_BAD_SHAPE;
  DN_PAYLOAD_DISPATCH(type, rowsum_kernel, dim3(grid_sb(chunk / SB)), dim3(256), 0, st, src, dst,
                      world, chunk / SB, scale);
  return dn_launch_status();
}

// payload elements of `elems` data elements (sub-block headers included; 0 stays 0)
DN_API long dn_payload_numel(long elems) { return (elems + SB - 1) / SB * SBS; }
DN_API long dn_payload_subblock() { return SB; }
