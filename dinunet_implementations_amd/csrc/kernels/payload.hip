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

constexpr int HDR = 8;  // header elements per block (16 B at 16 bits)

// block exponent of a range with max |x| = amax: max |x| * 2^e < 2^15
__device__ __forceinline__ int scale_exp(float amax) {
  if (!(amax > 0.f) || !__builtin_isfinite(amax)) return 0;  // zero / inf / nan: unscaled
  int k;
  (void)__builtin_frexpf(amax, &k);  // amax = m * 2^k, m in [0.5, 1)
  const int e = 15 - k;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}

__device__ __forceinline__ float exp2i(int e) { return __builtin_ldexpf(1.f, e); }

// max |x| over n -> *word (float bits of a non-negative value order like unsigned ints).  One
// atomic per WORKGROUP (LDS across its 4 waves) from at most 64 workgroups: same-address atomics
// serialise at the L2, and one per wave from 512 workgroups (2,048) cost ~20 us of the fp16
// exchange (tools/comm_model.py local kernels: fp16 40 us vs bf16 16 us)
__global__ void __launch_bounds__(256) amax_kernel(const float* __restrict__ x, long n, unsigned* word) {
  __shared__ float wm[4];
  float m = 0.f;
  const long n4 = n >> 2;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a = __builtin_fabsf(v[k]);
      m = a > m || a != a ? a : m;  // a NaN wins (and disables scaling)
    }
  }
  for (long i = 4 * n4 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float a = __builtin_fabsf(x[i]);
    m = a > m || a != a ? a : m;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float t = __shfl_xor(m, o, 64);
    m = t > m || t != t ? t : m;
  }
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 1; w < 4; ++w) m = wm[w] > m || wm[w] != wm[w] ? wm[w] : m;
    atomicMax(word, __float_as_uint(m));
  }
}

// src fp32 [n] -> dst T: W blocks of [HDR | chunk] (zeros past n), scaled by scale * 2^e
template <int T>
__global__ void __launch_bounds__(256) pack_kernel(const float* __restrict__ src, void* __restrict__ dst,
                                                   long n, int W, long chunk, float scale,
                                                   const unsigned* __restrict__ amax) {
  const int e = (T == PT_F16 && amax) ? scale_exp(__uint_as_float(*amax)) : 0;
  const float sc = scale * exp2i(e);
  const long c8 = chunk / 8, m8 = W * c8;
  if (blockIdx.x == 0 && threadIdx.x < W) {
    float h[8] = {(float)e, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    store8<T>(dst, threadIdx.x * (c8 + 1), h);
  }
  for (long i = blockIdx.x * 256L + threadIdx.x; i < m8; i += (long)gridDim.x * 256) {
    float o[8];
    if (8 * i + 8 <= n) {
      load8<PT_F32>(src, i, o);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] *= sc;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = 8 * i + k < n ? src[8 * i + k] * sc : 0.f;
    }
    const long b = i / c8;
    store8<T>(dst, i + b + 1, o);  // past the headers of blocks 0..b
  }
}

// src T: W blocks of [HDR | chunk] -> dst fp32 [n], each block unscaled by its 2^-e, * scale;
// resets the amax word for the next exchange
template <int T>
__global__ void __launch_bounds__(256) unpack_kernel(const void* __restrict__ src, float* __restrict__ dst,
                                                     long n, long chunk, float scale, unsigned* amax) {
  const long n8 = (n + 7) / 8, c8 = chunk / 8;
  if (amax && blockIdx.x == 0 && threadIdx.x == 0) *amax = 0u;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long b = i / c8;
    float h[8];
    load8<T>(src, b * (c8 + 1), h);
    const float sc = scale * exp2i(-(int)h[0]);
    if (8 * i + 8 <= n) {
      float o[8];
      load8<T>(src, i + b + 1, o);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] *= sc;
      store8<PT_F32>(dst, i, o);
    } else {
      for (long k = 8 * i; k < n; ++k) dst[k] = load1<T>(src, (b + 1) * HDR + k) * sc;
    }
  }
}

// src T: W blocks of [HDR | chunk] -> dst T one block = scale * sum_w unscaled src[w] (fp32
// accumulation in rank order), rescaled by the smallest block exponent
template <int T>
__global__ void __launch_bounds__(256) rowsum_kernel(const void* __restrict__ src, void* __restrict__ dst,
                                                     int W, long c8, float scale) {
  int emin = 1 << 20;
  for (int w = 0; w < W; ++w) {
    float h[8];
    load8<T>(src, w * (c8 + 1), h);
    emin = min(emin, (int)h[0]);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float h[8] = {(float)emin, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    store8<T>(dst, 0, h);
  }
  const float out_sc = scale * exp2i(emin);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < c8; i += (long)gridDim.x * 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, v[8], h[8];
    for (int w = 0; w < W; ++w) {
      load8<T>(src, w * (c8 + 1), h);
      const float un = exp2i(-(int)h[0]);
      load8<T>(src, w * (c8 + 1) + 1 + i, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k] * un;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= out_sc;
    store8<T>(dst, 1 + i, acc);
  }
}

int grid8(long n8) {
  const long b = (n8 + 255) / 256;
  return (int)(b < 1024 ? (b > 0 ? b : 1) : 1024);
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

DN_API int dn_payload_amax(const float* x, long n, unsigned* word, hipStream_t st) {
  if (n <= 0) return DN_OK;
  if (((uintptr_t)x) & 15) return DN_BAD_SHAPE;
  const long b = (n + 1023) / 1024;
  hipLaunchKernelGGL(amax_kernel, dim3((int)(b < 64 ? b : 64)), dim3(256), 0, st, x, n, word);
  return dn_launch_status();
}

DN_API int dn_payload_pack(const float* src, void* dst, long n, int world, long chunk, float scale,
                           const unsigned* amax, int type, hipStream_t st) {
  if (n < 0 || world < 1 || chunk <= 0 || chunk % 8 || world * chunk < n || world > 256 || !aligned(src, dst))
    return DN_BAD_SHAPE;
  DN_PAYLOAD_DISPATCH(type, pack_kernel, dim3(grid8(world * chunk / 8)), dim3(256), 0, st, src, dst, n,
                      world, chunk, scale, amax);
  return dn_launch_status();
}

DN_API int dn_payload_unpack(const void* src, float* dst, long n, long chunk, float scale, unsigned* amax,
                             int type, hipStream_t st) {
  if (n < 0 || chunk <= 0 || chunk % 8 || !aligned(src, dst)) return DN_BAD_SHAPE;
  if (n == 0) return DN_OK;
  DN_PAYLOAD_DISPATCH(type, unpack_kernel, dim3(grid8((n + 7) / 8)), dim3(256), 0, st, src, dst, n, chunk,
                      scale, amax);
  return dn_launch_status();
}

DN_API int dn_payload_rowsum(const void* src, void* dst, int world, long chunk, float scale, int type,
                             hipStream_t st) {
  if (world < 1 || chunk <= 0 || chunk % 8 || !aligned(src, dst)) return DN_BAD_SHAPE;
  DN_PAYLOAD_DISPATCH(type, rowsum_kernel, dim3(grid8(chunk / 8)), dim3(256), 0, st, src, dst, world,
                      chunk / 8, scale);
  return dn_launch_status();
}
