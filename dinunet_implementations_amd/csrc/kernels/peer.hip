// Peer exchange over IPC-mapped HBM: the site-mean and the factor all-gather of the engines
// without RCCL (parallel/peer.py).
//
// Every site process allocates one UNCACHED arena (hipExtMallocWithFlags(hipDeviceMallocUncached))
// and exports it with hipIpcGetMemHandle; every peer maps it with hipIpcOpenMemHandle.  On an
// MI355X node the mapped pointer of a peer's arena is that GPU's HBM across the xGMI link between
// the two (7 links per GPU, one per peer: a write to peer d uses the d link only, so pushing to
// all peers at once drives all 7 links); several site processes sharing one GPU map each other's
// arenas on the same device, which is how the exchange is exercised with real cross-process
// device traffic on a one-GPU box.
//
// Uncached memory keeps the hand-offs simple: a byte a peer wrote over xGMI lands in the owner's
// HBM, and no L2 of the owner can hold a stale copy of it (coarse-grained HBM would need every
// reader's L2 invalidated at system scope).  Flags are u32 words in the same arenas.
//
// Site-mean of n fp32 elements over W sites, wire type T (fp32 / bf16 / fp16 with the block-scaled
// sub-blocks of payload.hip: [8-element header | 2,048 elements], fp16 scaled per sub-block), in
// three launches, each only ever waiting for an EARLIER phase of its peers -- so no launch depends
// on a peer launch being resident at the same time as itself (several processes on one GPU, or a
// peer still in host code):
//
//   push    (no waits)   my range in W chunks of `chunk` elements; chunk d, sub-block s is packed
//                        and written into site d's inbox slot [me][s]; then flag rs[d][s][me] = 1
//   reduce  (waits push) sub-block s of MY chunk: wait rs[me][s][w] for every w (and clear them),
//                        fp32 sum in site order, * 1/W, rounded once to T, written into EVERY site's
//                        gather slot [me][s]; then flag ag[j][me][s] = 1 at every site j
//   unpack  (waits reduce) gather slot [d][s] -> my fp32 range, after ag[me][d][s] (cleared)
//
// Reuse is safe without epochs: a site writes a peer's inbox / rs flags of exchange k+1 only after
// its own unpack of exchange k, i.e. after that peer's reduce of k (which cleared the flags and
// read the inbox); a site writes a peer's gather slot / ag flag of k+1 only after every site's push
// of k+1, i.e. after every unpack of k.  Every site computes the mean of its own chunk once and
// ships it: all replicas hold bit-identical means.
//
// Factor all-gather (rank-dAD) of m elements per site: gpush writes my sub-blocks into every site's
// gather slot [me] after that site has returned the slot's credit, gcollect waits for each
// site's data flag, unpacks it and returns the credit.  (A gather has no later phase that orders the
// next push after every reader, hence the credits: a slot is written again only once its reader
// has read it.)
//
// Hand-off form (system scope, uncached memory): every storing wave waits for its stores
// (vmcnt(0)), the workgroup barrier, then ONE lane fences release at system scope and stores the
// flag (system-scope atomic store, a vector store); the consumer's lane 0 polls with system-scope
// relaxed loads (bounded by a wall-clock timeout: a wait that gives up sets the sticky error word
// and the launch finishes -- runtime.health reports it), fences acquire at system scope, and the
// workgroup follows through a barrier.
#include "common.h"

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int PX_MAXW = 16;
constexpr int HDR = 8, SB = 2048, SBS = HDR + SB;  // as payload.hip
constexpr int PT_BF16 = 0, PT_F16 = 1, PT_F32 = 2;

template <int T> struct Wire;
template <> struct Wire<PT_BF16> { typedef bf16x8 v8; typedef bf16 s; };
template <> struct Wire<PT_F16> { typedef f16x8 v8; typedef f16 s; };

template <int T>
__device__ __forceinline__ void ld8(const void* p, long i8, float (&o)[8]) {
  if constexpr (T == PT_F32) {
    const f32x4* q = reinterpret_cast<const f32x4*>(p) + 2 * i8;
    const f32x4 a = q[0], b = q[1];
#pragma unroll
    for (int k = 0; k < 4; ++k) { o[k] = a[k]; o[4 + k] = b[k]; }
  } else {
    const typename Wire<T>::v8 v = reinterpret_cast<const typename Wire<T>::v8*>(p)[i8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (float)v[k];
  }
}

template <int T>
__device__ __forceinline__ void st8(void* p, long i8, const float (&o)[8]) {
  if constexpr (T == PT_F32) {
    f32x4* q = reinterpret_cast<f32x4*>(p) + 2 * i8;
    q[0] = f32x4{o[0], o[1], o[2], o[3]};
    q[1] = f32x4{o[4], o[5], o[6], o[7]};
  } else {
    typename Wire<T>::v8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (typename Wire<T>::s)o[k];
    reinterpret_cast<typename Wire<T>::v8*>(p)[i8] = v;
  }
}

template <int T>
__device__ __forceinline__ float ld1(const void* p, long i) {
  if constexpr (T == PT_F32) return reinterpret_cast<const float*>(p)[i];
  else return (float)reinterpret_cast<const typename Wire<T>::s*>(p)[i];
}

// element pointer arithmetic on a wire buffer
template <int T>
__device__ __forceinline__ char* wptr(void* base, long elems) {
  return reinterpret_cast<char*>(base) + elems * (T == PT_F32 ? 4 : 2);
}

__device__ __forceinline__ int scale_exp(float amax) {
  if (!(amax > 0.f) || !__builtin_isfinite(amax)) return 0;
  int k;
  (void)__builtin_frexpf(amax, &k);
  const int e = 15 - k;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}

__device__ __forceinline__ float exp2i(int e) { return __builtin_ldexpf(1.f, e); }

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

struct PxArgs {
  void* inbox[PX_MAXW];      // site w's inbox (mean: W slots x chunk payload)
  void* gath[PX_MAXW];       // site w's gather slots (W slots x chunk payload)
  unsigned* flags[PX_MAXW];  // site w's flag words (layout per kind, see the kernels)
  const float* src;          // my fp32 input
  float* dst;                // my fp32 output (may alias src)
  unsigned* err;             // my sticky error word (normal device memory)
  long n;                    // fp32 elements of src / dst (gather: per site)
  long chunk;                // elements per slot, a multiple of SB
  long dstride;              // gather: dst elements between sites
  long timeout;              // wait limit in s_memrealtime ticks (100 MHz)
  int W, me, scaled;
  float scale;               // unpack / gcollect: * scale
  float scale_red;           // reduce: * scale_red (1/W: the mean)
  int mode;                  // bit 0: release = store drain only (every payload byte is an
                             // uncached store: no L2 line to write back); bit 1: no acquire
                             // invalidate, the payload is read with system-scope (sc0 sc1) loads;
                             // bit 2: waits done by a preceding px_wait_kernel launch
};

typedef __attribute__((address_space(1))) unsigned px_gu32;

__device__ __forceinline__ void px_set(unsigned* f, unsigned v) {
  __hip_atomic_store((px_gu32*)f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned px_get(unsigned* f) {
  return __hip_atomic_load((px_gu32*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// lane 0: wait until *f == 1 (bounded), then clear it; a timeout sets the error word to `code`.
// mode bit 2: the flags were already taken by a one-workgroup wait launch (px_wait_kernel)
__device__ __forceinline__ void px_take(unsigned* f, const PxArgs& a, unsigned code) {
  if (a.mode & 4) return;
  const long t0 = (long)__builtin_amdgcn_s_memrealtime();
  while (px_get(f) != 1u) {
    if ((long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
      px_set(a.err, code);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  px_set(f, 0u);
}

// every storing wave drains its stores, the workgroup meets, lane 0 releases at system scope
// (mode bit 0: the drain is the release -- the payload went to uncached memory)
__device__ __forceinline__ void px_drain_release(int mode) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && !(mode & 1)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// lane 0 acquired (after its waits): the workgroup follows (mode bit 1: no invalidate, every
// payload load is a system-scope load, px_ldw8)
__device__ __forceinline__ void px_acquire_join(int mode) {
  if (threadIdx.x == 0 && !(mode & 2)) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

typedef __attribute__((ext_vector_type(4))) unsigned px_u32x4;

// 8 payload elements at wire element offset `at` + 8 * i8 of a peer-written region: plain loads
// after an acquire, or system-scope (sc0 sc1) buffer loads (mode bit 1)
template <int T>
__device__ __forceinline__ void px_ldw8(const void* base, long at, long i8, int mode,
                                        float (&o)[8]) {
  const char* p = wptr<T>(const_cast<void*>(base), at);
  if (!(mode & 2)) {
    ld8<T>(p, i8, o);
    return;
  }
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(p), 0,
                                                                     0x7fffffff, 0x00020000);
  if constexpr (T == PT_F32) {
    const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(32 * i8), 0, 17));
    const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(32 * i8 + 16), 0, 17));
#pragma unroll
    for (int k = 0; k < 4; ++k) { o[k] = a[k]; o[4 + k] = b[k]; }
  } else {
    const typename Wire<T>::v8 v = __builtin_bit_cast(
        typename Wire<T>::v8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(16 * i8), 0, 17));
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (float)v[k];
  }
}

// the sub-block header (element 0 = its exponent) of a peer-written region
template <int T>
__device__ __forceinline__ int px_ldexp(const void* base, long at, int mode) {
  if (!(mode & 2)) return (int)ld1<T>(base, at);
  const char* p = wptr<T>(const_cast<void*>(base), at);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(p), 0,
                                                                     0x7fffffff, 0x00020000);
  const unsigned u = __builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 17);
  if constexpr (T == PT_F32) return (int)__uint_as_float(u);
  else return (int)(float)__builtin_bit_cast(typename Wire<T>::s, (unsigned short)(u & 0xffff));
}

// fp32 x[e0 .. e0 + 8) (zeros past n) -> scaled sub-block element values, exponent of the
// sub-block (fp16 + scaled: from its max |x|)
template <int T>
__device__ __forceinline__ int px_load_scaled(const float* x, long e0, long n, int scaled,
                                              float (&o)[8], float* wm) {
  if (e0 + 8 <= n) {
    ld8<PT_F32>(x, e0 / 8, o);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = e0 + k < n ? x[e0 + k] : 0.f;
  }
  int e = 0;
  if (T == PT_F16 && scaled) {
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float v = __builtin_fabsf(o[k]);
      m = v > m || v != v ? v : m;
    }
    e = scale_exp(wg_amax(m, wm));
  }
  const float sc = exp2i(e);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] *= sc;
  return e;
}

// write one packed sub-block (header + 8 elements per lane) at wire element offset `at`
template <int T>
__device__ __forceinline__ void px_store_sb(void* base, long at, int e, const float (&o)[8]) {
  char* p = wptr<T>(base, at);
  st8<T>(p, 1 + threadIdx.x, o);
  if (threadIdx.x == 0) {
    float h[8] = {(float)e, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    st8<T>(p, 0, h);
  }
}

// ---- site-mean ---------------------------------------------------------------------------------
// flags of site w: rs at [s * W + sender] (s < nsbc), ag at [nsbc * W + owner * nsbc + s]

template <int T>
__global__ void __launch_bounds__(256) px_push_kernel(PxArgs a) {
  __shared__ float wm[4];
  const int s = blockIdx.x, d = blockIdx.y;
  const long nsbc = a.chunk / SB;
  float o[8];
  const int e = px_load_scaled<T>(a.src, d * a.chunk + (long)s * SB + 8 * threadIdx.x, a.n,
                                  a.scaled, o, wm);
  px_store_sb<T>(a.inbox[d], ((long)a.me * nsbc + s) * SBS, e, o);
  px_drain_release(a.mode);
  if (threadIdx.x == 0) px_set(a.flags[d] + (long)s * a.W + a.me, 1u);
}

// sub-block s of MY chunk: wait for every site's push, fp32 sum in site order, into every site's
// gather slot
template <int T>
__device__ __forceinline__ void px_reduce_task(const PxArgs& a, int s) {
  const int W = a.W;
  const long nsbc = a.chunk / SB;
  if (threadIdx.x == 0)
    for (int w = 0; w < W; ++w) px_take(a.flags[a.me] + (long)s * W + w, a, 0x100u | (unsigned)w);
  px_acquire_join(a.mode);
  const void* in = a.inbox[a.me];
  int ew[PX_MAXW];
  int emin = 1 << 20;
  for (int w = 0; w < W; ++w) {
    ew[w] = px_ldexp<T>(in, ((long)w * nsbc + s) * SBS, a.mode);
    emin = min(emin, ew[w]);
  }
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, v[8];
  for (int w = 0; w < W; ++w) {  // site order: every replica sums the same way
    const long at = ((long)w * nsbc + s) * SBS;
    const float un = exp2i(-ew[w]);
    px_ldw8<T>(in, at, 1 + threadIdx.x, a.mode, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += v[k] * un;
  }
  const float sc = a.scale_red * exp2i(emin);
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] *= sc;
  const long at = ((long)a.me * nsbc + s) * SBS;
  for (int j = 0; j < W; ++j) px_store_sb<T>(a.gath[j], at, emin, acc);
  px_drain_release(a.mode);
  if (threadIdx.x == 0)
    for (int j = 0; j < W; ++j) px_set(a.flags[j] + nsbc * W + (long)a.me * nsbc + s, 1u);
}

// owner d's sub-block s of the mean -> my fp32 range
template <int T>
__device__ __forceinline__ void px_unpack_task(const PxArgs& a, int d, int s) {
  const long nsbc = a.chunk / SB;
  if (threadIdx.x == 0)
    px_take(a.flags[a.me] + nsbc * a.W + (long)d * nsbc + s, a, 0x200u | (unsigned)d);
  px_acquire_join(a.mode);
  const long at = ((long)d * nsbc + s) * SBS;
  const void* g = a.gath[a.me];
  const float sc = a.scale * exp2i(-px_ldexp<T>(g, at, a.mode));
  const long e0 = d * a.chunk + (long)s * SB + 8 * threadIdx.x;
  if (e0 >= a.n) return;
  float o[8];
  px_ldw8<T>(g, at, 1 + threadIdx.x, a.mode, o);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] *= sc;
  if (e0 + 8 <= a.n) {
    st8<PT_F32>(a.dst, e0 / 8, o);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (e0 + k < a.n) a.dst[e0 + k] = o[k];
  }
}

template <int T>
__global__ void __launch_bounds__(256) px_reduce_kernel(PxArgs a) { px_reduce_task<T>(a, blockIdx.x); }

template <int T>
__global__ void __launch_bounds__(256) px_unpack_kernel(PxArgs a) {
  px_unpack_task<T>(a, blockIdx.y, blockIdx.x);
}

// ---- separate waits -------------------------------------------------------------------------
// When site processes SHARE a GPU (the one-GPU rehearsal), a launch whose every workgroup waits
// holds a wave slot on many CUs while it waits -- and a peer's persistent LSTM workgroup, which
// needs a whole CU's registers, then finds no CU, so the peer never reaches the push being waited
// for (cross-process deadlock broken only by the timeout: seen at 4 sites on one GPU).  There, each
// wait is its own ONE-workgroup launch ahead of the data launch (mode bit 2): it polls a
// contiguous range [lo, hi) of my flag words until every word is 1, clears them, and acquires;
// the data launch then runs without waiting.  One site per GPU (production) keeps the waits
// inside the data launches (one launch fewer per phase).
__global__ void __launch_bounds__(256) px_wait_kernel(unsigned* f, long lo, long hi, unsigned* err,
                                                      long timeout, unsigned code) {
  const long t0 = (long)__builtin_amdgcn_s_memrealtime();
  bool late = false;
  for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    while (px_get(f + i) != 1u) {
      if ((long)__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        late = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (late) break;
    px_set(f + i, 0u);
  }
  if (late) px_set(err, code);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");
}

// ---- factor all-gather --------------------------------------------------------------------------
// flags of site w: data at [sender * nsb + s], credits at [W * nsb + dest * nsb + s] (1 = the slot
// I write at site `dest` is free; initialised to 1 by the host, returned by dest's gcollect)

template <int T>
__global__ void __launch_bounds__(256) px_gpush_kernel(PxArgs a) {
  __shared__ float wm[4];
  const int s = blockIdx.x, d = blockIdx.y, W = a.W;
  const long nsb = a.chunk / SB;
  if (threadIdx.x == 0) px_take(a.flags[a.me] + W * nsb + (long)d * nsb + s, a, 0x300u | (unsigned)d);
  px_acquire_join(a.mode);
  float o[8];
  const int e = px_load_scaled<T>(a.src, (long)s * SB + 8 * threadIdx.x, a.n, a.scaled, o, wm);
  px_store_sb<T>(a.gath[d], ((long)a.me * nsb + s) * SBS, e, o);
  px_drain_release(a.mode);
  if (threadIdx.x == 0) px_set(a.flags[d] + (long)a.me * nsb + s, 1u);
}

template <int T>
__global__ void __launch_bounds__(256) px_gcollect_kernel(PxArgs a) {
  const int s = blockIdx.x, w = blockIdx.y, W = a.W;
  const long nsb = a.chunk / SB;
  if (threadIdx.x == 0) px_take(a.flags[a.me] + (long)w * nsb + s, a, 0x400u | (unsigned)w);
  px_acquire_join(a.mode);
  const long at = ((long)w * nsb + s) * SBS;
  const void* g = a.gath[a.me];
  const float sc = a.scale * exp2i(-px_ldexp<T>(g, at, a.mode));
  const long e0 = (long)s * SB + 8 * threadIdx.x;
  float o[8];
  if (e0 < a.n) {
    px_ldw8<T>(g, at, 1 + threadIdx.x, a.mode, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] *= sc;
    float* out = a.dst + (long)w * a.dstride;
    if (e0 + 8 <= a.n && (a.dstride & 7) == 0) {
      st8<PT_F32>(out, e0 / 8, o);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (e0 + k < a.n) out[e0 + k] = o[k];
    }
  }
  // every lane has read the slot: return its credit to the writer
  px_drain_release(a.mode);
  if (threadIdx.x == 0) px_set(a.flags[w] + W * nsb + (long)a.me * nsb + s, 1u);
}

}  // namespace

long g_dn_peer_timeout_ms = 20000;

DN_API int dn_peer_set_timeout_ms(long ms) {
  g_dn_peer_timeout_ms = ms < 0 ? 20000 : ms;
  return DN_OK;
}

// ---- arena: uncached HBM, exported / mapped through IPC handles --------------------------------
DN_API int dn_peer_alloc(long bytes, void** out) {
  if (bytes <= 0 || !out) return DN_BAD_SHAPE;
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    return DN_LAUNCH_FAILED;
  }
  if (hipMemset(p, 0, (size_t)bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    return DN_LAUNCH_FAILED;
  }
  *out = p;
  return DN_OK;
}

DN_API int dn_peer_free(void* p) { return hipFree(p) == hipSuccess ? DN_OK : DN_LAUNCH_FAILED; }

DN_API long dn_peer_handle_size() { return (long)sizeof(hipIpcMemHandle_t); }

DN_API int dn_peer_export(void* p, void* handle_out) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) {
    (void)hipGetLastError();
    return DN_LAUNCH_FAILED;
  }
  __builtin_memcpy(handle_out, &h, sizeof(h));
  return DN_OK;
}

DN_API int dn_peer_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
    (void)hipGetLastError();
    return DN_LAUNCH_FAILED;
  }
  *out = p;
  return DN_OK;
}

DN_API int dn_peer_close(void* p) {
  return hipIpcCloseMemHandle(p) == hipSuccess ? DN_OK : DN_LAUNCH_FAILED;
}

// host-side writes of flag words (credits start at 1) into my own arena
DN_API int dn_peer_fill_u32(unsigned* p, unsigned v, long count) {
  if (!p || count < 0) return DN_BAD_SHAPE;
  if (count && (hipMemsetD32(p, (int)v, (size_t)count) != hipSuccess ||
                hipDeviceSynchronize() != hipSuccess))
    return DN_LAUNCH_FAILED;
  return DN_OK;
}

// diagnostics: copy `bytes` of arena memory to the host (flag-state dumps after a timeout)
DN_API int dn_peer_peek(const void* src, void* host, long bytes) {
  if (!src || !host || bytes < 0) return DN_BAD_SHAPE;
  return hipMemcpy(host, src, (size_t)bytes, hipMemcpyDeviceToHost) == hipSuccess ? DN_OK
                                                                                   : DN_LAUNCH_FAILED;
}

DN_API long dn_peer_args_size() { return (long)sizeof(PxArgs); }

#define DN_PX_DISPATCH(T, KERNEL, ...)                                                           \
  switch (T) {                                                                                   \
    case PT_BF16: hipLaunchKernelGGL(KERNEL<PT_BF16>, __VA_ARGS__); break;                       \
    case PT_F16: hipLaunchKernelGGL(KERNEL<PT_F16>, __VA_ARGS__); break;                         \
    case PT_F32: hipLaunchKernelGGL(KERNEL<PT_F32>, __VA_ARGS__); break;                         \
    default: return DN_BAD_SHAPE;                                                                \
  }

static bool px_ok(const PxArgs& a) {
  if (a.W < 1 || a.W > PX_MAXW || a.me < 0 || a.me >= a.W || a.chunk <= 0 || a.chunk % SB ||
      a.n < 0 || !a.err)
    return false;
  for (int w = 0; w < a.W; ++w)
    if (!a.inbox[w] || !a.gath[w] || !a.flags[w]) return false;
  return (((uintptr_t)a.src | (uintptr_t)a.dst) & 15) == 0;
}

// the one-workgroup wait of `phase` (1 reduce, 2 unpack, 3 gpush, 4 gcollect) for my flag words
DN_API int dn_peer_wait(const PxArgs* args, int phase, hipStream_t st) {
  if (!args) return DN_BAD_SHAPE;
  const PxArgs& a = *args;
  if (!px_ok(a)) return DN_BAD_SHAPE;
  const long t = g_dn_spin_limit == 0 ? 0 : g_dn_peer_timeout_ms * 100000L;
  const long nsb = a.chunk / SB, W = a.W;
  long lo, hi;
  switch (phase) {
    case 1: lo = 0, hi = nsb * W; break;                 // rs flags of my chunk
    case 2: lo = nsb * W, hi = 2 * nsb * W; break;       // ag flags of every owner
    case 3: lo = W * nsb, hi = 2 * W * nsb; break;       // gather credits
    case 4: lo = 0, hi = W * nsb; break;                 // gather data
    default: return DN_BAD_SHAPE;
  }
  hipLaunchKernelGGL(px_wait_kernel, dim3(1), dim3(256), 0, st, a.flags[a.me], lo, hi, a.err, t,
                     (unsigned)(phase << 8) | 0xffu);
  return dn_launch_status();
}

// phase: 0 push, 1 reduce, 2 unpack (site-mean); 3 gpush, 4 gcollect (gather)
DN_API int dn_peer_launch(const PxArgs* args, int phase, int type, hipStream_t st) {
  if (!args) return DN_BAD_SHAPE;
  PxArgs a = *args;
  if (!px_ok(a)) return DN_BAD_SHAPE;
  const long t = g_dn_spin_limit == 0 ? 0 : g_dn_peer_timeout_ms * 100000L;
  a.timeout = t;
  const long nsb = a.chunk / SB;
  if (nsb > 65535) return DN_BAD_SHAPE;
  if ((phase == 0 || phase == 2) && (long)a.W * a.chunk < a.n) return DN_BAD_SHAPE;
  if (phase >= 3 && a.chunk < a.n) return DN_BAD_SHAPE;
  if (phase == 4 && a.dstride < a.n) return DN_BAD_SHAPE;
  const dim3 gw((unsigned)nsb, (unsigned)a.W), g1((unsigned)nsb);
  switch (phase) {
    case 0: DN_PX_DISPATCH(type, px_push_kernel, gw, dim3(256), 0, st, a); break;
    case 1: DN_PX_DISPATCH(type, px_reduce_kernel, g1, dim3(256), 0, st, a); break;
    case 2: DN_PX_DISPATCH(type, px_unpack_kernel, gw, dim3(256), 0, st, a); break;
    case 3: DN_PX_DISPATCH(type, px_gpush_kernel, gw, dim3(256), 0, st, a); break;
    case 4: DN_PX_DISPATCH(type, px_gcollect_kernel, gw, dim3(256), 0, st, a); break;
    default: return DN_BAD_SHAPE;
  }
  return dn_launch_status();
}
