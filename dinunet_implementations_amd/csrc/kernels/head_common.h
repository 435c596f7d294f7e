// Helpers shared by the fused MLP-head kernels (mlp_head.hip: batch <= 64, head_big.hip:
// any batch): dropout hash, LDS transpose fragment reads, column sums of MFMA accumulators.
#pragma once
#include "common.h"

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__host__ __device__ constexpr int rup32(int v) { return (v + 31) & ~31; }

// 32-bit counter hash (Wellons' lowbias32 finaliser over idx ^ key(seed, layer)): two 32-bit
// multiplies per hash.  The former 64-bit splitmix finaliser (six 64-bit multiplies, each a
// chain of quarter-rate 32-bit ones) made the layer-0 dropout the longest phase of the forward.
__device__ __forceinline__ uint32_t hmix(uint64_t seed, uint32_t layer, uint32_t idx) {
  const uint32_t key = (uint32_t)seed * 0x9E3779B9u ^ (uint32_t)(seed >> 32) * 0x85EBCA6Bu ^
                       (layer + 1u) * 0xC2B2AE35u;
  uint32_t x = idx ^ key;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// Keep decision of element (m, k) of a [.][K] activation: one hash serves the element PAIR
// idx / 2 (16 uniform bits each: low half for even idx, high half for odd), so a lane holding
// consecutive elements (every kernel's vector loads) hashes once per two -- the quarter-rate
// multiplies of the layer-0 input dropout were ~2 us of the replicated head's prologue.  Keep
// probabilities resolve to 2^-16.
__device__ __forceinline__ bool hkeep(uint64_t seed, int layer, int m, int k, int K, float p) {
  const uint32_t idx = (uint32_t)(m * K + k);
  const uint32_t h = hmix(seed, (uint32_t)layer, idx >> 1);
  const uint32_t u = (idx & 1u) ? (h >> 16) : (h & 0xffffu);
  return (float)u * (1.f / 65536.f) >= p;
}

// sum over the four lanes holding one accumulator column (l, l^16, l^32, l^48)
__device__ __forceinline__ float colsum4(float v) {
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

// Fragment with lane i <- column c0 + (i & 15) and element j <- row k0 + 8 * (i >> 4) + j of a
// row-major LDS image (row stride S elements): two hardware-transposed 4x16 reads.
__device__ __forceinline__ bf16x8 tr_frag(const bf16* img, int S, int c0, int k0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const bf16* a0 = img + (k0 + 8 * g + q) * S + c0 + 4 * p;
  const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * S));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
}

}  // namespace
// Any-batch head (head_big.hip): same arguments and workspace contract as dn_head_layout /
// dn_head_fwd / dn_head_bwd, which forward here for batches above the single-workgroup kernels.
int headb_layout(int nl, const int* dims, const int* flags, int B, long* out);
int headb_fwd(int nl, const int* dims, const int* flags, const float* drops, const float* bnp,
              void* const* ptrs, const float* x, long ldx, int B, const long long* y, float* out,
              float* loss, long long* pred, unsigned long long* rng, void* ws, int train,
              int log_out, hipStream_t st);
int headb_bwd(int nl, const int* dims, const int* flags, const float* drops, const float* bnp,
              void* const* ptrs, int B, void* ws, const float* dloss, float* dx, long lddx,
              hipStream_t st);
