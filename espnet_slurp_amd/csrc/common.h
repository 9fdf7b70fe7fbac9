// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of espnet_slurp_amd.
// Wave = 64 lanes; all reductions are written for 64-wide wavefronts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "espnet_mi355.h"  // the C ABI; definitions below must match it

#define ESP_API extern "C" __attribute__((visibility("default")))

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

namespace esp {

// last error string (host side), set by ESP_CHECK_LAUNCH / argument validation
void set_error(const char* fmt, ...);

// ---------------------------------------------------------------- counter RNG
// Counter hash (seed, index) -> 32 random bits, 32-bit arithmetic only: one round of Wellons'
// lowbias32 finaliser (2 v_mul_lo_u32, quarter-rate on CDNA) over the index with the seed's
// halves injected (xor low, add high) and the index's high word folded in by a rotate.  Dropout
// masks are generated inside MFMA epilogues and softmax passes, where the hash is the dominant
// VALU cost (round 1 used two rounds + a multiply for the high word: 5 v_mul_lo_u32 per
// element; the fused attention kernel spent ~100 us of 410 per layer on it at C2).  A bijection
// of the low index word for a fixed seed.  Stateless, so the backward pass regenerates the
// forward dropout mask from the same (seed, index).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t rng_u32(uint64_t seed, uint64_t idx) {
  const uint32_t hi = (uint32_t)(idx >> 32);
  const uint32_t x = ((uint32_t)idx ^ (uint32_t)seed ^ ((hi << 16) | (hi >> 16))) + (uint32_t)(seed >> 32);
  return mix32(x);
}
// Optional device-resident dropout key (esp_set_rng_key): every dropout kernel XORs its seed
// with *key, so a captured HIP graph draws fresh masks on every replay (the key is advanced
// on device by esp_rng_advance) while the host-side seeds stay baked into the graph.
const uint64_t* rng_key_ptr();
__device__ __forceinline__ uint64_t keyed(uint64_t seed, const uint64_t* key) { return key ? seed ^ *key : seed; }
// Dropout keep decision, probability (1-p) with threshold = p * 2^32 (host).  Each 32-bit hash
// serves an element PAIR (2k, 2k+1), 16 bits each against the threshold rounded to 1/65536
// (p = 0.1 -> 0.1000061): kernels that own consecutive elements draw half the hashes
// (keep_pair), and every other site still draws element by element — the same masks.
__device__ __forceinline__ uint32_t thr16_of(uint32_t thresh) {
  return (uint32_t)(((uint64_t)thresh + 32768u) >> 16);
}
// Host: the 32-bit threshold of dropout probability p, already on the 1/65536 grid the kernels
// compare against (thr16 << 16, so thr16_of returns thr16 exactly).  p > 0 never quantizes to
// "no dropout": p below half a quantum takes the smallest one (1/65536).  0 means no dropout.
// Callers reject p >= 1 (ESP_ARG_CHECK): the 16-bit grid has no all-drop threshold.
inline uint32_t drop_threshold(float p) {
  if (!(p > 0.f)) return 0;
  double q = (double)p * 65536.0 + 0.5;
  uint32_t t16 = q >= 65535.0 ? 65535u : (uint32_t)q;
  if (t16 == 0) t16 = 1;
  return t16 << 16;
}
// Host: the inverted-dropout rescale matching the quantized keep probability exactly,
// 1 / (1 - thr16 / 65536), so E[mask * scale] = 1 (1/(1-p) with the unrounded p would bias
// every dropout site by ~7e-6 at p = 0.1).
inline float drop_scale(uint32_t thresh) {
  if (!thresh) return 1.f;
  const uint32_t t16 = (uint32_t)(((uint64_t)thresh + 32768u) >> 16);
  return (float)(65536.0 / (65536.0 - (double)t16));
}
__device__ __forceinline__ bool keep_elem(uint64_t seed, uint64_t idx, uint32_t thresh) {
  const uint32_t h = rng_u32(seed, idx >> 1);
  return ((idx & 1) ? (h >> 16) : (h & 0xffffu)) >= thr16_of(thresh);
}
// elements idx_even and idx_even + 1 (idx_even even) from one hash
__device__ __forceinline__ void keep_pair(uint64_t seed, uint64_t idx_even, uint32_t thresh, bool& k0, bool& k1) {
  const uint32_t h = rng_u32(seed, idx_even >> 1), t = thr16_of(thresh);
  k0 = (h & 0xffffu) >= t;
  k1 = (h >> 16) >= t;
}
// the same for indices < 2^32 (the caller's whole index range): rng_u32's high-word fold is 0
// there, so these draw exactly the masks of keep_pair, on 32-bit index arithmetic
__device__ __forceinline__ void keep_pair32(uint64_t seed, uint32_t idx_even, uint32_t thresh, bool& k0, bool& k1) {
  const uint32_t h = mix32(((idx_even >> 1) ^ (uint32_t)seed) + (uint32_t)(seed >> 32)), t = thr16_of(thresh);
  k0 = (h & 0xffffu) >= t;
  k1 = (h >> 16) >= t;
}
__device__ __forceinline__ bool keep_elem32(uint64_t seed, uint32_t idx, uint32_t thresh) {
  const uint32_t h = mix32(((idx >> 1) ^ (uint32_t)seed) + (uint32_t)(seed >> 32));
  return ((idx & 1) ? (h >> 16) : (h & 0xffffu)) >= thr16_of(thresh);
}

// sigmoid on the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32, ~1 ulp each) instead of libm
// expf + an IEEE division (~30-45 VALU per element: the bulk of the FFN w_1 epilogue, 293 vs 210 us
// for the same GEMM shape with a one-multiply epilogue at C2).  Saturates cleanly: e -> inf gives 0.
__device__ __forceinline__ float fast_sigmoid(float v) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v * -1.4426950408889634f));
}

// ---------------------------------------------------------------- fp32 -> bf16 split planes
// v = hi + mid + lo exactly (finite v): hi = bf16(v), mid = bf16(v - hi), lo = bf16(v - hi - mid),
// round to nearest even, both residuals exact fp32 differences.  One element pair per call, each part
// packed as bf16x2 (element a in the low half).  Defined for finite a, b only: with ESP_SPLIT_DOT the
// residual is a dot over the packed pair, so an inf / NaN partner (or |b| rounding to a bf16 inf) makes the
// finite element's residual NaN (0 * inf); non-finite operands give a non-finite GEMM output either way,
// and the Trainer skips such a step (its finite check), so only non-finite results meet non-finite ones: one v_cvt_pk_bf16_f32 per part, the parts' fp32
// values taken back from the packed bits.  The GEMMs' in-register split (gemm_kernels.h
// split3_bf16) and every producer of planes (esp_f32_to_planes, LayerNorm, GEMM epilogues) use this,
// so a planes operand holds exactly the values the in-register split would form.
// ESP_SPLIT_DOT 1 (default): each residual is one v_dot2c_f32_bf16, r = v + (-1) * bf16part, which
// takes the part straight from the packed pair (no unpack): 7 VALU per pair instead of 11 (the split is
// the in-register GEMMs' VALU bound: 11 VALU per pair ~ the MFMA time of the six products,
// profiles/r05m_*).  The residual is exactly representable, so it is exact under any rounding of the
// dot's sum; 0: the unpack + v_sub form.
#ifndef ESP_SPLIT_DOT
#define ESP_SPLIT_DOT 1
#endif
__device__ __forceinline__ void split3_pair(float a, float b, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 b2;
  const b2 hp = __builtin_convertvector((f2){a, b}, b2);
#if ESP_SPLIT_DOT
  // the (-1, 0) / (0, -1) bf16 pairs from SGPRs: as an inline constant the assembler encodes (-1, 0) as
  // the fp32 -1.0, which the hardware reads as the pair (0, -1)
  uint32_t na, nb;
  asm("s_mov_b32 %0, 0xbf80" : "=s"(na));
  asm("s_mov_b32 %0, 0xbf800000" : "=s"(nb));
  const b2 NA = __builtin_bit_cast(b2, na), NB = __builtin_bit_cast(b2, nb);
  const float ra = __builtin_amdgcn_fdot2_f32_bf16(hp, NA, a, false);
  const float rb = __builtin_amdgcn_fdot2_f32_bf16(hp, NB, b, false);
  const b2 mp = __builtin_convertvector((f2){ra, rb}, b2);
  const float sa = __builtin_amdgcn_fdot2_f32_bf16(mp, NA, ra, false);
  const float sb = __builtin_amdgcn_fdot2_f32_bf16(mp, NB, rb, false);
#else
  const uint32_t hu = __builtin_bit_cast(uint32_t, hp);
  const float ra = a - __uint_as_float(hu << 16), rb = b - __uint_as_float(hu & 0xffff0000u);
  const b2 mp = __builtin_convertvector((f2){ra, rb}, b2);
  const uint32_t mu = __builtin_bit_cast(uint32_t, mp);
  const float sa = ra - __uint_as_float(mu << 16), sb = rb - __uint_as_float(mu & 0xffff0000u);
#endif
  hi = __builtin_bit_cast(uint32_t, hp);
  mid = __builtin_bit_cast(uint32_t, mp);
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){sa, sb}, b2));
}
// bf16x2 (round to nearest even) of a pair: the n = 1 "planes" (the reduced-precision operand)
__device__ __forceinline__ uint32_t bf16_pair(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 b2;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){a, b}, b2));
}
// store 4 consecutive values (c % 4 == 0) of a planes matrix: n = 3 split planes or n = 1 bf16 plane
__device__ __forceinline__ void store_planes4(uint16_t* y, long off, long ps, int n, float a, float b, float c,
                                              float d) {
  if (n == 3) {
    uint32_t h0, m0, l0, h1, m1, l1;
    split3_pair(a, b, h0, m0, l0);
    split3_pair(c, d, h1, m1, l1);
    *reinterpret_cast<uint2*>(y + off) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(y + off + ps) = make_uint2(m0, m1);
    *reinterpret_cast<uint2*>(y + off + 2 * ps) = make_uint2(l0, l1);
  } else {
    *reinterpret_cast<uint2*>(y + off) = make_uint2(bf16_pair(a, b), bf16_pair(c, d));
  }
}

// ---------------------------------------------------------------- reductions (wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block reduction, blockDim.x multiple of 64, up to 1024 threads; result broadcast
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* sh /* >= 16 */) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if constexpr (sizeof(T) == 8) v = wave_sum_d(v); else v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  T r = 0;
  for (int i = 0; i < nw; ++i) r += sh[i];
  return r;
}
template <typename T = float>
__device__ __forceinline__ T block_max(T v, T* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  T r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmax(r, sh[i]);
  return r;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

}  // namespace esp

#define ESP_CHECK_LAUNCH(name)                                              \
  do {                                                                      \
    hipError_t e__ = hipGetLastError();                                     \
    if (e__ != hipSuccess) {                                                \
      esp::set_error("%s: %s", name, hipGetErrorString(e__));               \
      return (int)e__;                                                      \
    }                                                                       \
  } while (0)

#define ESP_ARG_CHECK(cond, ...)          \
  do {                                    \
    if (!(cond)) {                        \
      esp::set_error(__VA_ARGS__);        \
      return -1;                          \
    }                                     \
  } while (0)
