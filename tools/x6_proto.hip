// Prototype: fp32 GEMM on bf16x6 split products with the split done ONCE per element per block
// (register-staged loads -> split -> three bf16 planes in LDS), instead of by every wave that
// reads a fragment (the LDS-DMA kernel's in-register split: 7.3 VALU per MFMA on 64x64 wave tiles).
// C (M x N, ldc) = A B, A in mode KC ([M][K], lda) or RC ([K][M]), B in KC ([N][K]) or RC ([K][N]).
// 128 x 128 tiles, 4 waves (2 x 2, 64 x 64 each), BK = 32, planes double-buffered (120 KB: one
// block per CU), one slab of register prefetch, one barrier per slab.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/x6_proto.hip -o tools/libx6proto.so
// Measurement record only: its K-tail path is wrong for K % 32 != 0 (the quad offset
// is added twice); tools/x6_proto2.hip is the corrected 16-k-slab version.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace x6 {
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256, TB = 128, BK = 32;
constexpr int KC_PITCH = 80;                // bytes per plane row of a KC operand (32 bf16 + 16 B pad)
constexpr int PLANE = 128 * KC_PITCH;       // 10 KB: a KC plane (an RC plane uses 32 x 256 B = 8 KB)
constexpr int OPER = 3 * PLANE, BUF = 2 * OPER;  // per operand, per buffer (A then B)
constexpr int KC = 0, RC = 1;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}

// v = hi + mid + lo exactly (round-to-nearest-even residuals)
__device__ __forceinline__ void split4(float4 v, bf16x4& hi, bf16x4& mid, bf16x4& lo) {
  const float a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 h = (__bf16)a[e];
    const float r = a[e] - (float)h;
    const __bf16 m = (__bf16)r;
    hi[e] = h;
    mid[e] = m;
    lo[e] = (__bf16)(r - (float)m);
  }
}

// One operand's per-thread staging: 4 float4 per slab.
//   KC: slot s = 256 i + tid: row s >> 3, k quad s & 7            -> plane byte  row * 80 + 8 q
//   RC: slot s: k-row s >> 5, row chunk (s & 31) * 4 (4 rows)     -> plane byte  kr * 256 + swizzled chunk
template <int MODE>
struct Stage3 {
  uint32_t voff[4];
  uint32_t lds[4];
  int kq[4];  // KC: k offset (4 q) in the slab; RC: k-row
  __device__ void init(int tid, int rows_left, int ld) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s = 256 * i + tid;
      if constexpr (MODE == KC) {
        const int r = s >> 3, q = s & 7;
        const int rr = min(r, rows_left - 1);
        voff[i] = (uint32_t)((rr * ld + 4 * q) * 4);
        lds[i] = (uint32_t)(r * KC_PITCH + 8 * q);
        kq[i] = 4 * q;
      } else {
        const int kr = s >> 5, c = s & 31;
        const int m = min(4 * c, (rows_left - 1) & ~3);
        voff[i] = (uint32_t)((kr * ld + m) * 4);
        lds[i] = (uint32_t)(kr * 256 + ((((c >> 1) ^ ((kr & 3) << 2))) << 4) + 8 * (c & 1));
        kq[i] = kr;
      }
    }
  }
  // slab at k0: base = operand tile base (row / column offset applied)
  __device__ void load(const float* base, int ld, int k0, int K, float4 (&v)[4]) const {
    if (k0 + BK <= K) {
      const __amdgpu_buffer_rsrc_t r = rsrc(MODE == KC ? base + k0 : base + (long)k0 * ld);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = ld16(r, voff[i]);
    } else {  // K tail: clamp the source, zero k >= K
      const __amdgpu_buffer_rsrc_t r = rsrc(base);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (MODE == KC) {
          const int k = min(k0 + kq[i], (K - 1) & ~3);
          v[i] = ld16(r, voff[i] + 4u * (uint32_t)k);
          const int kt = k0 + kq[i];
          v[i].x = kt + 0 < K ? v[i].x : 0.f;
          v[i].y = kt + 1 < K ? v[i].y : 0.f;
          v[i].z = kt + 2 < K ? v[i].z : 0.f;
          v[i].w = kt + 3 < K ? v[i].w : 0.f;
        } else {
          const int k = min(k0 + kq[i], K - 1);
          v[i] = ld16(r, voff[i] + 4u * (uint32_t)k * (uint32_t)ld);
          if (k0 + kq[i] >= K) v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  }
  __device__ void store(const float4 (&v)[4], char* planes) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x4 h, m, l;
      split4(v[i], h, m, l);
      *reinterpret_cast<bf16x4*>(planes + lds[i]) = h;
      *reinterpret_cast<bf16x4*>(planes + PLANE + lds[i]) = m;
      *reinterpret_cast<bf16x4*>(planes + 2 * PLANE + lds[i]) = l;
    }
  }
};

// fragment of 32 rows starting at rbase, MFMA step st (k = 16 st + 8 h + 0..7), plane p
template <int MODE>
__device__ __forceinline__ bf16x8 frag(const char* plane, int rbase, int st, int lane) {
  const int h = lane >> 5, l32 = lane & 31;
  if constexpr (MODE == KC) {
    return *reinterpret_cast<const bf16x8*>(plane + (rbase + l32) * KC_PITCH + (16 * st + 8 * h) * 2);
  } else {
    const int g1 = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    const int mloc = rbase + 16 * g1 + 4 * p;
    const int kb = 16 * st + 8 * h;
    const int off = (kb + q) * 256 + (((mloc >> 3) ^ (q << 2)) << 4) + 8 * (p & 1);
    const __attribute__((address_space(3))) char* s =
        (const __attribute__((address_space(3))) char*)(__attribute__((address_space(3))) const void*)plane;
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(s + off));
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(s + off + 4 * 256));
    const int2 a = __builtin_bit_cast(int2, lo), b = __builtin_bit_cast(int2, hi);
    return __builtin_bit_cast(bf16x8, make_int4(a.x, a.y, b.x, b.y));
  }
}

template <int MA, int MB>
__global__ __launch_bounds__(NT, 1) void gemm_x6(int M, int N, int K, const float* A, int lda, const float* B, int ldb,
                                                float* C, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;
  const int m0 = blockIdx.y * TB, n0 = blockIdx.x * TB;
  const float* abase = MA == KC ? A + (long)m0 * lda : A + m0;
  const float* bbase = MB == KC ? B + (long)n0 * ldb : B + n0;
  Stage3<MA> sa;
  Stage3<MB> sb;
  sa.init(tid, M - m0, lda);
  sb.init(tid, N - n0, ldb);
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (K + BK - 1) / BK;
  float4 va[4], vb[4];
  sa.load(abase, lda, 0, K, va);
  sb.load(bbase, ldb, 0, K, vb);
  sa.store(va, smem);
  sb.store(vb, smem + OPER);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      sa.load(abase, lda, (kt + 1) * BK, K, va);
      sb.load(bbase, ldb, (kt + 1) * BK, K, vb);
    }
    const char* cur = smem + (kt & 1) * BUF;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      bf16x8 af[2][3], bf[2][3];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) af[i][p] = frag<MA>(cur + p * PLANE, wm * 64 + i * 32, st, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int p = 0; p < 3; ++p) bf[j][p] = frag<MB>(cur + OPER + p * PLANE, wn * 64 + j * 32, st, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][1], bf[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][2], bf[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bf[j][2], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][1], bf[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bf[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bf[j][0], acc[i][j], 0, 0, 0);
        }
    }
    if (more) {
      char* nxt = smem + ((kt + 1) & 1) * BUF;
      sa.store(va, nxt);
      sb.store(vb, nxt + OPER);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M && n < N) C[(long)m * ldc + n] = acc[i][j][r];
      }
    }
}
}  // namespace x6

extern "C" int x6_gemm(int M, int N, int K, const float* A, int lda, int ma, const float* B, int ldb, int mb,
                       float* C, int ldc, void* stream) {
  dim3 grid((N + 127) / 128, (M + 127) / 128);
  hipStream_t st = (hipStream_t)stream;
  if (ma == 0 && mb == 0) hipLaunchKernelGGL((x6::gemm_x6<0, 0>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C, ldc);
  else if (ma == 0 && mb == 1) hipLaunchKernelGGL((x6::gemm_x6<0, 1>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C, ldc);
  else if (ma == 1 && mb == 0) hipLaunchKernelGGL((x6::gemm_x6<1, 0>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C, ldc);
  else hipLaunchKernelGGL((x6::gemm_x6<1, 1>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C, ldc);
  return (int)hipGetLastError();
}
