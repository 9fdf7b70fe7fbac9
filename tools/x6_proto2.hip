// Prototype 2: fp32 GEMM on bf16x6 split products, each operand element split ONCE per block.
// Register-staged loads (two slabs ahead) -> split -> three bf16 planes in LDS (double-buffered,
// BK = 16: 72 KB per block, two blocks per CU) -> one v_mfma_f32_32x32x16_bf16 k-step per slab,
// 4 waves of 64 x 64 on a 128 x 128 tile.  Plain C = A B store; no split-K / epilogue kinds.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/x6_proto2.hip -o tools/libx6proto2.so
#include <hip/hip_runtime.h>

#include <cstdint>

namespace x6b {
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef short v4i16 __attribute__((ext_vector_type(4)));

constexpr int NT = 256, TB = 128, BK = 16;
constexpr int KC_PITCH = 48;            // bytes per KC plane row: 16 bf16 + 16 B pad (conflict-free b128 reads)
constexpr int PLANE = 128 * KC_PITCH;   // 6 KB (an RC plane: 16 k-rows x 256 B = 4 KB)
constexpr int OPER = 3 * PLANE, BUF = 2 * OPER;
constexpr int KC = 0, RC = 1;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}
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

// per-thread staging of one operand: 2 float4 per slab
//   KC: slot s = 256 i + tid: row s >> 2, k quad s & 3      -> plane byte row * 48 + 8 q
//   RC: slot s: k-row s >> 5, rows 4 (s & 31) .. +3        -> plane byte kr * 256 + swizzled chunk
template <int MODE>
struct Stage2 {
  uint32_t roff[2], lds[2];
  int kq[2];
  __device__ void init(int tid, int rows_left, int ld) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int s = 256 * i + tid;
      if constexpr (MODE == KC) {
        const int r = s >> 2, q = s & 3;
        roff[i] = (uint32_t)(min(r, rows_left - 1) * ld * 4);
        lds[i] = (uint32_t)(r * KC_PITCH + 8 * q);
        kq[i] = 4 * q;
      } else {
        const int kr = s >> 5, c = s & 31;
        roff[i] = (uint32_t)(min(4 * c, (rows_left - 1) & ~3) * 4);
        lds[i] = (uint32_t)(kr * 256 + (((c >> 1) ^ ((kr & 3) << 2)) << 4) + 8 * (c & 1));
        kq[i] = kr;
      }
    }
  }
  // sbase: the slab's base (tile base + k0 for KC, + k0 * ld for RC); offsets are slab-relative
  __device__ void load(const float* sbase, int ld, int k0, int K, float4 (&v)[2]) const {
    const __amdgpu_buffer_rsrc_t r = rsrc(sbase);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = k0 + kq[i];
      if constexpr (MODE == KC) {
        v[i] = ld16(r, roff[i] + 4u * (uint32_t)(min(k, (K - 1) & ~3) - k0));
        if (k0 + BK > K) {
          v[i].x = k + 0 < K ? v[i].x : 0.f;
          v[i].y = k + 1 < K ? v[i].y : 0.f;
          v[i].z = k + 2 < K ? v[i].z : 0.f;
          v[i].w = k + 3 < K ? v[i].w : 0.f;
        }
      } else {
        v[i] = ld16(r, roff[i] + 4u * (uint32_t)(min(k, K - 1) - k0) * (uint32_t)ld);
        if (k >= K) v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  __device__ void store(const float4 (&v)[2], char* planes) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bf16x4 h, m, l;
      split4(v[i], h, m, l);
      *reinterpret_cast<bf16x4*>(planes + lds[i]) = h;
      *reinterpret_cast<bf16x4*>(planes + PLANE + lds[i]) = m;
      *reinterpret_cast<bf16x4*>(planes + 2 * PLANE + lds[i]) = l;
    }
  }
};

template <int MODE>
__device__ __forceinline__ bf16x8 frag(const char* plane, int rbase, int lane) {
  const int h = lane >> 5, l32 = lane & 31;
  if constexpr (MODE == KC) {
    return *reinterpret_cast<const bf16x8*>(plane + (rbase + l32) * KC_PITCH + 16 * h);
  } else {
    const int g1 = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    const int mloc = rbase + 16 * g1 + 4 * p;
    const int off = (8 * h + q) * 256 + (((mloc >> 3) ^ (q << 2)) << 4) + 8 * (p & 1);
    const __attribute__((address_space(3))) char* s =
        (const __attribute__((address_space(3))) char*)(__attribute__((address_space(3))) const void*)plane;
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(s + off));
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(s + off + 4 * 256));
    const int2 a = __builtin_bit_cast(int2, lo), b = __builtin_bit_cast(int2, hi);
    return __builtin_bit_cast(bf16x8, make_int4(a.x, a.y, b.x, b.y));
  }
}

template <int MA, int MB>
__global__ __launch_bounds__(NT, 2) void gemm_x6b(int M, int N, int K, const float* A, int lda, const float* B, int ldb,
                                                 float* C, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;
  const int m0 = blockIdx.y * TB, n0 = blockIdx.x * TB;
  const float* abase = MA == KC ? A + (long)m0 * lda : A + m0;
  const float* bbase = MB == KC ? B + (long)n0 * ldb : B + n0;
  Stage2<MA> sa;
  Stage2<MB> sb;
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
  auto slab_a = [&](int k0) { return MA == KC ? abase + k0 : abase + (long)k0 * lda; };
  auto slab_b = [&](int k0) { return MB == KC ? bbase + k0 : bbase + (long)k0 * ldb; };
  float4 va[2][2], vb[2][2];
  sa.load(slab_a(0), lda, 0, K, va[0]);
  sb.load(slab_b(0), ldb, 0, K, vb[0]);
  if (nk > 1) {
    sa.load(slab_a(BK), lda, BK, K, va[1]);
    sb.load(slab_b(BK), ldb, BK, K, vb[1]);
  }
  sa.store(va[0], smem);
  sb.store(vb[0], smem + OPER);
  __syncthreads();
  auto step = [&](int kt, auto par) {
    constexpr int P = decltype(par)::value;  // kt % 2
    if (kt + 2 < nk) {
      const int k2 = (kt + 2) * BK;
      sa.load(slab_a(k2), lda, k2, K, va[P]);
      sb.load(slab_b(k2), ldb, k2, K, vb[P]);
    }
    const char* cur = smem + P * BUF;
    bf16x8 af[2][3], bf[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p) af[i][p] = frag<MA>(cur + p * PLANE, wm * 64 + i * 32, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p) bf[j][p] = frag<MB>(cur + OPER + p * PLANE, wn * 64 + j * 32, lane);
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
    if (kt + 1 < nk) {
      char* nxt = smem + (1 - P) * BUF;
      sa.store(va[1 - P], nxt);
      sb.store(vb[1 - P], nxt + OPER);
    }
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < nk) step(kt + 1, std::integral_constant<int, 1>{});
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
}  // namespace x6b

extern "C" int x6_gemm(int M, int N, int K, const float* A, int lda, int ma, const float* B, int ldb, int mb,
                       float* C, int ldc, void* stream) {
  dim3 grid((N + 127) / 128, (M + 127) / 128);
  hipStream_t st = (hipStream_t)stream;
  if (ma == 0 && mb == 0) hipLaunchKernelGGL((x6b::gemm_x6b<0, 0>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C, ldc);
  else if (ma == 0 && mb == 1) hipLaunchKernelGGL((x6b::gemm_x6b<0, 1>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C, ldc);
  else if (ma == 1 && mb == 0) hipLaunchKernelGGL((x6b::gemm_x6b<1, 0>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C, ldc);
  else hipLaunchKernelGGL((x6b::gemm_x6b<1, 1>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C, ldc);
  return (int)hipGetLastError();
}
