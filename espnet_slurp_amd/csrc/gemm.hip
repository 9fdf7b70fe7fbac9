// FP32 MFMA GEMM for gfx950 (v_mfma_f32_32x32x2_f32: exact f32 fma chain, 64 FLOP/clk/SIMD).
//
//   C[z](m,n) = alpha * epi( sum_k A[z](m,k) * B[z](k,n) + bias[n] ) + beta * R[z](m,n)
//
// Operand access modes (template):
//   KC     element (r,k) at p[r*ld + k]      (A row-major [M][K] / B as [N][K] = W of nn.Linear)
//   RC     element (r,k) at p[k*ld + r]      (A as [K][M] / B row-major [K][N])
//   I2C_KC im2col view of an NHWC map, (r = output pixel, k = (kt,kf,c))   [conv2 forward, A]
//   I2C_RC same map with roles swapped (r = (kt,kf,c), k = output pixel)   [conv2 dW, B]
// Batches: z = z1*nb2 + z2, operand offset = z1*s1 + z2*s2 (two-level strides cover the
// (batch, head) layouts of attention without copies).
//
// Tiling: 128x128 block tile, BK=16, 256 threads = 4 waves (2x2), each wave 64x64 =
// 2x2 MFMA 32x32 tiles. A lane of half h uses k = 8h+s for MFMA step s (both operands agree);
// see store_slab/load_frag for the two LDS images. Global->LDS is register-staged and double
// buffered (next slab's loads are issued before the current slab's MFMAs).
// Epilogue (fused): bias, ReLU/Swish (pre-activation optionally stored to `aux`),
// counter-RNG dropout, alpha scale and beta*R residual.
#include <stdlib.h>

#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;  // BK: split-K granularity

enum Mode { KC = 0, RC = 1, I2C_KC = 2, I2C_RC = 3 };
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SWISH = 2 };

struct Im2col {  // NHWC input map [Bn][H][W][C], 3x3 kernel, stride 2, no padding
  int H, W, C, Ho, Wo;
};

struct Operand {
  const float* p;
  long ld;
  long s1, s2;
  int vec;  // float4 along the contiguous dim is legal
  Im2col ic;
};

struct GemmArgs {
  int M, N, K, nb2;
  Operand a, b;
  float* c;
  long ldc, c1, c2;
  const float* r;  // residual (same layout as C), may alias c
  float* aux;      // pre-activation store (same layout as C)
  const float* bias;
  float alpha, beta;
  int act;
  uint32_t drop_thresh;  // 0 = no dropout
  float drop_scale;
  uint64_t seed;
  int batch;
  int splits, kchunk;  // split-K: blockIdx.z = z*splits + split; partials -> work
  float* work;
};

// fused epilogue for output element (z, m, n) with raw accumulator `acc`
__device__ __forceinline__ void epi_store(const GemmArgs& g, int z, int m, int n, float acc) {
  const int z1 = z / g.nb2, z2 = z - z1 * g.nb2;
  const long off = (long)z1 * g.c1 + (long)z2 * g.c2 + (long)m * g.ldc + n;
  float v = acc + (g.bias ? g.bias[n] : 0.f);
  if (g.aux) g.aux[off] = v;
  if (g.act == ACT_RELU) v = fmaxf(v, 0.f);
  else if (g.act == ACT_SWISH) v = v / (1.0f + expf(-v));
  if (g.drop_thresh) {
    const uint64_t idx = ((uint64_t)z * g.M + m) * (uint64_t)g.N + n;
    v = esp::keep_elem(g.seed, idx, g.drop_thresh) ? v * g.drop_scale : 0.f;
  }
  v *= g.alpha;
  if (g.r) v += g.beta * g.r[off];
  g.c[off] = v;
}

// address of im2col element: pixel index `pix` of the output grid, column `col` = (kt,kf,c)
__device__ __forceinline__ const float* i2c_ptr(const float* base, const Im2col& ic, long pix, int col) {
  const int hw = ic.Ho * ic.Wo;
  const long bi = pix / hw;
  const int rem = (int)(pix - bi * hw);
  const int ho = rem / ic.Wo, wo = rem - (rem / ic.Wo) * ic.Wo;
  const int kk = col / ic.C, c = col - kk * ic.C;
  const int kt = kk / 3, kf = kk - kt * 3;
  return base + (((bi * ic.H + 2 * ho + kt) * (long)ic.W) + 2 * wo + kf) * ic.C + c;
}

// Load this thread's NL float4 pieces of a (128 rows x BKT) operand slab into registers.
// rows = M (A) or N (B); row0 = tile origin; k0 = slab origin; K = end of this split's range.
template <int MODE, int BKT>
__device__ __forceinline__ void load_slab(const Operand& op, const float* base, int rows, int K,
                                          int row0, int k0, float4 (&reg)[BKT / 8]) {
  constexpr int QPR = BKT / 4;  // quads per row (KC)
#pragma unroll
  for (int it = 0; it < BKT / 8; ++it) {
    const int idx = threadIdx.x + it * NT;
    if constexpr (MODE == KC || MODE == I2C_KC) {
      const int r = idx / QPR, kq = (idx % QPR) * 4;
      const int gr = row0 + r, gk = k0 + kq;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gr < rows) {
        if (MODE == KC) {
          const float* p = base + (long)gr * op.ld + gk;
          if (op.vec && gk + 3 < K) {
            v = *reinterpret_cast<const float4*>(p);
          } else {
            if (gk + 0 < K) v.x = p[0];
            if (gk + 1 < K) v.y = p[1];
            if (gk + 2 < K) v.z = p[2];
            if (gk + 3 < K) v.w = p[3];
          }
        } else {
          if (gk + 3 < K) {  // C % 4 == 0 enforced on host: quad never straddles a tap
            v = *reinterpret_cast<const float4*>(i2c_ptr(base, op.ic, gr, gk));
          } else {
            if (gk + 0 < K) v.x = *i2c_ptr(base, op.ic, gr, gk + 0);
            if (gk + 1 < K) v.y = *i2c_ptr(base, op.ic, gr, gk + 1);
            if (gk + 2 < K) v.z = *i2c_ptr(base, op.ic, gr, gk + 2);
          }
        }
      }
      reg[it] = v;
    } else {
      // BKT k-rows x 32 quads along r
      const int kr = idx >> 5, rq = (idx & 31) * 4;
      const int gk = k0 + kr, gr = row0 + rq;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gk < K) {
        if (MODE == RC) {
          const float* p = base + (long)gk * op.ld + gr;
          if (op.vec && gr + 3 < rows) {
            v = *reinterpret_cast<const float4*>(p);
          } else {
            if (gr + 0 < rows) v.x = p[0];
            if (gr + 1 < rows) v.y = p[1];
            if (gr + 2 < rows) v.z = p[2];
            if (gr + 3 < rows) v.w = p[3];
          }
        } else {
          if (gr + 3 < rows) {
            v = *reinterpret_cast<const float4*>(i2c_ptr(base, op.ic, gk, gr));
          } else {
            if (gr + 0 < rows) v.x = *i2c_ptr(base, op.ic, gk, gr + 0);
            if (gr + 1 < rows) v.y = *i2c_ptr(base, op.ic, gk, gr + 1);
            if (gr + 2 < rows) v.z = *i2c_ptr(base, op.ic, gk, gr + 2);
          }
        }
      }
      reg[it] = v;
    }
  }
}

// LDS images (no transposition on either side):
//   KC operands  [row][BKT+4] : float4 along k written as loaded; a lane's BKT/2 k-values are
//                               BKT/8 ds_read_b128 (stride (BKT+4) floats = odd # of quads:
//                               16 distinct rows hit 16 distinct 16-B slots, conflict-free)
//   RC operands  [BKT][128+4] : float4 along rows written as loaded; a lane reads its row's
//                               value per k with ds_read_b32 (32 consecutive floats per half)
constexpr int LDS_RC = BM + 4;
template <int BKT>
struct Lds {
  static constexpr int KC_S = BKT + 4;
  static constexpr int TILE = (BM * KC_S > BKT * LDS_RC) ? BM * KC_S : BKT * LDS_RC;
};

template <int MODE, int BKT>
__device__ __forceinline__ void store_slab(float* lds, const float4 (&reg)[BKT / 8]) {
  constexpr int QPR = BKT / 4;
#pragma unroll
  for (int it = 0; it < BKT / 8; ++it) {
    const int idx = threadIdx.x + it * NT;
    if constexpr (MODE == KC || MODE == I2C_KC) {
      const int r = idx / QPR, kq = idx % QPR;
      *reinterpret_cast<float4*>(lds + r * Lds<BKT>::KC_S + kq * 4) = reg[it];
    } else {
      const int kr = idx >> 5, rq = (idx & 31) * 4;
      *reinterpret_cast<float4*>(lds + kr * LDS_RC + rq) = reg[it];
    }
  }
}

// the KH = BKT/2 k-values (k = KH*h + s) of row `r` of the current slab
template <int MODE, int BKT>
__device__ __forceinline__ void load_frag(const float* lds, int r, int h, float (&f)[BKT / 2]) {
  constexpr int KH = BKT / 2;
  if constexpr (MODE == KC || MODE == I2C_KC) {
#pragma unroll
    for (int q = 0; q < KH / 4; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(lds + r * Lds<BKT>::KC_S + KH * h + 4 * q);
      f[4 * q + 0] = v.x; f[4 * q + 1] = v.y; f[4 * q + 2] = v.z; f[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < KH; ++q) f[q] = lds[(KH * h + q) * LDS_RC + r];
  }
}

// half hs (0/1) of the BK=32 fragment: k = 16h + 8hs + q, q = 0..7
template <int MODE>
__device__ __forceinline__ void load_frag_half(const float* lds, int r, int h, int hs, float (&f)[8]) {
  if constexpr (MODE == KC || MODE == I2C_KC) {
    const float* p = lds + r * Lds<32>::KC_S + 16 * h + 8 * hs;
    const float4 v0 = *reinterpret_cast<const float4*>(p);
    const float4 v1 = *reinterpret_cast<const float4*>(p + 4);
    f[0] = v0.x; f[1] = v0.y; f[2] = v0.z; f[3] = v0.w;
    f[4] = v1.x; f[5] = v1.y; f[6] = v1.z; f[7] = v1.w;
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = lds[(16 * h + 8 * hs + q) * LDS_RC + r];
  }
}

// one slab of MFMAs on the fragments in registers
template <int KH>
__device__ __forceinline__ void mfma_slab(f32x16 (&acc)[2][2], const float (&af)[2][KH], const float (&bf)[2][KH]) {
#pragma unroll
  for (int s = 0; s < KH; ++s)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
}

// VARIANT 0: BK=16, register-staged double-buffered LDS (next slab's global loads in flight
//            during this slab's MFMAs), one barrier per slab.
// VARIANT 1: BK=32, single LDS buffer, no software pipelining (two barriers per slab); the
//            overlap comes from 4 resident blocks per CU (36 KB LDS, ~110 VGPRs each).
// VARIANT 2: BK=32, register-staged prefetch of slab k+1 during slab k's MFMAs into a
//            single LDS buffer (two barriers per slab; 2 waves/SIMD by VGPRs).
// VARIANT 3: VARIANT 1 with the slab's MFMAs in two halves (fragments for 8 k-steps live at a
//            time) so the kernel fits 128 VGPRs: 4 waves/SIMD.
template <int MA, int MB, int VARIANT>
__global__ __launch_bounds__(NT, VARIANT == 3 ? 4 : 2) void gemm_f32_kernel(GemmArgs g) {
  constexpr int BKT = VARIANT == 0 ? 16 : 32;
  constexpr int KH = BKT / 2;
  constexpr int NBUF = VARIANT == 0 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) float As[NBUF][Lds<BKT>::TILE];
  __shared__ __attribute__((aligned(16))) float Bs[NBUF][Lds<BKT>::TILE];

  const int split = blockIdx.z % g.splits;
  const int z = blockIdx.z / g.splits;
  const int z1 = z / g.nb2, z2 = z - z1 * g.nb2;
  const int kbeg = split * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const float* Ab = g.a.p + z1 * g.a.s1 + z2 * g.a.s2;
  const float* Bb = g.b.p + z1 * g.b.s1 + z2 * g.b.s2;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, l32 = lane & 31;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float4 ra[BKT / 8], rb[BKT / 8];
  const int nk = kend > kbeg ? (kend - kbeg + BKT - 1) / BKT : 0;
  if constexpr (VARIANT == 0) {
    load_slab<MA, BKT>(g.a, Ab, g.M, kend, m0, kbeg, ra);
    load_slab<MB, BKT>(g.b, Bb, g.N, kend, n0, kbeg, rb);
    store_slab<MA, BKT>(As[0], ra);
    store_slab<MB, BKT>(Bs[0], rb);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) {
        load_slab<MA, BKT>(g.a, Ab, g.M, kend, m0, kbeg + (kt + 1) * BKT, ra);
        load_slab<MB, BKT>(g.b, Bb, g.N, kend, n0, kbeg + (kt + 1) * BKT, rb);
      }
      float af[2][KH], bf[2][KH];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        load_frag<MA, BKT>(As[cur], wm * 64 + t * 32 + l32, h, af[t]);
        load_frag<MB, BKT>(Bs[cur], wn * 64 + t * 32 + l32, h, bf[t]);
      }
      mfma_slab<KH>(acc, af, bf);
      if (kt + 1 < nk) {
        store_slab<MA, BKT>(As[cur ^ 1], ra);
        store_slab<MB, BKT>(Bs[cur ^ 1], rb);
      }
      __syncthreads();
    }
  } else if constexpr (VARIANT == 2) {  // NOLINT
    if (nk > 0) {
      load_slab<MA, BKT>(g.a, Ab, g.M, kend, m0, kbeg, ra);
      load_slab<MB, BKT>(g.b, Bb, g.N, kend, n0, kbeg, rb);
    }
    for (int kt = 0; kt < nk; ++kt) {
      if (kt > 0) __syncthreads();  // previous slab fully read
      store_slab<MA, BKT>(As[0], ra);
      store_slab<MB, BKT>(Bs[0], rb);
      __syncthreads();
      if (kt + 1 < nk) {  // next slab's global loads fly during this slab's MFMAs
        load_slab<MA, BKT>(g.a, Ab, g.M, kend, m0, kbeg + (kt + 1) * BKT, ra);
        load_slab<MB, BKT>(g.b, Bb, g.N, kend, n0, kbeg + (kt + 1) * BKT, rb);
      }
      float af[2][KH], bf[2][KH];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        load_frag<MA, BKT>(As[0], wm * 64 + t * 32 + l32, h, af[t]);
        load_frag<MB, BKT>(Bs[0], wn * 64 + t * 32 + l32, h, bf[t]);
      }
      __builtin_amdgcn_sched_barrier(0);
      mfma_slab<KH>(acc, af, bf);
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) {
      load_slab<MA, BKT>(g.a, Ab, g.M, kend, m0, kbeg + kt * BKT, ra);
      load_slab<MB, BKT>(g.b, Bb, g.N, kend, n0, kbeg + kt * BKT, rb);
      if (kt > 0) __syncthreads();  // everyone finished reading the previous slab
      store_slab<MA, BKT>(As[0], ra);
      store_slab<MB, BKT>(Bs[0], rb);
      __syncthreads();
      if constexpr (VARIANT == 3) {
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
          float af[2][8], bf[2][8];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            load_frag_half<MA>(As[0], wm * 64 + t * 32 + l32, h, hs, af[t]);
            load_frag_half<MB>(Bs[0], wn * 64 + t * 32 + l32, h, hs, bf[t]);
          }
          mfma_slab<8>(acc, af, bf);
        }
      } else {
        float af[2][KH], bf[2][KH];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          load_frag<MA, BKT>(As[0], wm * 64 + t * 32 + l32, h, af[t]);
          load_frag<MB, BKT>(Bs[0], wn * 64 + t * 32 + l32, h, bf[t]);
        }
        // issue every LDS read of the slab before the first MFMA (one latency per slab
        // instead of one per MFMA group); the MFMA chain then runs back to back
        __builtin_amdgcn_sched_barrier(0);
        mfma_slab<KH>(acc, af, bf);
      }
    }
  }

// ---------------------------------------------------------------- epilogue
  float* W = g.splits > 1 ? g.work + ((long)split * g.batch + z) * (long)g.M * g.N : nullptr;  // [split][z][M][N]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + l32;
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m >= g.M) continue;
        if (W) W[(long)m * g.N + n] = acc[i][j][r];
        else epi_store(g, z, m, n, acc[i][j][r]);
      }
    }
}

// split-K reduction in fixed split order + the fused epilogue (4 outputs per thread when
// N % 4 == 0: float4 partial loads)
__global__ void splitk_reduce_kernel(GemmArgs g) {
  const long MN = (long)g.M * g.N;
  const long split_stride = MN * g.batch;
  if ((g.N & 3) == 0) {
    const long total4 = split_stride >> 2;
    for (long e4 = blockIdx.x * (long)blockDim.x + threadIdx.x; e4 < total4; e4 += (long)gridDim.x * blockDim.x) {
      const long e = e4 << 2;
      float4 acc = *reinterpret_cast<const float4*>(g.work + e);
      for (int s = 1; s < g.splits; ++s) {
        const float4 v = *reinterpret_cast<const float4*>(g.work + s * split_stride + e);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      const int z = (int)(e / MN);
      const long r = e - (long)z * MN;
      const int m = (int)(r / g.N), n = (int)(r - (long)m * g.N);
      epi_store(g, z, m, n, acc.x);
      epi_store(g, z, m, n + 1, acc.y);
      epi_store(g, z, m, n + 2, acc.z);
      epi_store(g, z, m, n + 3, acc.w);
    }
    return;
  }
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < split_stride; e += (long)gridDim.x * blockDim.x) {
    const int z = (int)(e / MN);
    const long r = e - (long)z * MN;
    const int m = (int)(r / g.N), n = (int)(r - (long)m * g.N);
    float acc = 0.f;
    for (int s = 0; s < g.splits; ++s) acc += g.work[s * split_stride + e];
    epi_store(g, z, m, n, acc);
  }
}

int g_variant = -1;
int variant() {
  if (g_variant < 0) {
    const char* e = getenv("ESP_GEMM_VARIANT");
    g_variant = e ? atoi(e) : 1;
  }
  return g_variant;
}

template <int MA, int MB>
int launch(const GemmArgs& g, int batch, hipStream_t st) {
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, batch * g.splits);
  if (variant() == 0) hipLaunchKernelGGL((gemm_f32_kernel<MA, MB, 0>), grid, dim3(NT), 0, st, g);
  else if (variant() == 2) hipLaunchKernelGGL((gemm_f32_kernel<MA, MB, 2>), grid, dim3(NT), 0, st, g);
  else if (variant() == 3) hipLaunchKernelGGL((gemm_f32_kernel<MA, MB, 3>), grid, dim3(NT), 0, st, g);
  else hipLaunchKernelGGL((gemm_f32_kernel<MA, MB, 1>), grid, dim3(NT), 0, st, g);
  if (g.splits > 1) {
    long total = (long)g.M * g.N * batch;
    long nb = (total + 255) / 256;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)(nb > 16384 ? 16384 : nb)), dim3(256), 0, st, g);
  }
  ESP_CHECK_LAUNCH("gemm_f32");
  return 0;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

// C-ABI: see include/espnet_mi355.h for the contract.
ESP_API int esp_gemm_f32(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2,
                         const float* A, long lda, long sa1, long sa2,
                         const float* B, long ldb, long sb1, long sb2,
                         float* C, long ldc, long sc1, long sc2,
                         const float* bias, float alpha, float beta, const float* R,
                         int act, float* aux, float drop_p, unsigned long long seed,
                         const int* im2col_a, const int* im2col_b, float* work, long work_bytes,
                         void* stream) {
  ESP_ARG_CHECK(M >= 0 && N >= 0 && K >= 0 && batch >= 1 && nb2 >= 1 && batch % nb2 == 0,
                "esp_gemm_f32: bad sizes M=%d N=%d K=%d batch=%d nb2=%d", M, N, K, batch, nb2);
  ESP_ARG_CHECK(mode_a >= 0 && mode_a <= 3 && mode_b >= 0 && mode_b <= 3, "esp_gemm_f32: bad mode");
  ESP_ARG_CHECK(drop_p >= 0.f && drop_p < 1.f, "esp_gemm_f32: bad dropout p");
  if (M == 0 || N == 0) return 0;
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K; g.nb2 = nb2;
  g.a = Operand{A, lda, sa1, sa2, 0, {}};
  g.b = Operand{B, ldb, sb1, sb2, 0, {}};
  g.a.vec = aligned16(A) && lda % 4 == 0 && sa1 % 4 == 0 && sa2 % 4 == 0;
  g.b.vec = aligned16(B) && ldb % 4 == 0 && sb1 % 4 == 0 && sb2 % 4 == 0;
  if (mode_a >= 2) {
    ESP_ARG_CHECK(im2col_a && im2col_a[2] % 4 == 0 && aligned16(A), "esp_gemm_f32: im2col A needs C%%4==0");
    g.a.ic = Im2col{im2col_a[0], im2col_a[1], im2col_a[2], im2col_a[3], im2col_a[4]};
  }
  if (mode_b >= 2) {
    ESP_ARG_CHECK(im2col_b && im2col_b[2] % 4 == 0 && aligned16(B), "esp_gemm_f32: im2col B needs C%%4==0");
    g.b.ic = Im2col{im2col_b[0], im2col_b[1], im2col_b[2], im2col_b[3], im2col_b[4]};
  }
  g.c = C; g.ldc = ldc; g.c1 = sc1; g.c2 = sc2;
  g.r = R; g.aux = aux; g.bias = bias; g.alpha = alpha; g.beta = beta; g.act = act;
  g.seed = seed;
  if (drop_p > 0.f) {
    double t = (double)drop_p * 4294967296.0;
    g.drop_thresh = (uint32_t)(t >= 4294967295.0 ? 4294967295.0 : t);
    if (g.drop_thresh == 0) g.drop_thresh = 1;
    g.drop_scale = 1.0f / (1.0f - drop_p);
  }
  // split-K when the tile grid cannot fill the 256 CUs (weight gradients: small M x N, huge K)
  g.batch = batch;
  g.splits = 1;
  g.kchunk = K;
  {
    const long tiles = (long)((N + BN - 1) / BN) * ((M + BM - 1) / BM) * batch;
    // target two blocks per CU.  Measured (tools/gemm_bench.py, B=64 FFN w2 M=23936 N=256
    // K=1024): split 2 + reduce 153 us vs no split 191 us, although the reduce pass alone is
    // ~20% of the GEMM's GRBM_GUI_ACTIVE cycles
    const long target = 2 * 256;
    if (work && tiles < target && K >= 2 * 128) {
      long sp = (target + tiles - 1) / tiles;
      const long by_k = K / 128;  // keep >= 8 slabs of BK per split
      if (sp > by_k) sp = by_k;
      const long cap = work_bytes / (4L * M * N * batch);
      if (sp > cap) sp = cap;
      if (sp > 64) sp = 64;
      if (sp >= 2) {
        int chunk = (int)((K + sp - 1) / sp);
        chunk = (chunk + BK - 1) / BK * BK;
        g.splits = (int)((K + chunk - 1) / chunk);
        g.kchunk = chunk;
        g.work = work;
      }
    }
  }
  hipStream_t st = (hipStream_t)stream;
  const int key = mode_a * 4 + mode_b;
  switch (key) {
    case KC * 4 + KC: return launch<KC, KC>(g, batch, st);
    case KC * 4 + RC: return launch<KC, RC>(g, batch, st);
    case RC * 4 + KC: return launch<RC, KC>(g, batch, st);
    case RC * 4 + RC: return launch<RC, RC>(g, batch, st);
    case I2C_KC * 4 + KC: return launch<I2C_KC, KC>(g, batch, st);
    case RC * 4 + I2C_RC: return launch<RC, I2C_RC>(g, batch, st);
    default:
      esp::set_error("esp_gemm_f32: unsupported mode pair %d,%d", mode_a, mode_b);
      return -1;
  }
}
