#pragma once
// gemm_kernels.h: device code of the GEMM family (included by gemm.hip and the gemm_glds_*.hip
// instantiation units, which compile in parallel).
//
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

#include <algorithm>

#include <type_traits>

#include "common.h"

namespace espg {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;  // BK: split-K granularity
// split-K arrival tickets: the last ESP_GEMM_TICKET_BYTES of the GEMM workspace (zero-filled by
// the caller before first use; every launch leaves them zero), one int per output tile
#define ESP_GEMM_TICKET_BYTES 65536L
#define ESP_GEMM_TICKETS 16384L
// 1 (default): the fp32 GEMMs (PREC 0) of the LDS-DMA kernel run as bf16x6 split products on
// the bf16 MFMA (split3_bf16; measured as accurate as the f32 MFMA against fp64,
// profiles/r03h_f32_gemm_accuracy.txt); 0: v_mfma_f32_32x32x2_f32 (make VARIANT=_f32
// EXTRA=-DESP_F32_SPLIT=0 builds libespnet_mi355_f32.so for A/B runs)
#ifndef ESP_F32_SPLIT
#define ESP_F32_SPLIT 1
#endif
// 1 (default): the fp32 split-product GEMMs run the software-pipelined k-loop (gemm_glds_kernel PIPE);
// 0: the round-4 k-loop (an A/B build: make VARIANT=_np EXTRA=-DESP_GEMM_PIPE=0)
#ifndef ESP_GEMM_PIPE
#define ESP_GEMM_PIPE 1
#endif

enum Mode { KC = 0, RC = 1, I2C_KC = 2, I2C_RC = 3, I2CT_KC = 4 };
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SWISH = 2, ACT_MUL = 3 /* bwd_act only: v *= pre */ };
// act flag: aux receives the local derivative dh/dv of h = drop(act(v)) (0 where dropped)
// instead of the pre-activation v, so the backward epilogue is one multiply (bwd_act = ACT_MUL)
// instead of regenerating the dropout mask and re-evaluating act'.
constexpr int ACT_AUX_DERIV = 16;

// n / d for n < 2^31: (n * m) >> (31 + l), m = ceil(2^(31+l) / d), l = ceil(log2 d).  For d >= 2
// m < 2^32, so the quotient is umulhi(n, m) >> (l - 1): one v_mul_hi_u32 and a shift (the 64-bit
// product compiled to two v_mad_u64_u32 per division, in the implicit-im2col GEMMs' k-loops).
struct FastDiv {
  uint32_t m;   // d >= 2: ceil(2^(31+l) / d); d == 1: unused
  uint32_t sh;  // l - 1
  uint32_t d;
};
static FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  FastDiv f;
  f.d = d;
  f.sh = l ? l - 1 : 0;
  f.m = d >= 2 ? (uint32_t)(((1ull << (31 + l)) + d - 1) / d) : 0u;
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return f.d == 1 ? n : (__umulhi(n, f.m) >> f.sh);
}

struct Im2col {  // NHWC input map [Bn][H][W][C], 3x3 kernel, stride 2, no padding
  int H, W, C, Ho, Wo;
};

struct Operand {
  const float* p;
  long ld;
  long s1, s2;
  int vec;   // float4 along the contiguous dim is legal
  Im2col ic;
  int glds;  // 16-B LDS-DMA of any in-range quad stays inside the operand (see glds_ok)
  long ps = 0;  // PREC 3 B operand: plane stride in bf16 elements (p, ld, s1, s2 in bf16 elements)
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
  const uint64_t* key;  // device dropout key (esp_set_rng_key) or NULL
  int batch;
  int splits, kchunk;  // split-K: blockIdx.z = z*splits + split; partials -> work
  float* work;
  int bf16;  // MFMA precision: 0 fp32; 1 bf16 MFMA on fp32 operands rounded after staging
             // (esp_set_gemm_compute(1)); 2 bf16 operands in HBM (esp_gemm_bf16: K, ld, strides
             // given in fp32 units, i.e. bf16 pairs; KC x KC only); 3 fp32 with B given as its
             // three bf16 split planes (esp_gemm_f32_bp: B's ld, strides, ps in bf16 elements)
  int bnt;  // LDS-DMA kernel tile width (128, or 64 for narrow / mid-size grids); 0 = fallback kernel
  int bm;   // LDS-DMA kernel tile height: 128, or 64 (with bnt 64) for under-filled grids
  int bwd_act;       // != 0: backward epilogue  v = drop'(acc) * act'(pre)  (act code, dropout regenerated)
  const float* pre;  // pre-activation (same layout as C) for bwd_act
  float* rowsum;     // != NULL: rowsum[m] += sum_k A(m,k)  (bias gradient of a weight-gradient GEMM)
  float* rs_work;    // split-K partial row sums [split][M]
  // in-kernel split-K combine (LDS-DMA kernel): partials W[split][z][Mp][Np] on whole tiles
  // (Mp, Np: the tile grid's padded extent), one arrival ticket per output tile; the unit that
  // arrives last sums the splits in fixed order and runs the epilogue (no reduction launch)
  int* tickets;      // NULL: the separate splitk_reduce kernel (layout [split][z][M][N])
  int sk_mp, sk_np;
  int wide;          // float4 epilogue legal (N, ldc, batch strides % 4 == 0, 16-B aligned C/R/aux/pre/bias/work)
  int ragged4;       // the same except N % 4 != 0 (ldc % 4 == 0 pads every row to whole quads): the
                     // plain specialised kinds store the last quad of a row element by element
  // output row map (conv2 input gradient, one parity class (ph, pw) of the conv1 output grid):
  // row m = (b, a, e) of the class grid (Ha x We) -> pixel (b, 2a+ph, 2e+pw) of the T1 x F1 map
  int cmap;
  FastDiv cm_hw, cm_w;
  int cm_T1, cm_F1, cm_ph, cm_pw;
  // EPI_RMASKMAP's ReLU mask as the conv1 map's packed bit map (esp_conv1_fwd_bits: bit c % 32 of word
  // pixel * cm_bw + c / 32 = (z1[pixel][c] > 0)) instead of the fp32 map in pre; NULL: pre
  const uint32_t* cm_bits;
  int cm_bw;
  // EPI_C1FOLD: the masked input gradient of the conv1 map is not stored; its conv1 weight / bias gradient
  // partials (x = the conv1 input, T x F per utterance) accumulate per wave in registers across the block's
  // tiles and land in c1_part, [grid][tn C1NT][wave 4][lane 64][10] (c1fold_reduce / c1fold_finalize)
  const float* c1_x;
  int c1_T, c1_F;
  float* c1_part;
  // EPI_SMB (esp_attn_dscores): the dP = dctx V^T GEMM of rel-pos attention finishes the softmax
  // and rel_shift adjoints in its epilogue; pre = the attention probabilities (C's layout)
  int smb_rel;           // 0 off, 1 latest, 2 legacy rel_shift adjoint
  const float* smb_dot;  // [batch * M] row dots  sum_j P_drop[i][j] dP[i][j] = dctx_i . ctx_i
  float* smb_dbd;        // bd gradient rows (batch*M rows of pitch smb_ldp)
  long smb_ldp;
  // planes output (the *_PL kinds): c points at plane 0 (bf16), ldc / c1 / c2 in bf16 elements, plane p
  // at c + p * cps; cpn = 3 (exact split) or 1 (bf16)
  int cpn;
  long cps;
  // banded A (KC; esp_relpos_dqv): row m of A is zero outside columns [band_c0 - m, band_c0 - m + band_w),
  // so a row tile's k-loop runs only over its rows' union (LDS-DMA kernel; band_w = 0: the whole K)
  int band_c0, band_w;
};

// the class-grid row m as (utterance b, conv1-map row t1, column f1)
__device__ __forceinline__ void row_btf(const GemmArgs& g, int m, int& b, int& t1, int& f1) {
  b = (int)fdiv((uint32_t)m, g.cm_hw);
  const int rem = m - b * (int)g.cm_hw.d;
  const int a = (int)fdiv((uint32_t)rem, g.cm_w), e = rem - a * (int)g.cm_w.d;
  t1 = 2 * a + g.cm_ph;
  f1 = 2 * e + g.cm_pw;
}
__device__ __forceinline__ long row_pix(const GemmArgs& g, int m) {
  const int b = (int)fdiv((uint32_t)m, g.cm_hw);
  const int rem = m - b * (int)g.cm_hw.d;
  const int a = (int)fdiv((uint32_t)rem, g.cm_w), e = rem - a * (int)g.cm_w.d;
  return ((long)b * g.cm_T1 + 2 * a + g.cm_ph) * g.cm_F1 + 2 * e + g.cm_pw;
}
__device__ __forceinline__ long row_off(const GemmArgs& g, int m) {
  if (!g.cmap) return (long)m * g.ldc;
  return row_pix(g, m) * g.ldc;
}

// Fused epilogue for output element (m, n) of batch z with raw accumulator `acc`.  The kind is
// chosen once per launch (a template argument), so the per-element path is straight-line:
//   EPI 0: alpha*acc (+ beta*R)
//   EPI 1: forward  alpha*drop(act(acc + bias)) (+ beta*R), pre-activation to aux
//   EPI 2: backward  drop'(acc + bias) * act'(pre)  (dropout mask regenerated), alpha, R
// cbase = offset of batch z in C/R/aux/pre, dbase = z*M*N (dropout index base).
enum { EPI_PLAIN = 0, EPI_FWD = 1, EPI_BWD = 2, EPI_BIAS = 3, EPI_BDR = 4, EPI_FFN_SWISH = 5, EPI_FFN_RELU = 6,
       EPI_BMUL = 7, EPI_P0 = 8, EPI_PR = 9, EPI_SMB = 10, EPI_BRELU = 11, EPI_RMASK = 12, EPI_RMASKMAP = 13,
       // the same kinds with C written as bf16 planes (GemmArgs cpn): the FFN hidden state, the attention context
       EPI_FFN_SWISH_PL = 14, EPI_FFN_RELU_PL = 15, EPI_P0_PL = 16,
       // ... and the FFN's input gradient through the stored derivative (its only readers: w_1's GEMMs)
       EPI_BMUL_PL = 17,
       // ... and the gradient through a ReLU output (the subsampling's dz2: its readers are conv2's GEMMs)
       EPI_RMASK_PL = 18,
       // EPI_RMASKMAP (bit-map mask) that writes no C: the conv1 weight gradient folded in (store_c1fold)
       EPI_C1FOLD = 19 };
// the fp32-output kind a planes-output kind computes
constexpr int epi_base(int e) {
  return e == EPI_FFN_SWISH_PL ? EPI_FFN_SWISH
         : e == EPI_FFN_RELU_PL ? EPI_FFN_RELU
         : e == EPI_P0_PL      ? EPI_P0
         : e == EPI_BMUL_PL    ? EPI_BMUL
         : e == EPI_RMASK_PL   ? EPI_RMASK
                               : e;
}
__host__ __device__ inline int epi_kind(const GemmArgs& g) {
  return g.bwd_act ? EPI_BWD : ((g.bias || g.aux || g.act || g.drop_thresh) ? EPI_FWD : EPI_PLAIN);
}
// the specialised kind (store_spec) when the launch's features match one exactly, else the
// generic kind; only for wide (float4) epilogues (the conv2 output row map: EPI_RMASKMAP only)
__host__ inline int epi_kind_spec(const GemmArgs& g) {
  if (g.smb_rel) return EPI_SMB;
  const int k = epi_kind(g);
  if (g.cpn) {  // planes output: the kinds that have a planes form, else none (-1)
    if (g.splits > 1 || g.rowsum || g.r) return -1;
    if (k == EPI_PLAIN) return EPI_P0_PL;
    // (dropout p = 0 included: every element is kept, the scale is 1)
    if (g.bias && g.aux && !g.bwd_act && g.act == (ACT_SWISH | ACT_AUX_DERIV)) return EPI_FFN_SWISH_PL;
    if (g.bias && g.aux && !g.bwd_act && g.act == (ACT_RELU | ACT_AUX_DERIV)) return EPI_FFN_RELU_PL;
    if (k == EPI_BWD && g.bwd_act == ACT_MUL && !g.drop_thresh && !g.bias && g.alpha == 1.0f) return EPI_BMUL_PL;
    if (k == EPI_BWD && g.bwd_act == ACT_RELU && !g.drop_thresh && !g.bias && g.alpha == 1.0f) return EPI_RMASK_PL;
    return -1;
  }
  if (g.cmap)
    return (g.wide && k == EPI_BWD && g.bwd_act == ACT_RELU && !g.drop_thresh && !g.r && !g.bias && g.alpha == 1.0f &&
            g.splits == 1)
               ? (g.c1_part && g.cm_bits ? EPI_C1FOLD : EPI_RMASKMAP)
               : k;
  if (!g.wide) {
    if (g.ragged4 && k == EPI_PLAIN && g.splits == 1 && !g.rowsum) return g.r ? EPI_PR : EPI_P0;
    return k;
  }
  if (k == EPI_PLAIN) return (g.splits > 1 || g.rowsum) ? k : (g.r ? EPI_PR : EPI_P0);
  if (k == EPI_BWD) {
    if (g.drop_thresh || g.r || g.bias || g.alpha != 1.0f) return k;
    return g.bwd_act == ACT_MUL ? EPI_BMUL : g.bwd_act == ACT_RELU ? EPI_RMASK : k;
  }
  if (g.bias && !g.aux && !g.act && !g.drop_thresh && !g.r) return EPI_BIAS;
  if (g.bias && !g.aux && g.act == ACT_RELU && !g.drop_thresh && !g.r && g.alpha == 1.0f) return EPI_BRELU;
  if (g.bias && !g.aux && !g.act && g.drop_thresh && g.r) return EPI_BDR;
  if (g.bias && g.aux && g.drop_thresh && !g.r && g.act == (ACT_SWISH | ACT_AUX_DERIV)) return EPI_FFN_SWISH;
  if (g.bias && g.aux && g.drop_thresh && !g.r && g.act == (ACT_RELU | ACT_AUX_DERIV)) return EPI_FFN_RELU;
  return k;
}
// h = drop(act(v)) for one element (dropout index idx); with ACT_AUX_DERIV in g.act also
// d = dh/dv = keep * scale * act'(v)  (0 where dropped).  Swish: v / (1 + e^-v), act' =
// s (1 + v (1 - s)) with s = sigmoid(v).
__device__ __forceinline__ float fwd_elem(const GemmArgs& g, uint64_t seed, uint64_t idx, float v, float& d) {
  const int a = g.act & 3;
  const bool deriv = g.act & ACT_AUX_DERIV;
  float w = v;
  d = 1.f;
  if (a == ACT_RELU) {
    w = fmaxf(v, 0.f);
    if (deriv) d = v > 0.f ? 1.f : 0.f;
  } else if (a == ACT_SWISH) {
    const float sg = esp::fast_sigmoid(v);
    w = v * sg;
    if (deriv) d = sg * (1.0f + v * (1.0f - sg));
  }
  if (g.drop_thresh) {
    const bool keep = esp::keep_elem(seed, idx, g.drop_thresh);
    w = keep ? w * g.drop_scale : 0.f;
    d = keep ? d * g.drop_scale : 0.f;
  }
  return w;
}
template <int EPI>
__device__ __forceinline__ void epi_store(const GemmArgs& g, long cbase, uint64_t dbase, int m, int n, float acc) {
  const long off = cbase + row_off(g, m) + n;
  const uint64_t seed = g.drop_thresh ? esp::keyed(g.seed, g.key) : 0;
  float v = acc;
  if constexpr (EPI == EPI_FWD) {
    if (g.bias) v += g.bias[n];
    float d;
    const float x = v;
    v = fwd_elem(g, seed, dbase + (uint64_t)m * (uint64_t)g.N + n, x, d);
    if (g.aux) g.aux[off] = (g.act & ACT_AUX_DERIV) ? d : x;
  } else if constexpr (EPI == EPI_BWD) {
    // gradient w.r.t. the pre-activation of  h = drop(act(pre))  given dL/dh = v
    if (g.bias) v += g.bias[n];
    if (g.drop_thresh) {
      const uint64_t idx = dbase + (uint64_t)m * (uint64_t)g.N + n;
      v = esp::keep_elem(seed, idx, g.drop_thresh) ? v * g.drop_scale : 0.f;
    }
    const float x = g.pre[off];
    if (g.bwd_act == ACT_MUL) v *= x;
    else if (g.bwd_act == ACT_RELU) v = x > 0.f ? v : 0.f;
    else {
      const float sg = esp::fast_sigmoid(x);
      v = v * (sg * (1.0f + x * (1.0f - sg)));
    }
  }
  v *= g.alpha;
  if (g.r) v += g.beta * g.r[off];
  g.c[off] = v;
}
__device__ __forceinline__ long c_base(const GemmArgs& g, int z) {
  const int z1 = z / g.nb2, z2 = z - z1 * g.nb2;
  return (long)z1 * g.c1 + (long)z2 * g.c2;
}

// store a wave's TM x TN 32x32 accumulator tiles (rows mrow0 + 32i + ..., cols ncol0 + 32j + l32).
// Per 32x32 tile, every load the epilogue needs (residual R, pre-activation) is issued, in
// program order, before the tile's first store: R / pre may alias C, so a load placed after a
// store cannot be hoisted by the compiler and each element would pay a memory round trip.
template <int EPI, int TM, int TN>
__device__ __forceinline__ void store_tiles(const GemmArgs& g, int z, int mrow0, int ncol0, int h, int l32,
                                            const f32x16 (&acc)[TM][TN]) {
  const long cbase = c_base(g, z);
  const uint64_t dbase = (uint64_t)z * (uint64_t)g.M * (uint64_t)g.N;
  const bool has_r = g.r != nullptr;
  const uint64_t seed = (EPI != EPI_PLAIN && g.drop_thresh) ? esp::keyed(g.seed, g.key) : 0;  // before any store
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = ncol0 + j * 32 + l32;
    if (n >= g.N) continue;
    const float bn = (EPI != EPI_PLAIN && g.bias) ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float rr[16], pp[EPI == EPI_BWD ? 16 : 1];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mrow0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const long off = cbase + row_off(g, m) + n;
        rr[r] = (has_r && m < g.M) ? g.r[off] : 0.f;
        if constexpr (EPI == EPI_BWD) pp[r] = m < g.M ? g.pre[off] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mrow0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m >= g.M) continue;
        const long off = cbase + row_off(g, m) + n;
        float v = acc[i][j][r] + bn;
        if constexpr (EPI == EPI_FWD) {
          float d;
          const float x = v;
          v = fwd_elem(g, seed, dbase + (uint64_t)m * (uint64_t)g.N + n, x, d);
          if (g.aux) g.aux[off] = (g.act & ACT_AUX_DERIV) ? d : x;
        } else if constexpr (EPI == EPI_BWD) {
          if (g.drop_thresh) {
            const uint64_t idx = dbase + (uint64_t)m * (uint64_t)g.N + n;
            v = esp::keep_elem(seed, idx, g.drop_thresh) ? v * g.drop_scale : 0.f;
          }
          const float x = pp[r];
          if (g.bwd_act == ACT_MUL) v *= x;
          else if (g.bwd_act == ACT_RELU) v = x > 0.f ? v : 0.f;
          else {
            const float sg = esp::fast_sigmoid(x);
            v = v * (sg * (1.0f + x * (1.0f - sg)));
          }
        }
        v *= g.alpha;
        if (has_r) v += g.beta * rr[r];
        g.c[off] = v;
      }
    }
  }
}
// ---------------------------------------------------------------- widened epilogue
// A 32x32 f32 MFMA accumulator holds one COLUMN per lane (16 rows), so a direct store is 16
// dword stores per tile.  Two DPP butterfly stages transpose 4x4 blocks inside each lane quad:
// afterwards lane (h, l32 = 4q + j) holds in registers 4g..4g+3 the row 8g + 4h + j, columns
// 4q..4q+3 — one float4 per group, 4 dwordx4 stores per tile (the store tail is issue-bound:
// 4x fewer instructions for the same bytes).  Residual / pre-activation loads widen alike.
__device__ __forceinline__ float dpp_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
}
__device__ __forceinline__ float dpp_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));  // quad_perm 2,3,0,1
}
__device__ __forceinline__ void quad_transpose(f32x16& v, int lane) {
  const bool odd = lane & 1, hi = lane & 2;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float a0 = v[4 * g], a1 = v[4 * g + 1], a2 = v[4 * g + 2], a3 = v[4 * g + 3];
    // stage 1: reg k of lane j takes reg k^1 of lane j^1 where the parities of j and k differ
    const float s0 = dpp_xor1(a1), s1 = dpp_xor1(a0), s2 = dpp_xor1(a3), s3 = dpp_xor1(a2);
    const float b0 = odd ? s0 : a0, b1 = odd ? a1 : s1, b2 = odd ? s2 : a2, b3 = odd ? a3 : s3;
    // stage 2: the same with bit 1
    const float t0 = dpp_xor2(b2), t1 = dpp_xor2(b3), t2 = dpp_xor2(b0), t3 = dpp_xor2(b1);
    v[4 * g] = hi ? t0 : b0;
    v[4 * g + 1] = hi ? t1 : b1;
    v[4 * g + 2] = hi ? b2 : t2;
    v[4 * g + 3] = hi ? b3 : t3;
  }
}

// 16-B output store; nt = streaming (non-temporal) hint, so the write does not displace the
// operand panels the co-resident tiles still read from L2 (ESP_GEMM_ABL bit 32, measured)
typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st4(float* p, const float (&v)[4], bool nt) {
  const f32x4v w = {v[0], v[1], v[2], v[3]};
  if (nt) __builtin_nontemporal_store(w, reinterpret_cast<f32x4v*>(p));
  else *reinterpret_cast<f32x4v*>(p) = w;
}
// needs N % 4 == 0, ldc % 4 == 0 and 16-B aligned C / R / aux / pre / bias (host: g.wide).
// Generic (runtime feature flags) form; the production call sites use store_spec below.
template <int EPI, int TM, int TN>
__device__ __forceinline__ void store_tiles_wide(const GemmArgs& g, int z, int mrow0, int ncol0, int lane,
                                                 f32x16 (&acc)[TM][TN], bool nt = false) {
  const int h = lane >> 5, l32 = lane & 31;
  const long cbase = c_base(g, z);
  const uint64_t dbase = (uint64_t)z * (uint64_t)g.M * (uint64_t)g.N;
  const bool has_r = g.r != nullptr;
  const uint64_t seed = (EPI != EPI_PLAIN && g.drop_thresh) ? esp::keyed(g.seed, g.key) : 0;  // before any store
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = ncol0 + j * 32 + 4 * (l32 >> 2);
    const bool nok = n < g.N;
    float4 bn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (EPI != EPI_PLAIN && g.bias && nok) bn = *reinterpret_cast<const float4*>(g.bias + n);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      quad_transpose(acc[i][j], lane);
      float4 rr[4], pp[EPI == EPI_BWD ? 4 : 1];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = mrow0 + i * 32 + 8 * q + 4 * h + (l32 & 3);
        const long off = cbase + row_off(g, m) + n;
        const bool ok = nok && m < g.M;
        rr[q] = (has_r && ok) ? *reinterpret_cast<const float4*>(g.r + off) : make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (EPI == EPI_BWD)
          pp[q] = ok ? *reinterpret_cast<const float4*>(g.pre + off) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = mrow0 + i * 32 + 8 * q + 4 * h + (l32 & 3);
        if (!nok || m >= g.M) continue;
        const long off = cbase + row_off(g, m) + n;
        float v[4] = {acc[i][j][4 * q] + bn.x, acc[i][j][4 * q + 1] + bn.y, acc[i][j][4 * q + 2] + bn.z,
                      acc[i][j][4 * q + 3] + bn.w};
        const float r4[4] = {rr[q].x, rr[q].y, rr[q].z, rr[q].w};
        if constexpr (EPI == EPI_FWD) {
          if (g.aux && !(g.act & ACT_AUX_DERIV)) st4(g.aux + off, v, nt);
        }
        float dv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float w = v[e];
          if constexpr (EPI == EPI_FWD) {
            w = fwd_elem(g, seed, dbase + (uint64_t)m * (uint64_t)g.N + n + e, w, dv[e]);
          } else if constexpr (EPI == EPI_BWD) {
            if (g.drop_thresh) {
              const uint64_t idx = dbase + (uint64_t)m * (uint64_t)g.N + n + e;
              w = esp::keep_elem(seed, idx, g.drop_thresh) ? w * g.drop_scale : 0.f;
            }
            const float xp = e == 0 ? pp[q].x : e == 1 ? pp[q].y : e == 2 ? pp[q].z : pp[q].w;
            if (g.bwd_act == ACT_MUL) w *= xp;
            else if (g.bwd_act == ACT_RELU) w = xp > 0.f ? w : 0.f;
            else {
              const float sg = esp::fast_sigmoid(xp);
              w = w * (sg * (1.0f + xp * (1.0f - sg)));
            }
          }
          w *= g.alpha;
          if (has_r) w += g.beta * r4[e];
          v[e] = w;
        }
        if constexpr (EPI == EPI_FWD) {
          if (g.aux && (g.act & ACT_AUX_DERIV)) st4(g.aux + off, dv, nt);
        }
        st4(g.c + off, v, nt);
      }
    }
  }
}

// ---------------------------------------------------------------- specialised epilogues
// The generic epilogues test every feature (bias, activation, dropout, aux, residual, row map,
// bounds) per element at run time: hundreds of branches per tile and VGPR pressure that spills.
// The production call sites use fixed feature sets, compiled in:
//   EPI_BIAS       acc + bias                                    (q/k/v, pointwise_conv1, ...)
//   EPI_BRELU      relu(acc + bias)                              (conv2: Conv2d + ReLU, implicit im2col A)
//   EPI_BDR        alpha * drop(acc + bias) + beta * R           (linear_out, FFN w_2, pointwise_conv2)
//   EPI_FFN_SWISH  h = drop(swish(acc + bias)), aux = dh/dv      (FFN w_1, ACT_AUX_DERIV)
//   EPI_FFN_RELU   the same with ReLU                            (decoder FFN w_1)
//   EPI_BMUL       acc * pre                                     (FFN w_2 input gradient, ACT_MUL)
//   EPI_RMASK      pre > 0 ? acc : 0                             (input gradient through a ReLU output)
//   EPI_RMASKMAP   EPI_RMASK through the conv2 output row map    (implicit conv2 input gradient classes)
//   EPI_P0         alpha * acc                                   (plain, unsplit)
//   EPI_PR         alpha * acc + beta * R                        (gradient accumulation)
//   EPI_SMB        dS = P * (drop'(acc) - dot_row) * alpha -> C, and its rel_shift adjoint -> dbd
//                  (attention.py:64-96 + 145-165 backward; P in pre, FlashAttention-2's row dot)
// (wide stores, no output row map but EPI_RMASKMAP's; chosen by epi_kind on the host).  A wave whose 32-row /
// 32-column sub-tiles are all in range takes a path without per-element bounds checks.
template <int EPI_>
struct EpiSpec {
  static constexpr bool pl = EPI_ != epi_base(EPI_);  // C written as bf16 planes
  static constexpr int EPI = epi_base(EPI_);
  static constexpr int act =
      EPI == EPI_FFN_SWISH ? ACT_SWISH : (EPI == EPI_FFN_RELU || EPI == EPI_BRELU) ? ACT_RELU : ACT_NONE;
  static constexpr bool bias = EPI == EPI_BIAS || EPI == EPI_BDR || act != ACT_NONE;
  static constexpr bool res = EPI == EPI_BDR || EPI == EPI_PR;
  static constexpr bool drop = EPI == EPI_BDR || EPI == EPI_FFN_SWISH || EPI == EPI_FFN_RELU;
  static constexpr bool aux = EPI == EPI_FFN_SWISH || EPI == EPI_FFN_RELU;  // derivative stream
  static constexpr bool mul = EPI == EPI_BMUL || EPI == EPI_RMASK || EPI == EPI_RMASKMAP;
  static constexpr bool rmap = EPI == EPI_RMASKMAP;
};
template <int EPI, int TM, int TN, bool FULL, bool A1 = false>  // A1: alpha == 1 (no scaling multiply)
__device__ __forceinline__ void store_spec(const GemmArgs& g, int z, int mrow0, int ncol0, int lane,
                                           f32x16 (&acc)[TM][TN]) {
  using S = EpiSpec<EPI>;
  const int h = lane >> 5, l32 = lane & 31;
  const long cbase = c_base(g, z);
  const uint64_t dbase = (uint64_t)z * (uint64_t)g.M * (uint64_t)g.N;
  const uint64_t seed = S::drop ? esp::keyed(g.seed, g.key) : 0;  // before any store
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = ncol0 + j * 32 + 4 * (l32 >> 2);
    const bool nok = FULL || n < g.N;
    const float4 bn = (S::bias && nok) ? *reinterpret_cast<const float4*>(g.bias + n) : zero4;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      quad_transpose(acc[i][j], lane);
      if constexpr (EPI == EPI_SMB) {
        // lane: rows m (q = 0..3) x columns n..n+3; M = N = T (one (head, utterance) per z)
        const int T = g.M;
        const uint64_t kseed = esp::keyed(g.seed, g.key);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = mrow0 + i * 32 + 8 * q + 4 * h + (l32 & 3);
          if (!nok || m >= g.M) continue;
          const long off = cbase + (long)m * g.ldc + n;
          const float4 pa = *reinterpret_cast<const float4*>(g.pre + off);  // rows padded to whole quads
          const float pr[4] = {pa.x, pa.y, pa.z, pa.w};
          const long zr = (long)z * T + m;
          const float dot = g.smb_dot[zr];
          const uint64_t row = dbase + (uint64_t)m * (uint64_t)g.N + n;
          float* db = g.smb_dbd + zr * g.smb_ldp;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float gv = acc[i][j][4 * q + e];
            if (g.drop_thresh) gv = esp::keep_elem(kseed, row + e, g.drop_thresh) ? gv * g.drop_scale : 0.f;
            v[e] = pr[e] * (gv - dot) * g.alpha;
          }
          if (n + 4 <= g.N) {
            st4(g.c + off, v, false);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < g.N) g.c[off + e] = v[e];
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int jj = n + e;
            if (jj >= g.N) continue;
            if (g.smb_rel == 1 || jj <= m) db[jj + T - 1 - m] = v[e];
            else if (jj >= m + 2) db[g.smb_ldp + jj - m - 2] = v[e];  // legacy: row m+1's lower part
          }
        }
        continue;
      }
      float4 x4[4];  // residual (BDR) or local derivative (BMUL)
      long roff[4];  // row offsets (EPI_RMASKMAP: through the class -> pixel row map)
      long pix[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = mrow0 + i * 32 + 8 * q + 4 * h + (l32 & 3);
        pix[q] = S::rmap ? row_pix(g, min(m, g.M - 1)) : 0;
        roff[q] = S::rmap ? pix[q] * g.ldc : (long)m * g.ldc;
      }
      if (S::rmap && g.cm_bits) {
        // the mask from the packed bit map: one word per 32 channels, the same word for the 8 lanes
        // of a row (columns n .. n+3 of one 32-column sub-tile): 1/32 of the fp32 map's bytes
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = mrow0 + i * 32 + 8 * q + 4 * h + (l32 & 3);
          const uint32_t w = (FULL || (nok && m < g.M)) ? g.cm_bits[pix[q] * g.cm_bw + (n >> 5)] >> (n & 31) : 0u;
          x4[q] = make_float4((float)(w & 1u), (float)((w >> 1) & 1u), (float)((w >> 2) & 1u), (float)((w >> 3) & 1u));
        }
      } else if constexpr (S::res || S::mul) {
        const float* src = S::res ? g.r : g.pre;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = mrow0 + i * 32 + 8 * q + 4 * h + (l32 & 3);
          x4[q] = (FULL || (nok && m < g.M)) ? *reinterpret_cast<const float4*>(src + cbase + roff[q] + n) : zero4;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = mrow0 + i * 32 + 8 * q + 4 * h + (l32 & 3);
        if (!FULL && (!nok || m >= g.M)) continue;
        const long off = cbase + roff[q] + n;
        const float xs[4] = {x4[q].x, x4[q].y, x4[q].z, x4[q].w};
        const float bs[4] = {bn.x, bn.y, bn.z, bn.w};
        float v[4], d[4];
        const uint64_t row = dbase + (uint64_t)m * (uint64_t)g.N + n;  // a multiple of 4 (N % 4 == 0)
        bool kp[4] = {true, true, true, true};
        if constexpr (S::drop) {
          esp::keep_pair(seed, row, g.drop_thresh, kp[0], kp[1]);
          esp::keep_pair(seed, row + 2, g.drop_thresh, kp[2], kp[3]);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float w = S::bias ? acc[i][j][4 * q + e] + bs[e] : acc[i][j][4 * q + e];  // (x + 0.f is not foldable)
          float dd = 1.f;
          if constexpr (S::act == ACT_RELU) {
            dd = w > 0.f ? 1.f : 0.f;
            w = fmaxf(w, 0.f);
          } else if constexpr (S::act == ACT_SWISH) {
            const float sg = esp::fast_sigmoid(w);
            dd = sg * (1.0f + w * (1.0f - sg));
            w = w * sg;
          }
          if constexpr (S::drop) {
            w = kp[e] ? w * g.drop_scale : 0.f;
            dd = kp[e] ? dd * g.drop_scale : 0.f;
          }
          if constexpr (S::EPI == EPI_RMASK || S::EPI == EPI_RMASKMAP) w = xs[e] > 0.f ? w : 0.f;
          else if constexpr (S::mul) w *= xs[e];
          if constexpr (!A1) w *= g.alpha;
          if constexpr (S::res) w += g.beta * xs[e];
          v[e] = w;
          d[e] = dd;
        }
        if constexpr (S::aux) st4(g.aux + off, d, false);
        if constexpr (S::pl) {  // N % 4 == 0 (host): whole quads; aux shares the offsets (ld = planes ld)
          esp::store_planes4(reinterpret_cast<uint16_t*>(g.c), off, g.cps, g.cpn, v[0], v[1], v[2], v[3]);
        } else if (FULL || n + 4 <= g.N) {
          st4(g.c + off, v, false);
        } else {  // last quad of a row with N % 4 != 0 (EPI_P0 / EPI_PR only): loads stayed inside ldc
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < g.N) g.c[off + e] = v[e];
        }
      }
    }
  }
}
// Column epilogue: stores (and residual / pre-activation loads) straight in the accumulator
// layout (lane = one column, 16 rows per 32x32 tile), no transpose.  Every access is a
// buffer_load/store_dword with a wave-uniform row offset in soffset and a per-lane column offset
// in voffset, so a full tile's epilogue issues no VALU besides its arithmetic: the float4 path pays
// 4 DPP / select VALU per element for the transpose, and f32 MFMAs do not hide VALU.
// Rows m = mrow0 + 32i + 8g + 4h + jj (4h in voffset), columns 32j in the instruction offset.
// Kinds without dropout (dropout keeps the float4 path and its one hash per element pair).
// Host: the tile's rows span < 2^31 bytes (ldc < 2^24).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff, 0x00020000);
}
template <int EPI>
constexpr bool col_epi_ok() {
  return EPI == EPI_P0 || EPI == EPI_PR || EPI == EPI_BIAS || EPI == EPI_BRELU || EPI == EPI_RMASK || EPI == EPI_BMUL;
}
// AUX: buffer cache policy of the stores (16 = sc1: write-through, for the split-K hand-off)
template <int EPI, int TM, int TN, bool A1, int AUX = 0>
__device__ __forceinline__ void store_cols(const GemmArgs& g, long cbase, long ldc, int mrow0, int ncol0, int lane,
                                           const f32x16 (&acc)[TM][TN], float* cptr) {
  using S = EpiSpec<EPI>;
  const int h = lane >> 5, l32 = lane & 31;
  const long tile0 = cbase + (long)mrow0 * ldc + ncol0;
  const __amdgpu_buffer_rsrc_t cr = buf_rsrc(cptr + tile0);
  __amdgpu_buffer_rsrc_t xr = cr;
  if constexpr (S::res) xr = buf_rsrc(g.r + tile0);
  if constexpr (S::mul) xr = buf_rsrc(g.pre + tile0);
  const int voff = (int)((4 * h * ldc + l32) * 4);
  float bn[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bn[j] = S::bias ? g.bias[ncol0 + 32 * j + l32] : 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float xs[16];
      if constexpr (S::res || S::mul) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          xs[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                   xr, voff + 128 * j, (int)((i * 32 + 8 * (r >> 2) + (r & 3)) * ldc * 4), 0));
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float w = S::bias ? acc[i][j][r] + bn[j] : acc[i][j][r];
        if constexpr (S::act == ACT_RELU) w = fmaxf(w, 0.f);
        if constexpr (EPI == EPI_RMASK) w = xs[r] > 0.f ? w : 0.f;
        else if constexpr (S::mul) w *= xs[r];
        if constexpr (!A1) w *= g.alpha;
        if constexpr (S::res) w += g.beta * xs[r];
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, w), cr, voff + 128 * j,
                                              (int)((i * 32 + 8 * (r >> 2) + (r & 3)) * ldc * 4), AUX);
      }
    }
}

// the generic per-element epilogue of a split-K combine (kind chosen at run time: the combine
// runs once per output tile)
__device__ __forceinline__ void reduce_store(const GemmArgs& g, int z, int m, int n, float acc) {
  const long cb = c_base(g, z);
  const uint64_t db = (uint64_t)z * (uint64_t)g.M * (uint64_t)g.N;
  switch (epi_kind(g)) {
    case EPI_BWD: epi_store<EPI_BWD>(g, cb, db, m, n, acc); break;
    case EPI_FWD: epi_store<EPI_FWD>(g, cb, db, m, n, acc); break;
    default: epi_store<EPI_PLAIN>(g, cb, db, m, n, acc);
  }
}

// In-kernel split-K combine, run by every unit after it stored its partial tile write-through
// (sc1) and drained (s_waitcnt vmcnt(0)): one agent-scope ticket add per unit; the unit whose add
// returns splits - 1 re-reads the tile's partials with sc1 loads, in split order 0..splits-1
// (deterministic whoever arrives last), applies the epilogue and re-arms the ticket to 0.
// Hand-off form: MI355X_MICROARCH.md "Valid forms" (write-through stores, drained per wave, a
// workgroup barrier, one lane's agent atomic add; the last adder's waves load after a barrier),
// plus an agent acquire, since 2-3 workgroups share a CU here.
template <int BMT, int BNT>
__device__ __forceinline__ void splitk_combine(const GemmArgs& g, int z, int tm, int tn, int ntx, int nty,
                                               int* flag_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through partials are done
  __builtin_amdgcn_s_barrier();
  const int tile = (z * nty + tm) * ntx + tn;
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(g.tickets + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag_lds = old == g.splits - 1;
  }
  __syncthreads();
  const bool last = *flag_lds != 0;
  __syncthreads();  // everyone read the flag before a later tile's combine rewrites it
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int m0 = tm * BMT, n0 = tn * BNT;
  const long plane = (long)g.sk_mp * g.sk_np;
  const long zoff = (long)z * plane + (long)m0 * g.sk_np + n0;
  const long sstride = plane * g.batch;
  constexpr int Q = BNT / 4;  // float4 slots per tile row
  for (int e = threadIdx.x; e < BMT * Q; e += NT) {
    const int r = e / Q, c = (e - r * Q) * 4;
    const int m = m0 + r, n = n0 + c;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    const long off = zoff + (long)r * g.sk_np + c;
    for (int sp = 0; sp < g.splits; ++sp) {
      const float4 v = *reinterpret_cast<const float4*>(g.work + sp * sstride + off);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    if (m < g.M) {
      if (n + 0 < g.N) reduce_store(g, z, m, n + 0, a.x);
      if (n + 1 < g.N) reduce_store(g, z, m, n + 1, a.y);
      if (n + 2 < g.N) reduce_store(g, z, m, n + 2, a.z);
      if (n + 3 < g.N) reduce_store(g, z, m, n + 3, a.w);
    }
  }
  if (g.rowsum && tn == 0) {  // the fused bias gradient: the tile's rows, splits in order
    for (int r = threadIdx.x; r < BMT; r += NT) {
      const int m = m0 + r;
      if (m >= g.M) continue;
      float a = 0.f;
      for (int sp = 0; sp < g.splits; ++sp)
        a += __hip_atomic_load(g.rs_work + (long)sp * g.M + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      g.rowsum[m] += a;
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(g.tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int EPI, int TM, int TN>
__device__ __forceinline__ void store_spec_tiles(const GemmArgs& g, int z, int mrow0, int ncol0, int lane,
                                                 f32x16 (&acc)[TM][TN]) {
  const bool full = mrow0 + TM * 32 <= g.M && ncol0 + TN * 32 <= g.N;
  if (EPI != EPI_SMB && g.alpha == 1.0f) {
    if (full) store_spec<EPI, TM, TN, true, true>(g, z, mrow0, ncol0, lane, acc);
    else store_spec<EPI, TM, TN, false, true>(g, z, mrow0, ncol0, lane, acc);
  } else {
    if (full) store_spec<EPI, TM, TN, true>(g, z, mrow0, ncol0, lane, acc);
    else store_spec<EPI, TM, TN, false>(g, z, mrow0, ncol0, lane, acc);
  }
}
// EPI_C1FOLD records per block: C1NT column tiles (N <= 512 at 128-wide tiles)
constexpr int C1NT = 4;
// EPI_C1FOLD: conv1's weight / bias gradient folded into the implicit conv2 input-gradient tile (the conv1-map
// gradient dz1 itself is never stored).  Per 32-column sub-tile j a lane holds, after the quad transpose, rows
// m (4 per 32-row tile) x columns n..n+3; dz1 = mask(bit map) * acc, and for every such value the 9 conv1
// taps x[b, 2 t1 + kt, 2 f1 + kf] and 1 (bias) are accumulated: 40 sums over the lane's 8 rows.  A
// reduce-scatter over the 8 lanes sharing the columns (lane bits 5, 1, 0) leaves lane s = (l32 & 3) + 4 h with
// sums 5 s .. 5 s + 4 (sum v: column n + v / 10, tap v % 10) over the wave's 64 rows, added into k[5 j ..].
// The lane's 8 rows are decomposed once for both sub-tiles (14.57 -> 14.27 ms per C2 B=256 call, r06v; with the
// accumulators kept live and no fold the class GEMMs take 12.0 ms: the fold epilogue is ~2.3 ms of VALU + loads).
// Host: N % 128 == 0 and 128 x 128 tiles (TM = TN = 2), the mask as a bit map (cm_bits).
template <int TM, int TN>
__device__ __forceinline__ void store_c1fold(const GemmArgs& g, int mrow0, int ncol0, int lane, f32x16 (&acc)[TM][TN],
                                             float (&k)[5 * TN]) {
  const int h = lane >> 5, l32 = lane & 31, b1 = (l32 >> 1) & 1, b0 = l32 & 1;
  // the lane's 8 rows decomposed once for both 32-column sub-tiles: mask-word and conv1-input addresses
  const uint32_t* wrow[TM][4];
  const float* xrow[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = min(mrow0 + i * 32 + 8 * q + 4 * h + (l32 & 3), g.M - 1);
      int b, t1, f1;
      row_btf(g, m, b, t1, f1);
      wrow[i][q] = g.cm_bits + (((long)b * g.cm_T1 + t1) * g.cm_F1 + f1) * g.cm_bw + (ncol0 >> 5);
      xrow[i][q] = g.c1_x + ((long)b * g.c1_T + 2 * t1) * g.c1_F + 2 * f1;
    }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int sh = 4 * (l32 >> 2);
    float a[40];
#pragma unroll
    for (int v = 0; v < 40; ++v) a[v] = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      quad_transpose(acc[i][j], lane);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = mrow0 + i * 32 + 8 * q + 4 * h + (l32 & 3);
        if (m >= g.M) continue;
        const uint32_t w = wrow[i][q][j] >> sh;
        const float* xp = xrow[i][q];
        float pt[9];
#pragma unroll
        for (int kt = 0; kt < 3; ++kt)
#pragma unroll
          for (int kf = 0; kf < 3; ++kf)
            pt[kt * 3 + kf] = xp[kt * g.c1_F + kf];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = (w >> e) & 1u ? acc[i][j][4 * q + e] : 0.f;
#pragma unroll
          for (int t = 0; t < 9; ++t) a[e * 10 + t] = fmaf(d, pt[t], a[e * 10 + t]);
          a[e * 10 + 9] += d;
        }
      }
    }
    // reduce-scatter: lane bit 5 (h) keeps sums [20 h, 20 h + 20), bit 1 [10 b1, +10) of those, bit 0 [5 b0, +5)
    float r20[20];
#pragma unroll
    for (int u = 0; u < 20; ++u) {
      const float send = h ? a[u] : a[20 + u];
      r20[u] = (h ? a[20 + u] : a[u]) + __shfl_xor(send, 32, 64);
    }
    float r10[10];
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const float send = b1 ? r20[u] : r20[10 + u];
      r10[u] = (b1 ? r20[10 + u] : r20[u]) +
               __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0x4E, 0xF, 0xF, false));
    }
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const float send = b0 ? r10[u] : r10[5 + u];
      k[5 * j + u] += (b0 ? r10[5 + u] : r10[u]) +
                      __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1, 0xF, 0xF, false));
    }
  }
}
template <int TM, int TN>
__device__ __forceinline__ void store_partials_wide(const GemmArgs& g, float* W, int mrow0, int ncol0, int lane,
                                                    f32x16 (&acc)[TM][TN]) {
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      quad_transpose(acc[i][j], lane);
      const int n = ncol0 + j * 32 + 4 * (l32 >> 2);
      if (n >= g.N) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = mrow0 + i * 32 + 8 * q + 4 * h + (l32 & 3);
        if (m < g.M)
          *reinterpret_cast<float4*>(W + (long)m * g.N + n) =
              make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]);
      }
    }
}

// split-K partial stores: W[split][z][M][N]
template <int TM, int TN>
__device__ __forceinline__ void store_partials(const GemmArgs& g, float* W, int mrow0, int ncol0, int h, int l32,
                                               const f32x16 (&acc)[TM][TN]) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = ncol0 + j * 32 + l32;
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mrow0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < g.M) W[(long)m * g.N + n] = acc[i][j][r];
      }
    }
}
template <int TM, int TN>
__device__ __forceinline__ void epilogue(const GemmArgs& g, float* W, int z, int mrow0, int ncol0, int h, int l32,
                                         const f32x16 (&acc)[TM][TN]) {
  if (W) store_partials<TM, TN>(g, W, mrow0, ncol0, h, l32, acc);
  else if (g.bwd_act) store_tiles<EPI_BWD, TM, TN>(g, z, mrow0, ncol0, h, l32, acc);
  else if (g.bias || g.aux || g.act || g.drop_thresh) store_tiles<EPI_FWD, TM, TN>(g, z, mrow0, ncol0, h, l32, acc);
  else store_tiles<EPI_PLAIN, TM, TN>(g, z, mrow0, ncol0, h, l32, acc);
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
  epilogue<2, 2>(g, W, z, m0 + wm * 64, n0 + wn * 64, h, l32, acc);
}

// ============================================================================ bf16 kernel
// bf16-input MFMA GEMM (v_mfma_f32_32x32x16_bf16, fp32 accumulate) for the reduced-precision
// training mode (bf16 GEMM inputs, fp32 master weights / activations in HBM).
// Register-staged FALLBACK for operands the LDS-DMA kernel cannot take (unaligned pitches);
// the production bf16 path is gemm_glds_kernel<..., BF16 = true> below.
// Operands stay fp32 in HBM; each 128 x 32 slab is loaded as float4, rounded to bf16 (RNE,
// v_cvt_pk_bf16_f32) and written to LDS as [row][k] with a 40-element (80 B) row pitch, so the
// per-lane fragment of a 32x32x16 step (8 consecutive k of one row, k = 16s + 8h + j) is one
// conflict-free ds_read_b128 (row pitch 20 dwords: 16 rows cover the 64 banks once).
//   KC operands: the thread's float4 is 4 consecutive k of one row -> one ds_write_b64.
//   RC operands: the thread loads 4 float4 (k .. k+3) x (rows r .. r+3) and transposes in
//                registers -> four ds_write_b64 (row r+i, k .. k+3).
// The next slab's global loads fly during this slab's MFMAs (single LDS buffer, two barriers
// per slab).  Epilogues, split-K partials and the row-sum side pass are those of the fp32 path.
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
constexpr int BF_KS = 32 + 8;  // LDS row pitch in bf16 elements

template <int MODE>
__device__ __forceinline__ float4 ld4_rc(const Operand& op, const float* base, int rows, int K, int gk, int gr) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (gk >= K) return v;
  if constexpr (MODE == RC) {
    const float* p = base + (long)gk * op.ld + gr;
    if (op.vec && gr + 3 < rows) return *reinterpret_cast<const float4*>(p);
    if (gr + 0 < rows) v.x = p[0];
    if (gr + 1 < rows) v.y = p[1];
    if (gr + 2 < rows) v.z = p[2];
    if (gr + 3 < rows) v.w = p[3];
  } else {  // I2C_RC
    if (gr + 3 < rows) return *reinterpret_cast<const float4*>(i2c_ptr(base, op.ic, gk, gr));
    if (gr + 0 < rows) v.x = *i2c_ptr(base, op.ic, gk, gr + 0);
    if (gr + 1 < rows) v.y = *i2c_ptr(base, op.ic, gk, gr + 1);
    if (gr + 2 < rows) v.z = *i2c_ptr(base, op.ic, gk, gr + 2);
  }
  return v;
}

// this thread's 16 elements of a (128 rows x 32 k) slab
template <int MODE>
__device__ __forceinline__ void load_slab_bf(const Operand& op, const float* base, int rows, int K, int row0,
                                             int k0, float4 (&reg)[4]) {
  if constexpr (MODE == KC || MODE == I2C_KC) {
    load_slab<MODE, 32>(op, base, rows, K, row0, k0, reg);  // reg[it]: row (t + 256 it) / 8, k 4 * (t % 8)
  } else {
    const int rq = (threadIdx.x & 31) * 4, kq = (threadIdx.x >> 5) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) reg[j] = ld4_rc<MODE>(op, base, rows, K, k0 + kq + j, row0 + rq);
  }
}

__device__ __forceinline__ bf16x4 to_bf4(float a, float b, float c, float d) {
  bf16x4 r;
  r[0] = (__bf16)a; r[1] = (__bf16)b; r[2] = (__bf16)c; r[3] = (__bf16)d;
  return r;
}

template <int MODE>
__device__ __forceinline__ void store_slab_bf(__bf16* lds, const float4 (&reg)[4]) {
  if constexpr (MODE == KC || MODE == I2C_KC) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = threadIdx.x + it * NT;
      const int r = idx >> 3, kq = (idx & 7) * 4;
      *reinterpret_cast<bf16x4*>(lds + r * BF_KS + kq) = to_bf4(reg[it].x, reg[it].y, reg[it].z, reg[it].w);
    }
  } else {
    const int rq = (threadIdx.x & 31) * 4, kq = (threadIdx.x >> 5) * 4;
    *reinterpret_cast<bf16x4*>(lds + (rq + 0) * BF_KS + kq) = to_bf4(reg[0].x, reg[1].x, reg[2].x, reg[3].x);
    *reinterpret_cast<bf16x4*>(lds + (rq + 1) * BF_KS + kq) = to_bf4(reg[0].y, reg[1].y, reg[2].y, reg[3].y);
    *reinterpret_cast<bf16x4*>(lds + (rq + 2) * BF_KS + kq) = to_bf4(reg[0].z, reg[1].z, reg[2].z, reg[3].z);
    *reinterpret_cast<bf16x4*>(lds + (rq + 3) * BF_KS + kq) = to_bf4(reg[0].w, reg[1].w, reg[2].w, reg[3].w);
  }
}

template <int MA, int MB>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[(BM + BN) * BF_KS];
  __bf16* As = lds;
  __bf16* Bs = lds + BM * BF_KS;

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

  float4 ra[4], rb[4];
  const int nk = kend > kbeg ? (kend - kbeg + 31) / 32 : 0;
  if (nk > 0) {
    load_slab_bf<MA>(g.a, Ab, g.M, kend, m0, kbeg, ra);
    load_slab_bf<MB>(g.b, Bb, g.N, kend, n0, kbeg, rb);
  }
  for (int kt = 0; kt < nk; ++kt) {
    if (kt > 0) __syncthreads();  // previous slab fully read
    store_slab_bf<MA>(As, ra);
    store_slab_bf<MB>(Bs, rb);
    __syncthreads();
    if (kt + 1 < nk) {
      load_slab_bf<MA>(g.a, Ab, g.M, kend, m0, kbeg + (kt + 1) * 32, ra);
      load_slab_bf<MB>(g.b, Bb, g.N, kend, n0, kbeg + (kt + 1) * 32, rb);
    }
    bf16x8 af[2][2], bf[2][2];  // [tile][k-step]
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        af[t][s] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + t * 32 + l32) * BF_KS + 16 * s + 8 * h);
        bf[t][s] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + t * 32 + l32) * BF_KS + 16 * s + 8 * h);
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
  }

  float* W = g.splits > 1 ? g.work + ((long)split * g.batch + z) * (long)g.M * g.N : nullptr;
  if (g.wide) {
    if (W) store_partials_wide<2, 2>(g, W, m0 + wm * 64, n0 + wn * 64, lane, acc);
    else if (g.bwd_act) store_tiles_wide<EPI_BWD, 2, 2>(g, z, m0 + wm * 64, n0 + wn * 64, lane, acc);
    else if (g.bias || g.aux || g.act || g.drop_thresh)
      store_tiles_wide<EPI_FWD, 2, 2>(g, z, m0 + wm * 64, n0 + wn * 64, lane, acc);
    else store_tiles_wide<EPI_PLAIN, 2, 2>(g, z, m0 + wm * 64, n0 + wn * 64, lane, acc);
  } else {
    epilogue<2, 2>(g, W, z, m0 + wm * 64, n0 + wn * 64, h, l32, acc);
  }
}

// ============================================================================ glds kernel
// The production path.  Global->LDS staging with global_load_lds_dwordx4 (LDS-DMA: no VGPR
// round trip, asynchronous until its vmcnt), two LDS buffers, raw s_barrier with explicit
// waits, so slab k+1 streams in while slab k's MFMAs run.  All LDS in ONE __shared__ array
// (a second object makes hipcc drain vmcnt before every ds_read).  Requires 16-B aligned
// operands with ld % 4 == 0 (the host falls back to the register-staged kernel otherwise).
//
// LDS images are lane-linear per wave instruction (1 KB = 64 lanes x 16 B); the swizzle is
// applied to the per-lane GLOBAL source address:
//   KC [rows][32]: quad q of row r at slot r*8 + (q ^ (r&7))   -> ds_read_b128 conflict-free
//   RC [32][rows]: element (k,r) at k*rows + (r ^ ((k>>4)<<5)) -> the two lane halves
//                  (k and k+16) land on opposite 32-bank halves, ds_read_b32 conflict-free
// Out-of-range rows / k are clamped to in-bounds addresses (their products only reach
// discarded outputs); the K tail of the last slab is zeroed in LDS before use.
// Block ids are remapped so that consecutive tiles (same A row panel) share an XCD's L2.


struct GldsArgs {
  FastDiv c_a, c_b;    // im2col channel count C
  FastDiv hw_b, wo_b;  // I2C_RC: output pixels per map (Ho*Wo), Wo
  FastDiv hw_a, wo_a;  // I2C_KC
  int ntx, nty;        // tile grid (N tiles, M tiles)
  int ntiles;          // ntx * nty * batch * splits
  // the tile-coordinate divisors as multiply-high reciprocals (set by the host launcher): on
  // wave-uniform operands they compile to s_mul_hi_u32, where an integer division took ~30
  // instructions incl. VALU reciprocals per tile
  FastDiv fd_grid, fd_ntx, fd_nty, fd_splits, fd_nb2;
  // I2CT_KC (conv2 input gradient as an implicit GEMM per parity class): A(r, k) =
  // dY[b, a - dt[t], e - df[t], o] (0 outside the T2 x F2 grid), r = (b, a, e) over Ha x We,
  // k = t*C + o (tap t of the class, channel o); C % 32 == 0 so a slab never straddles taps
  FastDiv t_hw, t_w;
  int t_T2, t_F2, t_C;
  int t_dt[4], t_df[4];
  const float* t_zeros;  // >= 16 zero bytes: the DMA source of lanes outside the grid
};
// (Round 6: the diagnostic ablation bits, the 3-slab ring, the all-GEMM 256 x 128 tiles, the iglp_opt hint and
// the product-major MFMA order -- timing builds and measured-slower variants, DESIGN 3.1 / 3.10 -- were removed
// from the product header; their code is in git history before this note.)

constexpr int GL_BK = 32;
// LDS slab ring depth of the LDS-DMA kernel: 2 (double buffer: slab k+1 in flight while k is read, every
// slab waits vmcnt(0))
// 256 x 128 tiles of 8 waves for the KC x RC GEMMs on B planes only (the pairs they speed up: the linear
// input gradients / P0 / FFN w_2 shapes 3-7 %, profiles/r05am_*)
#ifndef ESP_GEMM_WIDE_KCRC
#define ESP_GEMM_WIDE_KCRC 1
#endif
constexpr int GL_ST = 2;

// K-contiguous slab image: row r (128 B = 8 quads) holds global quad q at position q ^ kc_swz(r).
// A ds_read_b128 of frag16 serves 16-lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32)
// whose lanes read rows r = lane & 31 at one quad; rows r and r+1 share a 256-B bank row, so the
// 16 reads are conflict-free iff (r & 1, swz(r)) is distinct within each group: (r >> 1) & 7 is
// (the round-1 r & 7 repeats at r + 8 inside a group: 2-way, SQ_LDS_BANK_CONFLICT 4 cycles per
// ds_read, profiles/r02x_pmc_gemm.txt).
__device__ __forceinline__ int kc_swz(int r) { return (r >> 1) & 7; }

// One global_load_lds_dwordx4: lane l's 16 B at gptr land at lds_wave_base + 16*l.  Issued from
// inline asm so that hipcc does not see an LDS-DMA store: with the builtin it cannot prove
// the DMA target (the other buffer) disjoint from this slab's ds_reads and drains vmcnt(0)
// before every slab's first ds_read, serialising the pipeline.  The ordering the compiler
// no longer sees is made explicit: wait_vm0() + raw_barrier() before a slab is read, and the
// "memory" clobber keeps LDS accesses on their side of the asm.  M0 is set per instruction.
__device__ __forceinline__ void lds_dma16(const float* gptr, float* lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr), "s"(m0) : "memory", "m0");
}

// element offset of im2col column `col` (= (kt,kf,c)) relative to the receptive field origin
__device__ __forceinline__ long i2c_col_off(const Im2col& ic, const FastDiv& fc, int col) {
  const int kk = (int)fdiv((uint32_t)col, fc), c = col - kk * ic.C;
  const int kt = kk / 3, kf = kk - kt * 3;
  return ((long)kt * ic.W + kf) * ic.C + c;
}
// element offset of output pixel `pix`'s receptive field origin
__device__ __forceinline__ long i2c_pix_off(const Im2col& ic, const FastDiv& fhw, const FastDiv& fwo, int pix) {
  const int bi = (int)fdiv((uint32_t)pix, fhw);
  const int rem = pix - bi * (int)fhw.d;
  const int ho = (int)fdiv((uint32_t)rem, fwo), wo = rem - ho * (int)fwo.d;
  return (((long)bi * ic.H + 2 * ho) * ic.W + 2 * wo) * ic.C;
}

// the same on 24-bit multiplies (v_mad_u32_u24, full rate; v_mul_lo_u32 is quarter rate): legal
// when Bn*H*W < 2^24 and the map holds < 2^32 elements (host-checked for I2C_RC operands)
__device__ __forceinline__ uint32_t i2c_pix_off24(const Im2col& ic, const FastDiv& fhw, const FastDiv& fwo,
                                                  uint32_t pix) {
  const uint32_t bi = fdiv(pix, fhw);
  const uint32_t rem = pix - __umul24(bi, fhw.d);
  const uint32_t ho = fdiv(rem, fwo), wo = rem - __umul24(ho, fwo.d);
  return __umul24(__umul24(__umul24(bi, (uint32_t)ic.H) + 2 * ho, (uint32_t)ic.W) + 2 * wo, (uint32_t)ic.C);
}

// 16-byte chunk swizzle of a bf16 RC slab's k-row (see StageS)
__device__ __forceinline__ int bf16_rc_swz(int rowb, int kr) {
  return rowb == 256 ? (kr & 3) << 2 : ((kr >> 1) & 1) << 2;
}

// Per-lane source bookkeeping for one operand: NI wave-instructions per slab.
// B16 (PREC 2, bf16 pairs; I2C_RC: the bf16 conv2 weight gradient's gathered B): the slab is the bf16
// RC image of StageS (64 pixel k-rows x ROWS bf16 columns, 16-B chunks of 8 channels XOR-swizzled by
// k-row, bf16_rc_swz) and the im2col offsets are computed in bf16 elements (ic.C = bf16 channels)
template <int MODE, int ROWS, int NI, bool B16 = false, int NW = 4>
struct Stage {
  static constexpr int kNI = NI;  // DMA instructions per slab issue (per wave)
  static constexpr bool kKC = MODE == KC || MODE == I2C_KC || MODE == I2CT_KC;
  static_assert(!B16 || MODE == I2C_RC || kKC, "Stage<B16>: bf16 pairs for the gathered operands only");
  const float* p[NI];  // per instruction: base incl. the slab-invariant part
  int q[NI];           // KC: k offset inside the slab (4*quad) ; RC: k-row inside the slab
  int ga[MODE == I2CT_KC ? NI : 1], ge[MODE == I2CT_KC ? NI : 1];  // I2CT: class-grid row / column
  __device__ __forceinline__ void init(const Operand& op, const float* base, int rows, int K, int row0,
                                       const FastDiv& fc, const FastDiv& fhw, const FastDiv& fwo, int wave,
                                       int lane, const GldsArgs* x = nullptr) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int slot = (i * NW + wave) * 64 + lane;
      if constexpr (kKC) {
        const int r = slot >> 3, qs = slot & 7;
        const int qq = qs ^ kc_swz(r);
        const int gr = min(row0 + r, rows - 1);
        q[i] = 4 * qq;
        if constexpr (MODE == KC) p[i] = base + (long)gr * op.ld;
        else if constexpr (MODE == I2C_KC) p[i] = base + i2c_pix_off(op.ic, fhw, fwo, gr);
        else {
          const int bb = (int)fdiv((uint32_t)gr, x->t_hw);
          const int rem = gr - bb * (int)x->t_hw.d;
          const int a = (int)fdiv((uint32_t)rem, x->t_w), e = rem - a * (int)x->t_w.d;
          ga[i] = a;
          ge[i] = e;
          p[i] = base + (((long)bb * x->t_T2 + a) * x->t_F2 + e) * x->t_C;
        }
      } else if constexpr (B16) {  // I2C_RC in bf16: chunk of 8 channel columns, pixel k-row kr
        constexpr int QPR = ROWS / 8;  // 16-byte chunks per k-row
        const int kr = slot / QPR, c = slot % QPR;
        const int cs = c ^ bf16_rc_swz(ROWS * 2, kr);
        const int gn = min(row0 + 8 * cs, (rows - 1) & ~7);  // first column of the chunk
        q[i] = kr;
        p[i] = base + (i2c_col_off(op.ic, fc, gn) >> 1);  // bf16 elements -> pairs
      } else {
        constexpr int QPR = ROWS / 4;  // quads per k-row
        const int kr = slot / QPR, rs = slot % QPR;
        const int rq = rs ^ (((kr >> 4) & 1) << 3);
        const int gr = min(row0 + 4 * rq, (rows - 1) & ~3);
        q[i] = kr;
        if constexpr (MODE == RC) p[i] = base + gr;
        else p[i] = base + i2c_col_off(op.ic, fc, gr);
      }
    }
  }
  // issue this lane's NI LDS-DMA loads of the slab starting at k0 into `dst`
  __device__ __forceinline__ void issue(const Operand& op, int K, int k0, float* dst, int wave, const FastDiv& fc,
                                        const FastDiv& fhw, const FastDiv& fwo, const GldsArgs* x = nullptr) const {
    int dt = 0, df = 0, o0 = 0;
    long tap_off = 0;
    if constexpr (MODE == I2C_KC) {  // the slab's tap and channel offset (wave-uniform scalars)
      const int t = k0 / op.ic.C, kt = t / 3, kf = t - 3 * kt;
      tap_off = ((long)kt * op.ic.W + kf) * op.ic.C + (k0 - t * op.ic.C);
    }
    if constexpr (MODE == I2CT_KC) {  // the slab's tap (uniform: C % 32 == 0)
      const int t = k0 / x->t_C;
      o0 = k0 - t * x->t_C;
      dt = x->t_dt[t];
      df = x->t_df[t];
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      float* ldsw = dst + (i * NW + wave) * 256;
      if constexpr (kKC) {
        const int k = min(k0 + q[i], (K - 1) & ~3);
        if constexpr (MODE == KC) lds_dma16(p[i] + k, ldsw);
        else if constexpr (MODE == I2C_KC) {
          lds_dma16(p[i] + tap_off + q[i], ldsw);  // C % 32 == 0, K % 32 == 0 (host-checked)
        }
        else {
          const int a = ga[i] - dt, e = ge[i] - df;
          const bool in = a >= 0 && a < x->t_T2 && e >= 0 && e < x->t_F2;
          lds_dma16(in ? p[i] - ((long)dt * x->t_F2 + df) * x->t_C + o0 + q[i] : x->t_zeros, ldsw);
        }
      } else if constexpr (B16) {  // pixel 2 k0 + kr (K counts pixel pairs)
        const int pix = min(2 * k0 + q[i], 2 * K - 1);
        lds_dma16(p[i] + (i2c_pix_off24(op.ic, fhw, fwo, (uint32_t)pix) >> 1), ldsw);
      } else {
        const int k = min(k0 + q[i], K - 1);
        if constexpr (MODE == RC) lds_dma16(p[i] + (long)k * op.ld, ldsw);
        else lds_dma16(p[i] + i2c_pix_off24(op.ic, fhw, fwo, (uint32_t)k), ldsw);
      }
    }
  }
};

// One global_load_lds_dwordx4 in the scalar-base form: address = sbase (wave-uniform, SGPR pair)
// + voff (per-lane unsigned 32-bit byte offset).  The slab advance is scalar arithmetic on sbase,
// so a slab's DMAs cost no VALU (the 64-bit per-lane form paid ~6 VALU per DMA, and f32 MFMAs do
// not hide VALU: DESIGN §3.5).
// lds_wave_base: LDS byte address (wave-uniform) of the wave's 1 KB destination.
__device__ __forceinline__ void lds_dma16_s(const float* sbase, uint32_t voff, uint32_t lds_wave_base) {
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_wave_base)
               : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_addr(const float* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const float*)p);
}

// Per-lane source bookkeeping with a wave-uniform tile base (KC, RC, I2C_KC operands).  The
// per-lane part is a 32-bit byte offset inside the tile's panel: KC rows r < 128 of pitch ld
// (host: 127 * ld * 4 + 128 < 2^32), RC k-rows < 32 (32 * ld * 4 < 2^32), I2C_KC pixel offsets
// relative to the tile's first pixel (a 128-pixel run spans <= 2 maps; host: 2 maps < 2^32 B).
//   KC     sbase(k0) = base + (k0 - kb)               base = A_z + row0 * ld + kb
//   RC     sbase(k0) = base + (k0 - kb) * ld          base = A_z + kb * ld
//   I2C_KC sbase(k0) = base + tap_off(k0)             base = A_z + pix_off(row0)
// Lanes past the last row read a clamped row (their products only reach discarded outputs).  Only
// a slab that reaches past K clamps k per lane (KC: to the last whole quad, RC: to K - 1).
// B16 (PREC 2, bf16 operands viewed as fp32 pairs): KC operands are staged as in fp32 (a slab
// holds 32 pairs = 64 bf16 k per row); an RC operand's slab is 64 k-rows x ROWS bf16 (ROWS * 2
// bytes per k-row, the same 16 KB / 8 KB as every other slab), its 16-byte chunks XOR-swizzled
// by k-row (bf16_rc_swz) for the transposing reads of frag_tr16.  K and k0 count pairs; an RC
// k-row index is 2 * k + (0..63).  `rows` and `ld` of an RC operand: bf16 rows, ld in pairs.

template <int MODE, int ROWS, int NI, bool B16 = false, int NW = 4>
struct StageS {
  static constexpr int kNI = NI;
  static constexpr bool kKC = MODE == KC || MODE == I2C_KC;
  static constexpr bool kT16 = B16 && MODE == RC;  // transposed-read bf16 image
  const float* base;
  long ld;
  int kb;
  uint32_t off[NI];
  int q[NI];  // KC: k offset inside the slab (4 * quad); RC: k-row inside the slab
  __device__ __forceinline__ void init(const Operand& op, const float* zbase, int rows, int K, int row0, int kbeg,
                                       const FastDiv& fhw, const FastDiv& fwo, int wave, int lane) {
    ld = op.ld;
    kb = kbeg;
    long pix0 = 0;
    if constexpr (MODE == KC) base = zbase + (long)row0 * op.ld + kbeg;
    else if constexpr (kT16) base = zbase + (long)2 * kbeg * op.ld;
    else if constexpr (MODE == RC) base = zbase + (long)kbeg * op.ld;
    else {
      pix0 = i2c_pix_off(op.ic, fhw, fwo, row0);
      base = zbase + pix0;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int slot = (i * NW + wave) * 64 + lane;
      if constexpr (kKC) {
        const int r = slot >> 3, qq = (slot & 7) ^ kc_swz(r);
        const int gr = min(row0 + r, rows - 1);
        q[i] = 4 * qq;
        if constexpr (MODE == KC) off[i] = (uint32_t)(((uint32_t)(gr - row0) * (uint32_t)op.ld + 4 * qq) * 4u);
        else off[i] = (uint32_t)((i2c_pix_off(op.ic, fhw, fwo, gr) - pix0 + 4 * qq) * 4);
      } else if constexpr (kT16) {
        constexpr int QPR = ROWS / 8;  // 16-byte chunks (8 bf16 rows) per k-row
        const int kr = slot / QPR, c = slot % QPR;
        const int cs = c ^ bf16_rc_swz(ROWS * 2, kr);
        const int gp = min((row0 >> 1) + 4 * cs, ((rows >> 1) - 1) & ~3);  // first pair of the chunk
        q[i] = kr;
        off[i] = (uint32_t)(((uint32_t)kr * (uint32_t)op.ld + (uint32_t)gp) * 4u);
      } else {
        constexpr int QPR = ROWS / 4;  // quads per k-row
        const int kr = slot / QPR, rs = slot % QPR;
        const int rq = rs ^ (((kr >> 4) & 1) << 3);
        const int gr = min(row0 + 4 * rq, (rows - 1) & ~3);
        q[i] = kr;
        off[i] = (uint32_t)(((uint32_t)kr * (uint32_t)op.ld + (uint32_t)gr) * 4u);
      }
    }
  }
  // this lane's NI LDS-DMA loads of the slab starting at k0 into LDS byte address `dst`
  __device__ __forceinline__ void issue(const Operand& op, int K, int k0, uint32_t dst, int wave) const {
    const float* sb;
    if constexpr (MODE == KC) sb = base + (k0 - kb);
    else if constexpr (kT16) sb = base + (long)2 * (k0 - kb) * ld;
    else if constexpr (MODE == RC) sb = base + (long)(k0 - kb) * ld;
    else {  // the slab's tap and channel offset (C % 32 == 0, K % 32 == 0: host-checked)
      const int t = k0 / op.ic.C, kt = t / 3, kf = t - 3 * kt;
      sb = base + ((long)kt * op.ic.W + kf) * op.ic.C + (k0 - t * op.ic.C);
    }
    if (MODE == I2C_KC || k0 + GL_BK <= K) {
#pragma unroll
      for (int i = 0; i < NI; ++i) lds_dma16_s(sb, off[i], dst + (i * NW + wave) * 1024);
    } else {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        uint32_t o = off[i];
        if constexpr (MODE == KC) o -= 4u * (uint32_t)max(0, q[i] - (((K - 1) & ~3) - k0));
        else if constexpr (kT16) o -= 4u * (uint32_t)ld * (uint32_t)max(0, q[i] - (2 * (K - k0) - 1));
        else o -= 4u * (uint32_t)ld * (uint32_t)max(0, q[i] - (K - 1 - k0));
        lds_dma16_s(sb, o, dst + (i * NW + wave) * 1024);
      }
    }
  }
};

// bf16 RC operand (PREC 2): the four 32x32x16 MFMA fragments of the 32 tile rows starting at
// rbase, by ds_read_b64_tr_b16 (T10): a 16-lane group reads a 4 k-row x 16 row block and lane i
// receives row i's 4 k values.  Lane (h, l32) gets rows rbase + l32 at bf16 k = 32h + 8t + 0..7
// for step t -- the k a KC operand's lane supplies from its frag16 chunk t (both operands agree).
// Lane 4q+p supplies the address of k-row kb + q, rows 4p..4p+3 of its group's 16; the chunk
// swizzle of k-row kb + q is a function of q alone (kb % 4 == 0), so every read is the lane's
// base address + an immediate.  Conflict-free: a 32-lane half covers the 64 banks once.
typedef short v4i16 __attribute__((ext_vector_type(4)));
template <int ROWS>
__device__ __forceinline__ void frag_tr16(const float* slab, int rbase, int lane, float4 (&f)[4]) {
  constexpr int ROWB = ROWS * 2;
  const int g1 = (lane >> 4) & 1, h = lane >> 5, q = (lane >> 2) & 3, p = lane & 3;
  const int mloc = rbase + 16 * g1 + 4 * p;
  const int base = (32 * h + q) * ROWB + (((mloc >> 3) ^ bf16_rc_swz(ROWB, q)) << 4) + 8 * (p & 1);
  const __attribute__((address_space(3))) char* s =
      (const __attribute__((address_space(3))) char*)(__attribute__((address_space(3))) const float*)slab;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4i16*)(s + base + 8 * t * ROWB));
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4i16*)(s + base + (8 * t + 4) * ROWB));
    const int2 a = __builtin_bit_cast(int2, lo), b = __builtin_bit_cast(int2, hi);
    f[t] = make_float4(__int_as_float(a.x), __int_as_float(a.y), __int_as_float(b.x), __int_as_float(b.y));
  }
}

// ---------------------------------------------------------------- B as three bf16 planes (PREC 3)
// An fp32 B operand stored as its exact three-way split (esp_f32_to_planes: v = hi + mid + lo with
// split3_bf16's roundings), plane p at B + p * ps (bf16 elements; ld and batch strides in bf16
// elements too).  The fp32 product is the PREC 0 one -- the same six split products in the same
// order on the same values, bit for bit -- but only A is split in the k-loop: 3.7 instead of 7.3
// split VALU per MFMA, under the ~5 an MFMA gap hides.  A slab holds the three planes' images of
// ROWS x 32 k, PLB = ROWS * 64 bytes each:
//   KC  row r (64 B = 4 chunks of 8 k) holds global chunk c at position c ^ pl_kc_swz(r).  The
//       ds_read_b128 groups of frag_pl_kc ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) read rows
//       r = lane & 31 at one chunk; rows 4j..4j+3 share a 256-B bank row and (r & 3, swz(r)) is
//       distinct in each group: conflict-free.
//   RC  k-row kr (2 ROWS bytes) holds the 16-B chunk c (8 rows) at position c ^ bf16_rc_swz(2 ROWS, kr)
//       and is read transposed (frag_pl_rc, ds_read_b64_tr_b16; conflict-free as frag_tr16).
// Host: K % 8 == 0 (KC), N % 8 == 0 (RC), 16-B aligned planes, ld / strides / ps % 8 == 0.
__device__ __forceinline__ int pl_kc_swz(int r) { return (r >> 2) & 3; }

template <int MODE, int ROWS, int NW = 4>
struct StageP {
  static constexpr int PLB = ROWS * 64;           // bytes of one plane's slab image
  static constexpr int NI = PLB / 1024 / NW;      // wave instructions per plane per wave
  static constexpr int kNI = 3 * NI;
  const char* base;  // plane 0 at the tile's first row / k-row kb (bytes)
  long ld, psb;      // ld in bf16 elements, plane stride in bytes
  int kb;
  uint32_t off[NI];
  int q[NI];  // KC: k offset of the lane's chunk inside the slab; RC: k-row inside the slab
  __device__ __forceinline__ void init(const Operand& op, const float* zbase, int rows, int row0, int kbeg, int wave,
                                       int lane) {
    const __bf16* zb = reinterpret_cast<const __bf16*>(zbase);
    ld = op.ld;
    psb = op.ps * 2;
    kb = kbeg;
    base = reinterpret_cast<const char*>(MODE == KC ? zb + (long)row0 * op.ld + kbeg : zb + (long)kbeg * op.ld);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int slot = (i * NW + wave) * 64 + lane;
      if constexpr (MODE == KC) {
        const int r = slot >> 2, gc = (slot & 3) ^ pl_kc_swz(r);
        const int gr = min(row0 + r, rows - 1);
        q[i] = 8 * gc;
        off[i] = ((uint32_t)(gr - row0) * (uint32_t)op.ld + 8u * gc) * 2u;
      } else {
        constexpr int CPR = ROWS / 8;  // 16-B chunks per k-row
        const int kr = slot / CPR, cs = (slot % CPR) ^ bf16_rc_swz(ROWS * 2, kr);
        const int gr = min(row0 + 8 * cs, rows - 8);
        q[i] = kr;
        off[i] = ((uint32_t)kr * (uint32_t)op.ld + (uint32_t)gr) * 2u;
      }
    }
  }
  __device__ __forceinline__ void issue(int K, int k0, uint32_t dst, int wave) const {
    const char* sb = MODE == KC ? base + 2L * (k0 - kb) : base + 2L * (long)(k0 - kb) * ld;
    const bool full = k0 + GL_BK <= K;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        uint32_t o = off[i];
        if (!full) {  // clamp past-K chunks / k-rows to the last in-range one (finite values; A's tail is 0)
          if constexpr (MODE == KC) o -= 2u * (uint32_t)max(0, q[i] - (K - 8 - k0));
          else o -= 2u * (uint32_t)ld * (uint32_t)max(0, q[i] - (K - 1 - k0));
        }
        lds_dma16_s(reinterpret_cast<const float*>(sb + p * psb), o, dst + p * PLB + (i * NW + wave) * 1024);
      }
  }
};
// KC plane image: the 8 bf16 at k = 16h + 8hs + 0..7 of tile row r (frag16's k order, split in halves)
__device__ __forceinline__ bf16x8 frag_pl_kc(const float* plane, int r, int h, int hs) {
  return *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(plane) + r * 64 +
                                          (((2 * h + hs) ^ pl_kc_swz(r)) << 4));
}
// RC plane image: lane (h, l32) gets row rbase + l32 at k = 16h + 8hs + 0..7 (two transposing reads
// of 4 k-rows; k-rows 16h + 8hs + q (+4) share the swizzle of q: 16h + 8hs % 8 == 0)
template <int ROWS>
__device__ __forceinline__ bf16x8 frag_pl_rc(const float* plane, int rbase, int lane, int hs) {
  constexpr int ROWB = ROWS * 2;
  const int g1 = (lane >> 4) & 1, h = lane >> 5, q = (lane >> 2) & 3, p = lane & 3;
  const int mloc = rbase + 16 * g1 + 4 * p;
  const int base = (16 * h + 8 * hs + q) * ROWB + (((mloc >> 3) ^ bf16_rc_swz(ROWB, q)) << 4) + 8 * (p & 1);
  const __attribute__((address_space(3))) char* s =
      (const __attribute__((address_space(3))) char*)(__attribute__((address_space(3))) const float*)plane;
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(s + base));
  const v4i16 hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(s + base + 4 * ROWB));
  const int2 a = __builtin_bit_cast(int2, lo), b = __builtin_bit_cast(int2, hi);
  return __builtin_bit_cast(bf16x8, make_int4(a.x, a.y, b.x, b.y));
}

// the 16 k-values (k = 16h + s) of tile row r
template <int MODE, int ROWS>
__device__ __forceinline__ void frag16(const float* slab, int r, int h, float (&f)[16]) {
  if constexpr (MODE == KC || MODE == I2C_KC || MODE == I2CT_KC) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 v = *reinterpret_cast<const float4*>(slab + (r * 8 + ((4 * h + j) ^ kc_swz(r))) * 4);
      f[4 * j + 0] = v.x; f[4 * j + 1] = v.y; f[4 * j + 2] = v.z; f[4 * j + 3] = v.w;
    }
  } else {
    const int rr = r ^ (h << 5);
#pragma unroll
    for (int s = 0; s < 16; ++s) f[s] = slab[(16 * h + s) * ROWS + rr];
  }
}

// half of frag16: the 8 k-values k = 16h + 8hs + s (s = 0..7) of tile row r -- the values the fp32
// split products of k-step hs take (PREC 0 / 3), read one k-step ahead in the pipelined k-loop
template <int MODE, int ROWS>
__device__ __forceinline__ void frag8(const float* slab, int r, int h, int hs, float (&f)[8]) {
  if constexpr (MODE == KC || MODE == I2C_KC || MODE == I2CT_KC) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float4 v = *reinterpret_cast<const float4*>(slab + (r * 8 + ((4 * h + 2 * hs + j) ^ kc_swz(r))) * 4);
      f[4 * j + 0] = v.x; f[4 * j + 1] = v.y; f[4 * j + 2] = v.z; f[4 * j + 3] = v.w;
    }
  } else {
    const int rr = r ^ (h << 5);
#pragma unroll
    for (int s = 0; s < 8; ++s) f[s] = slab[(16 * h + 8 * hs + s) * ROWS + rr];
  }
}

__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <int N>
__device__ __forceinline__ void wait_vm_n() {
  static_assert(N >= 0 && N < 64, "vmcnt: 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_barrier without __syncthreads()'s fence (which would drain vmcnt); the empty asm keeps
// the compiler from moving LDS accesses across it
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Tile t of the launch -> coordinates.  Tiles are processed in rounds of G (the grid): tile t
// runs on block t % G, which the hardware placed on XCD (t % G) & 7; inside a round the tile
// order is remapped (bijectively, also for a partial last round) so that the tiles resident on
// one XCD at the same time are consecutive: they share A row panels in that XCD's L2.
struct TileCoord {
  int m0, n0, tn, z, split, kbeg, kend, nk;
};
template <int BNT, int BMT = BM>
__device__ __forceinline__ TileCoord tile_coord(const GemmArgs& g, const GldsArgs& x, int t, int G) {
  const int round = (int)fdiv((uint32_t)t, x.fd_grid), b = t - round * G;
  const int nr = min(G, x.ntiles - round * G);
  const int xcd = b & 7, per = nr >> 3, rem = nr & 7;
  const int wg = round * G + (xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per) + (b >> 3);
  TileCoord c;
  const int t2 = (int)fdiv((uint32_t)wg, x.fd_ntx);
  c.tn = wg - t2 * x.ntx;
  const int zz = (int)fdiv((uint32_t)t2, x.fd_nty);
  const int tm = t2 - zz * x.nty;
  c.z = (int)fdiv((uint32_t)zz, x.fd_splits);
  c.split = zz - c.z * g.splits;
  c.kbeg = c.split * g.kchunk;
  c.kend = min(g.K, c.kbeg + g.kchunk);
  if (g.band_w) {  // the row tile's band union, slab-aligned below (the rows' zeros outside cost nothing)
    const int m0 = tm * BMT;
    const int lo = max(0, g.band_c0 - (m0 + BMT - 1)) / GL_BK * GL_BK;
    const int hi = min(g.K, g.band_c0 - m0 + g.band_w);
    const int kb = max(c.kbeg, lo), ke = min(c.kend, hi);
    if (kb < ke) {
      c.kbeg = kb;
      c.kend = ke;
    } else {
      // a split-K chunk wholly below lo or at/above hi: its own first column, which is zero in
      // every row of the tile (lo and hi bound the union of the rows' bands), so the unit adds
      // exactly nothing.  (Not lo: the split that owns lo computes that column already.)
      c.kend = c.kbeg + 1;
    }
  }
  c.nk = (c.kend - c.kbeg + GL_BK - 1) / GL_BK;  // >= 1: the host routes K == 0 elsewhere
  c.m0 = tm * BMT;
  c.n0 = c.tn * BNT;
  return c;
}

// resident blocks per CU: 128x64 tiles (48 KB LDS) fit three, 128x128 tiles (64 KB) two; the
// generic fused epilogues need the registers of two (the specialised ones fit three)
// PREC 3 (B as three bf16 planes: 1.5x the B slab bytes) is also bounded by LDS: 128x128 tiles use
// exactly 80 KB (two per CU), 128x64 56 KB (two), 64x64 40 KB (four); PREC 5 (both operands as
// planes): 128x64 72 KB (two), 64x64 48 KB (three)
// 256 x 128 tiles (the KC x RC GEMMs on B planes, ESP_GEMM_WIDE_KCRC): 8 waves (two per SIMD in one block per
// CU), each wave the 64 x 64 of a 128 x 128 tile's wave, on the 2-slab ring
constexpr int glds_threads(int BMT) { return BMT == 256 ? 512 : NT; }
constexpr int glds_stage_bytes(int BNT, int BMT, int PREC) {
  return 4 * ((PREC == 5 ? 48 * BMT : BMT * GL_BK) + (PREC >= 3 ? 48 * BNT : BNT * GL_BK));
}
constexpr int glds_stages(int, int, int) { return GL_ST; }
constexpr int glds_lds_bytes(int BNT, int BMT, int PREC) {
  return glds_stages(BNT, BMT, PREC) * glds_stage_bytes(BNT, BMT, PREC) + (PREC >= 3 ? 0 : 16);
}
template <int BNT, int EPI, int BMT = BM, int PREC = 0>
constexpr int glds_occupancy() {
  // (256 x 128 tiles: 8 waves in one block per CU)
  constexpr int by_regs = BMT == 256 ? 1 : BMT == 64 ? 4 : (BNT == 64 && (EPI == EPI_PLAIN || EPI >= EPI_BIAS)) ? 3 : 2;
  constexpr int by_lds = 163840 / glds_lds_bytes(BNT, BMT, PREC);
  return by_regs < by_lds ? by_regs : by_lds;
}

// Persistent: block b processes tiles b, b+G, b+2G, ... as ONE continuous slab pipeline — the
// first slab of the next tile streams in during the last slab of the current one, and the
// current tile's epilogue stores drain while the next tile's MFMAs run (on this and the other
// resident blocks' waves).  With G = #tiles every block runs one tile (the classic launch).
//
// BF16 = true (esp_set_gemm_compute(1)): the same fp32 LDS-DMA pipeline, but each lane's 16
// staged k-values per tile row are rounded to bf16 in registers (v_cvt_pk_bf16_f32) and fed to
// two v_mfma_f32_32x32x16_bf16 per (i, j) tile pair instead of sixteen 32x32x2 f32 MFMAs: k-step
// 0 takes the lane's values s = 0..7 (k = 16h + s), step 1 s = 8..15, identically for A and B,
// so the two steps cover the slab's 32 k once.  The fused row sums stay fp32.
// PREC = 2 (esp_gemm_bf16): the operands are bf16 in HBM, viewed by the staging code as fp32
// arrays of bf16 PAIRS (K, ld and strides in pairs), so the LDS-DMA pipeline, the swizzle and
// the fragment reads are those of the fp32 path unchanged: a slab holds 64 bf16 k per row and
// a lane's 16 fetched "floats" are 32 bf16 k-values, fed as four bf16x8 operands to four
// v_mfma_f32_32x32x16_bf16 per (i, j) tile pair (k-step t takes values 8t..8t+7, identically
// for A and B, so the four steps cover the slab's 64 k once).  No conversion in the k-loop.
// BMT = 64 (with BNT = 64): 64 x 64 tiles, 2 x 2 waves of one 32 x 32 MFMA tile each, for the
// grids that 128-row tiles leave under-filled (decoder M ~ 5k tokens, 41-query source attention).
// fp32 operand split for the emulated fp32 MFMA (ESP_F32_SPLIT): v = hi + mid + lo exactly, each a
// bf16 (round-to-nearest-even at every step, so |mid| <= 2^-8 |v| and |lo| <= 2^-16 |v|; the two
// residuals are exact fp32 differences).
// Pairwise: one v_cvt_pk_bf16_f32 per part and pair, the parts' fp32 values taken back from the
// packed bits (<< 16, & 0xffff0000): 11 VALU per pair.
// (per element, hipcc converted each value twice: 12-13 VALU per pair; 1249.7 vs 1241.7 utt/s,
// profiles/r03i_abc_split_code.txt)
__device__ __forceinline__ void split3_bf16(const float* v, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
  uint32_t H[4], Md[4], L[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) esp::split3_pair(v[2 * p], v[2 * p + 1], H[p], Md[p], L[p]);
  hi = __builtin_bit_cast(bf16x8, make_uint4(H[0], H[1], H[2], H[3]));
  mid = __builtin_bit_cast(bf16x8, make_uint4(Md[0], Md[1], Md[2], Md[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(L[0], L[1], L[2], L[3]));
}


// The six split products of every (i, j) tile pair (smallest first: mid.mid, lo.hi, hi.lo, mid.hi, hi.mid,
// hi.hi), each pair's six MFMAs back to back (one accumulator chain at a time; the product-major order
// measured 0.6-0.7 % slower, r05l)
template <int TM, int TN>
__device__ __forceinline__ void mma6(f32x16 (&acc)[TM][TN], const bf16x8 (&ah)[TM][3], const bf16x8 (&bh)[TN][3]) {
  constexpr int PA[6] = {1, 2, 0, 1, 0, 0}, PB[6] = {1, 0, 2, 0, 1, 0};
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int p = 0; p < 6; ++p)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i][PA[p]], bh[j][PB[p]], acc[i][j], 0, 0, 0);
}

template <int MA, int MB, int BNT, bool RS, int EPI, int PREC = 0, int BMT = BM>
__global__ __launch_bounds__(glds_threads(BMT), (glds_occupancy<BNT, EPI, BMT, PREC>())) void gemm_glds_kernel(GemmArgs g, GldsArgs x) {
  constexpr int NTK = glds_threads(BMT), NW = NTK / 64, ST = glds_stages(BNT, BMT, PREC);
  constexpr int WN = BMT == 64 ? 2 : BNT / 64, WM = NW / WN, TM = BMT / (WM * 32), TN = BNT / (WN * 32);
  static_assert(BMT == 128 || (BMT == 64 && BNT == 64) || (BMT == 256 && BNT == 128 && PREC != 5),
                "64-row tiles are 64 wide; 256-row tiles: 128 wide");
  static_assert(PREC < 3 || MB == KC || MB == RC, "B planes: KC / RC operands");
  static_assert(PREC != 5 || MA == KC || MA == RC, "A planes: KC / RC operands");
  constexpr bool BP = PREC >= 3;                 // B as three bf16 planes (StageP)
  constexpr bool AP = PREC == 5;                 // A as three bf16 planes too: no split in the k-loop
  // the software-pipelined k-loop (k-step fragments one step ahead, the barrier between k-steps):
  // the fp32 split-product forms with A split in registers
  // (KC x RC only: measured at C2 B=256 the FFN input gradient 346 -> 305 us, the dgrad / P.V shapes
  // 1-1.3 % faster, while the RC x RC weight gradients and the conv2 GEMMs ran 3-8 % slower with it,
  // profiles/r05c_gemm_pipe_ab.txt)
  constexpr bool PIPE = ESP_GEMM_PIPE && ESP_F32_SPLIT && (PREC == 0 || PREC == 3) && MA == KC && MB == RC;
  struct FragA {
    float v[TM][8];
  };
  struct FragBf {
    float v[TN][8];
  };
  struct FragBp {
    bf16x8 v[TN][3];
  };
  using FragB = std::conditional_t<BP, FragBp, FragBf>;
  constexpr int PLF = BNT * 16;                  // floats per B plane image (BNT x 32 bf16)
  constexpr int PLA = BMT * 16;                  // floats per A plane image
  constexpr int A_SZ = AP ? 3 * PLA : BMT * GL_BK, B_SZ = BP ? 3 * PLF : BNT * GL_BK, BUF = A_SZ + B_SZ;
  constexpr int NIA = A_SZ / 4 / NTK, NIB = B_SZ / 4 / NTK;
  // + the split-K combine flag (the in-kernel combine is never used with B planes: their 128x128
  // tiles need exactly 80 KB for two blocks per CU)
  __shared__ __attribute__((aligned(16))) float smem[ST * BUF + (BP ? 0 : 4)];

  const int G = gridDim.x;
  int t = blockIdx.x;
  if (t >= x.ntiles) {
    if constexpr (EPI == EPI_C1FOLD) {  // a block without tiles: zero records (c1fold_reduce reads every block's)
      float* dst = g.c1_part + (long)blockIdx.x * C1NT * NTK * 10;
      for (int e = threadIdx.x; e < x.ntx * NTK * 10; e += NTK) dst[e] = 0.f;
    }
    return;
  }

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int h = lane >> 5, l32 = lane & 31;

  auto a_base = [&](const TileCoord& c) {
    const int z1 = (int)fdiv((uint32_t)c.z, x.fd_nb2), z2 = c.z - z1 * g.nb2;
    if constexpr (AP)  // bf16 element strides
      return reinterpret_cast<const float*>(reinterpret_cast<const __bf16*>(g.a.p) + z1 * g.a.s1 + z2 * g.a.s2);
    else
      return g.a.p + z1 * g.a.s1 + z2 * g.a.s2;
  };
  auto b_base = [&](const TileCoord& c) {
    const int z1 = (int)fdiv((uint32_t)c.z, x.fd_nb2), z2 = c.z - z1 * g.nb2;
    if constexpr (BP)  // bf16 element strides
      return reinterpret_cast<const float*>(reinterpret_cast<const __bf16*>(g.b.p) + z1 * g.b.s1 + z2 * g.b.s2);
    else
      return g.b.p + z1 * g.b.s1 + z2 * g.b.s2;
  };

  // scalar-base staging (StageS) for KC / RC / implicit-im2col A; the gathered operands keep
  // per-lane 64-bit addresses (Stage); B planes: StageP
  constexpr bool SA_S = MA == KC || MA == RC || MA == I2C_KC, SB_S = MB == KC || MB == RC;
  using SAt = std::conditional_t<AP, StageP<MA, BMT, NW>,
                                 std::conditional_t<SA_S, StageS<MA, BMT, NIA, PREC == 2, NW>, Stage<MA, BMT, NIA, false, NW>>>;
  using SBt = std::conditional_t<BP, StageP<MB, BNT, NW>,
                                 std::conditional_t<SB_S, StageS<MB, BNT, NIB, PREC == 2, NW>,
                                                    Stage<MB, BNT, NIB, PREC == 2 && MB == I2C_RC, NW>>>;
  SAt sa;
  SBt sb;
  auto init_ab = [&](const TileCoord& cc) {
    if constexpr (AP) sa.init(g.a, a_base(cc), g.M, cc.m0, cc.kbeg, wave, lane);
    else if constexpr (SA_S) sa.init(g.a, a_base(cc), g.M, g.K, cc.m0, cc.kbeg, x.hw_a, x.wo_a, wave, lane);
    else sa.init(g.a, a_base(cc), g.M, g.K, cc.m0, x.c_a, x.hw_a, x.wo_a, wave, lane, MA == I2CT_KC ? &x : nullptr);
    if constexpr (BP) sb.init(g.b, b_base(cc), g.N, cc.n0, cc.kbeg, wave, lane);
    else if constexpr (SB_S) sb.init(g.b, b_base(cc), g.N, g.K, cc.n0, cc.kbeg, x.hw_b, x.wo_b, wave, lane);
    else sb.init(g.b, b_base(cc), g.N, g.K, cc.n0, x.c_b, x.hw_b, x.wo_b, wave, lane);
  };
  const uint32_t smem_lds = lds_addr(smem);
  auto issue_ab = [&](int k0, float* dst) {
    const uint32_t dl = smem_lds + (uint32_t)(dst - smem) * 4u;
    if constexpr (AP) sa.issue(g.K, k0, dl, wave);
    else if constexpr (SA_S) sa.issue(g.a, g.K, k0, dl, wave);
    else sa.issue(g.a, g.K, k0, dst, wave, x.c_a, x.hw_a, x.wo_a, MA == I2CT_KC ? &x : nullptr);
    if constexpr (BP) sb.issue(g.K, k0, dl + 4u * A_SZ, wave);
    else if constexpr (SB_S) sb.issue(g.b, g.K, k0, dl + 4u * A_SZ, wave);
    else sb.issue(g.b, g.K, k0, dst + A_SZ, wave, x.c_b, x.hw_b, x.wo_b);
  };

  TileCoord c = tile_coord<BNT, BMT>(g, x, t, G);
  init_ab(c);
  issue_ab(c.kbeg, smem);
  wait_vm0();
  raw_barrier();
  int buf = 0;

  // EPI_C1FOLD: this wave's conv1-gradient sums over its tiles of one column tile tn (store_c1fold), written
  // (first time) or added (the block returns to tn) to its record when the column tile changes, and at the end
  constexpr int C1K = EPI == EPI_C1FOLD ? 5 * TN : 1;
  float c1k[C1K];
  int c1tn = -1;
  bool c1seen[C1NT] = {false, false, false, false};
  auto c1rec = [&](int tn) { return g.c1_part + ((((long)blockIdx.x * C1NT + tn) * NW + wave) * 64 + lane) * 10; };
  auto c1flush = [&]() {
    if constexpr (EPI == EPI_C1FOLD) {
      if (c1tn < 0) return;
      float* dst = c1rec(c1tn);
#pragma unroll
      for (int u = 0; u < C1K; ++u) {
        dst[u] = c1seen[c1tn] ? dst[u] + c1k[u] : c1k[u];
        c1k[u] = 0.f;
      }
      c1seen[c1tn] = true;
    }
  };
#pragma unroll
  for (int u = 0; u < C1K; ++u) c1k[u] = 0.f;

  for (;;) {
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // fused bias gradient (A = dy in RC mode): the first column tile's wn==0 waves sum their A
    // fragments over k; halves combined and splits reduced in fixed order (deterministic)
    const bool do_rs = RS && c.tn == 0 && wn == 0;
    float rs[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) rs[i] = 0.f;
    const int tnext = t + G;
    const bool has_next = tnext < x.ntiles;
    TileCoord cn = c;

    // frags + MFMAs of one staged slab (and the fused row sums)
    // kv < GL_BK (the last slab of a K range that is not a multiple of 32): the A fragment's
    // k >= kv values are zeroed in registers (B's staged tail holds finite clamped elements), so
    // no LDS zero pass and no extra barrier
    auto compute = [&](const float* cur, int kv) {
      if constexpr (PREC == 2) {
        // fragments as 4 chunks of 8 bf16 per tile (k = 32h + 8t + 0..7 for chunk t)
        float4 a4[TM][4], b4[TN][4];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if constexpr (MA == RC) {
            frag_tr16<BMT>(cur, wm * TM * 32 + i * 32, lane, a4[i]);
          } else {
            float f[16];
            frag16<MA, BMT>(cur, wm * TM * 32 + i * 32 + l32, h, f);
#pragma unroll
            for (int t = 0; t < 4; ++t) a4[i][t] = make_float4(f[4 * t], f[4 * t + 1], f[4 * t + 2], f[4 * t + 3]);
          }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (MB == RC || MB == I2C_RC) {
            frag_tr16<BNT>(cur + A_SZ, wn * TN * 32 + j * 32, lane, b4[j]);
          } else {
            float f[16];
            frag16<MB, BNT>(cur + A_SZ, wn * TN * 32 + j * 32 + l32, h, f);
#pragma unroll
            for (int t = 0; t < 4; ++t) b4[j][t] = make_float4(f[4 * t], f[4 * t + 1], f[4 * t + 2], f[4 * t + 3]);
          }
        }
        if (kv < GL_BK) {  // K tail (kv pairs): zero A's pairs at pair index >= kv
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const int k0p = 16 * h + 4 * t;  // pair index of the chunk's first value
              a4[i][t].x = k0p + 0 < kv ? a4[i][t].x : 0.f;
              a4[i][t].y = k0p + 1 < kv ? a4[i][t].y : 0.f;
              a4[i][t].z = k0p + 2 < kv ? a4[i][t].z : 0.f;
              a4[i][t].w = k0p + 3 < kv ? a4[i][t].w : 0.f;
            }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a4[i][t]),
                                                                  __builtin_bit_cast(bf16x8, b4[j][t]), acc[i][j], 0, 0, 0);
        if constexpr (RS) {  // fused bias gradient over the bf16 A values (torch AMP's bf16 dy sum)
          if (do_rs) {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              float a0 = 0.f;
#pragma unroll
              for (int t = 0; t < 4; ++t) {
                const float w[4] = {a4[i][t].x, a4[i][t].y, a4[i][t].z, a4[i][t].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const uint32_t u = __float_as_uint(w[e]);
                  a0 += __uint_as_float(u << 16) + __uint_as_float(u & 0xffff0000u);
                }
              }
              rs[i] += a0;
            }
          }
        }
        return;
      }
      if constexpr (AP) {
        // both operands' three planes read from LDS: the PREC 0 products in the PREC 0 order on the
        // same values, and no split VALU at all
        const float* bpl = cur + A_SZ;
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
          bf16x8 ah[TM][3], bh[TN][3];
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              if constexpr (MA == KC) ah[i][p] = frag_pl_kc(cur + p * PLA, wm * TM * 32 + i * 32 + l32, h, hs);
              else ah[i][p] = frag_pl_rc<BMT>(cur + p * PLA, wm * TM * 32 + i * 32, lane, hs);
            }
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              if constexpr (MB == KC) bh[j][p] = frag_pl_kc(bpl + p * PLF, wn * TN * 32 + j * 32 + l32, h, hs);
              else bh[j][p] = frag_pl_rc<BNT>(bpl + p * PLF, wn * TN * 32 + j * 32, lane, hs);
            }
          if (kv < GL_BK) {  // K tail: A's k >= kv are 0 (B's clamped tail holds finite values)
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (16 * h + 8 * hs + e >= kv)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                  for (int p = 0; p < 3; ++p) ah[i][p][e] = (__bf16)0.0f;
          }
          mma6<TM, TN>(acc, ah, bh);
          if constexpr (RS) {  // fused bias gradient: the fp32 A values are hi + mid + lo exactly
            if (do_rs) {
#pragma unroll
              for (int i = 0; i < TM; ++i) {
                float a0 = 0.f;
#pragma unroll
                for (int e = 0; e < 8; ++e)
                  a0 += ((float)ah[i][0][e] + (float)ah[i][1][e]) + (float)ah[i][2][e];
                rs[i] += a0;
              }
            }
          }
        }
        return;
      }
      if constexpr (BP) {
        // A split in registers (as PREC 0), B's three planes read from LDS: the PREC 0 products in
        // the PREC 0 order on the same values
        float af[TM][16];
#pragma unroll
        for (int i = 0; i < TM; ++i) frag16<MA, BMT>(cur, wm * TM * 32 + i * 32 + l32, h, af[i]);
        if (kv < GL_BK) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int s2 = 0; s2 < 16; ++s2) af[i][s2] = 16 * h + s2 < kv ? af[i][s2] : 0.f;
        }
        const float* bpl = cur + A_SZ;
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
          bf16x8 ah[TM][3], bh[TN][3];
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              if constexpr (MB == KC) bh[j][p] = frag_pl_kc(bpl + p * PLF, wn * TN * 32 + j * 32 + l32, h, hs);
              else bh[j][p] = frag_pl_rc<BNT>(bpl + p * PLF, wn * TN * 32 + j * 32, lane, hs);
            }
#pragma unroll
          for (int i = 0; i < TM; ++i) split3_bf16(&af[i][8 * hs], ah[i][0], ah[i][1], ah[i][2]);
          mma6<TM, TN>(acc, ah, bh);
        }
        if constexpr (RS) {
          if (do_rs) {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              float a0 = 0.f;
#pragma unroll
              for (int s = 0; s < 16; ++s) a0 += af[i][s];
              rs[i] += a0;
            }
          }
        }
        return;
      }
      float af[TM][16], bf[TN][16];
#pragma unroll
      for (int i = 0; i < TM; ++i) frag16<MA, BMT>(cur, wm * TM * 32 + i * 32 + l32, h, af[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) frag16<MB, BNT>(cur + A_SZ, wn * TN * 32 + j * 32 + l32, h, bf[j]);
      if (kv < GL_BK) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int s2 = 0; s2 < 16; ++s2) af[i][s2] = 16 * h + s2 < kv ? af[i][s2] : 0.f;
      }
      if constexpr (PREC == 1) {
        bf16x8 ah[TM][2], bh[TN][2];
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int e = 0; e < 8; ++e) ah[i][hs][e] = (__bf16)af[i][8 * hs + e];
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 8; ++e) bh[j][hs][e] = (__bf16)bf[j][8 * hs + e];
        }
#pragma unroll
        for (int hs = 0; hs < 2; ++hs)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i][hs], bh[j][hs], acc[i][j], 0, 0, 0);
      } else if constexpr (PREC == 0 && ESP_F32_SPLIT) {
        // fp32 product emulated on the bf16 MFMA: the six split products down to 2^-16 relative
        // (hi.hi, hi.mid, mid.hi, hi.lo, lo.hi, mid.mid), smallest first into the fp32 accumulator;
        // the dropped mid.lo + lo.mid + lo.lo are <= 2^-23 of |a b| (k order as in PREC 1)
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
          bf16x8 ah[TM][3], bh[TN][3];
#pragma unroll
          for (int i = 0; i < TM; ++i) split3_bf16(&af[i][8 * hs], ah[i][0], ah[i][1], ah[i][2]);
#pragma unroll
          for (int j = 0; j < TN; ++j) split3_bf16(&bf[j][8 * hs], bh[j][0], bh[j][1], bh[j][2]);
          mma6<TM, TN>(acc, ah, bh);
        }
      } else {
#pragma unroll
        for (int s = 0; s < 16; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
      }
      if constexpr (RS) {
        if (do_rs) {  // after the MFMAs were issued: the adds ride in their shadow
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            float a0 = 0.f;
#pragma unroll
            for (int s = 0; s < 16; ++s) a0 += af[i][s];
            rs[i] += a0;
          }
        }
      }
    };
    // one k-step (hs) of the fp32 split products: A's 8 values per tile row, B's 8 values (PREC 0) or
    // its three planes (PREC 3)
    auto load_half = [&](const float* cur, int hs, FragA& a, FragB& b) {
      if constexpr (PIPE) {
#pragma unroll
        for (int i = 0; i < TM; ++i) frag8<MA, BMT>(cur, wm * TM * 32 + i * 32 + l32, h, hs, a.v[i]);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (BP) {
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              if constexpr (MB == KC) b.v[j][p] = frag_pl_kc(cur + A_SZ + p * PLF, wn * TN * 32 + j * 32 + l32, h, hs);
              else b.v[j][p] = frag_pl_rc<BNT>(cur + A_SZ + p * PLF, wn * TN * 32 + j * 32, lane, hs);
            }
          } else {
            frag8<MB, BNT>(cur + A_SZ, wn * TN * 32 + j * 32 + l32, h, hs, b.v[j]);
          }
        }
      }
    };
    auto mma_half = [&](int hs, int kv, FragA& a, FragB& b) {
      if constexpr (PIPE) {
        if (kv < GL_BK) {  // K tail: A's k >= kv are 0 (B's clamped tail holds finite values)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int e = 0; e < 8; ++e) a.v[i][e] = 16 * h + 8 * hs + e < kv ? a.v[i][e] : 0.f;
        }
        bf16x8 ah[TM][3], bh[TN][3];
#pragma unroll
        for (int i = 0; i < TM; ++i) split3_bf16(a.v[i], ah[i][0], ah[i][1], ah[i][2]);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (BP) {
#pragma unroll
            for (int p = 0; p < 3; ++p) bh[j][p] = b.v[j][p];
          } else {
            split3_bf16(b.v[j], bh[j][0], bh[j][1], bh[j][2]);
          }
        }
        mma6<TM, TN>(acc, ah, bh);
        if constexpr (RS) {
          if (do_rs) {  // after the MFMAs were issued: the adds ride in their shadow
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              float a0 = 0.f;
#pragma unroll
              for (int e = 0; e < 8; ++e) a0 += a.v[i][e];
              rs[i] += a0;
            }
          }
        }
      }
    };
    auto finish_slab = [&]() {
      wait_vm0();     // this wave's DMA of the next slab has landed
      wait_lgkm0();   // this wave's reads of this slab are done
      raw_barrier();  // -> everyone's: next slab readable, this buffer free for the one after
      buf ^= 1;
    };

    if constexpr (PIPE) {
      // fp32 split products (PREC 0 / 3), software-pipelined by k-step: the fragments of k-step hs+1
      // are read while the MFMAs of k-step hs issue, and the slab barrier sits BETWEEN a slab's two
      // k-steps -- after it the wave issues k-step 1's MFMAs (operands already in registers) while
      // the next slab's first fragments are read, instead of waiting out a fragment read + split
      // after every barrier.  The fragments of k-step 1 are read before the barrier (that buffer is
      // re-filled right after it); the MFMAs, their order and the fused row sums are those of compute().
      FragA Fa, Ga;
      FragB Fb, Gb;
      load_half(smem + buf * BUF, 0, Fa, Fb);
      for (int kt = 0; kt < c.nk; ++kt) {
        float* cur = smem + buf * BUF;
        float* nxt = smem + (buf ^ 1) * BUF;  // last read before the previous barrier
        const bool last = kt + 1 == c.nk;
        if (!last) {
          issue_ab(c.kbeg + (kt + 1) * GL_BK, nxt);
        } else if (has_next) {  // the next tile's first slab streams in (this tile's stages are done)
          cn = tile_coord<BNT, BMT>(g, x, tnext, G);
          init_ab(cn);
          issue_ab(cn.kbeg, nxt);
        }
        const int kv = last ? c.kend - (c.kbeg + kt * GL_BK) : GL_BK;
        load_half(cur, 1, Ga, Gb);
        mma_half(0, kv, Fa, Fb);
        finish_slab();
        if (!last) load_half(smem + buf * BUF, 0, Fa, Fb);
        mma_half(1, kv, Ga, Gb);
      }
    } else {
      for (int kt = 0; kt + 1 < c.nk; ++kt) {  // all but the last slab: slab kt+1 streams in
        const int k1 = c.kbeg + (kt + 1) * GL_BK;
        float* nxt = smem + (buf ^ 1) * BUF;  // last read before the previous barrier
        issue_ab(k1, nxt);
        compute(smem + buf * BUF, GL_BK);
        finish_slab();
      }
      {  // last slab: the next tile's first slab streams in (this tile's stages are done)
        float* cur = smem + buf * BUF;
        float* nxt = smem + (buf ^ 1) * BUF;
        if (has_next) {
          cn = tile_coord<BNT, BMT>(g, x, tnext, G);
          init_ab(cn);
          issue_ab(cn.kbeg, nxt);
        }
        compute(cur, c.kend - (c.kbeg + (c.nk - 1) * GL_BK));
        finish_slab();
      }
    }
    // epilogue: fire-and-forget stores that drain under the next tile's first slab
    if (RS && do_rs) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float v = rs[i] + __shfl_xor(rs[i], 32, 64);  // k halves 0-15 / 16-31 of every slab
        const int m = c.m0 + wm * TM * 32 + i * 32 + l32;
        if (h == 0 && m < g.M) {
          if (g.splits > 1) __hip_atomic_store(g.rs_work + (long)c.split * g.M + m, v, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);  // write-through (combine hand-off)
          else g.rowsum[m] += v;
        }
      }
    }
    if (!BP && g.tickets) {  // in-kernel split-K: write-through partial tile, ticket, last unit combines
      float* Wz = g.work + ((long)c.split * g.batch + c.z) * ((long)g.sk_mp * g.sk_np);
      store_cols<EPI_P0, TM, TN, true, 16>(g, 0, g.sk_np, c.m0 + wm * TM * 32, c.n0 + wn * TN * 32, lane, acc, Wz);
      splitk_combine<BMT, BNT>(g, c.z, c.m0 / BMT, c.tn, x.ntx, x.nty, reinterpret_cast<int*>(smem + ST * BUF));
    } else {
      float* W = g.splits > 1 ? g.work + ((long)c.split * g.batch + c.z) * (long)g.M * g.N : nullptr;
      if constexpr (EPI == EPI_C1FOLD) {
        if (c.tn != c1tn) {
          c1flush();
          c1tn = c.tn;
        }
        if constexpr (TM == 2 && TN == 2) store_c1fold<TM, TN>(g, c.m0 + wm * TM * 32, c.n0 + wn * TN * 32, lane, acc, c1k);
      } else if constexpr (EPI >= EPI_BIAS) {  // specialised kinds: never split-K, always wide
        const int mr0 = c.m0 + wm * TM * 32, nc0 = c.n0 + wn * TN * 32;
        if (col_epi_ok<EPI>() && mr0 + TM * 32 <= g.M && nc0 + TN * 32 <= g.N) {
          const long cb = c_base(g, c.z);
          if (g.alpha == 1.0f) store_cols<EPI, TM, TN, true>(g, cb, g.ldc, mr0, nc0, lane, acc, g.c);
          else store_cols<EPI, TM, TN, false>(g, cb, g.ldc, mr0, nc0, lane, acc, g.c);
        } else {
          store_spec_tiles<EPI, TM, TN>(g, c.z, mr0, nc0, lane, acc);
        }
      } else if (g.wide) {
        if (W && c.m0 + wm * TM * 32 + TM * 32 <= g.M && c.n0 + wn * TN * 32 + TN * 32 <= g.N)
          store_cols<EPI_P0, TM, TN, true>(g, 0, g.N, c.m0 + wm * TM * 32, c.n0 + wn * TN * 32, lane, acc, W);
        else if (W) store_partials_wide<TM, TN>(g, W, c.m0 + wm * TM * 32, c.n0 + wn * TN * 32, lane, acc);
        else store_tiles_wide<EPI, TM, TN>(g, c.z, c.m0 + wm * TM * 32, c.n0 + wn * TN * 32, lane, acc, false);
      } else {
        if (W) store_partials<TM, TN>(g, W, c.m0 + wm * TM * 32, c.n0 + wn * TN * 32, h, l32, acc);
        else store_tiles<EPI, TM, TN>(g, c.z, c.m0 + wm * TM * 32, c.n0 + wn * TN * 32, h, l32, acc);
      }
    }
    if (!has_next) break;
    t = tnext;
    c = cn;
  }
  if constexpr (EPI == EPI_C1FOLD) {
    c1flush();
#pragma unroll
    for (int tn = 0; tn < C1NT; ++tn)
      if (tn < x.ntx && !c1seen[tn]) {
        float* dst = c1rec(tn);
#pragma unroll
        for (int u = 0; u < 10; ++u) dst[u] = 0.f;
      }
  }
}


// Map run-time (mode_a, mode_b, tile width, precision) onto compile-time constants for the mode
// pairs the host issues; calls f(MA, MB, BNT, PREC) with std::integral_constant arguments.
// false: no such instantiation.
template <int V>
using IC = std::integral_constant<int, V>;
// bm = 64 (64 x 64 tiles) exists for bnt = 64, KC / RC operand pairs and prec 0 / 1 only;
// prec 2 (bf16 operands) for the KC / RC pairs and I2C_KC x KC / I2CT_KC x RC with 128-row tiles.
template <class F>
bool glds_switch(int ma, int mb, int bnt, int prec, int bm, F&& f) {
  auto tile = [&](auto A, auto B) {
    if (bnt != 64 && bnt != 128) return false;
    constexpr bool small_ok = (decltype(A)::value == KC || decltype(A)::value == RC) &&
                              (decltype(B)::value == KC || decltype(B)::value == RC);
    // B planes (prec 3): the weight-B pairs (linear forward / input gradient, conv2 forward / input
    // gradient) and RC x RC (weight gradients)
    constexpr int MA_ = decltype(A)::value, MB_ = decltype(B)::value;
    constexpr bool planes_ok = (MB_ == KC && (MA_ == KC || MA_ == I2C_KC)) ||
                               (MB_ == RC && (MA_ == KC || MA_ == RC || MA_ == I2CT_KC));
    auto by_prec = [&](auto N, auto R) {
      if (prec == 0) {
        f(A, B, N, IC<0>{}, R);
      } else if (prec == 1) {
        f(A, B, N, IC<1>{}, R);
      } else if (prec == 3) {
        if constexpr (planes_ok) f(A, B, N, IC<3>{}, R);
        else return false;
      } else if (prec == 5) {  // both operands as planes: KC / RC pairs, 64-wide tiles (LDS)
        if constexpr (small_ok && decltype(N)::value == 64) f(A, B, N, IC<5>{}, R);
        else return false;
      } else if constexpr ((small_ok || (MA_ == I2C_KC && MB_ == KC) || (MA_ == I2CT_KC && MB_ == RC) ||
                            (MA_ == RC && MB_ == I2C_RC)) &&
                           decltype(R)::value == BM) {
        // bf16 operands: KC / RC pairs, and the conv2 forward / input gradient (implicit-im2col A of
        // bf16 pairs: the gathers run in pair units, C % 64 == 0) / weight gradient (gathered bf16 B)
        f(A, B, N, IC<2>{}, R);
      } else {
        return false;
      }
      return true;
    };
    if (bm == 64) {
      if constexpr (small_ok) {
        if (bnt == 64 && prec != 2) return by_prec(IC<64>{}, IC<64>{});  // (prec 5: A planes of 64 rows)
      }
      return false;
    }
    if (bm == 256) {  // 256 x 128 tiles, 8 waves: KC x RC on B planes (ESP_GEMM_WIDE_KCRC)
      if constexpr (ESP_GEMM_WIDE_KCRC && MA_ == KC && MB_ == RC) {
        if (bnt == 128 && prec == 3) return by_prec(IC<128>{}, IC<256>{});
      }
      return false;
    }
    return bnt == 64 ? by_prec(IC<64>{}, IC<BM>{}) : by_prec(IC<128>{}, IC<BM>{});
  };
  switch (ma * 8 + mb) {
    case KC * 8 + KC: return tile(IC<KC>{}, IC<KC>{});
    case KC * 8 + RC: return tile(IC<KC>{}, IC<RC>{});
    case RC * 8 + KC: return tile(IC<RC>{}, IC<KC>{});
    case RC * 8 + RC: return tile(IC<RC>{}, IC<RC>{});
    case I2C_KC * 8 + KC: return tile(IC<I2C_KC>{}, IC<KC>{});
    case RC * 8 + I2C_RC: return tile(IC<RC>{}, IC<I2C_RC>{});
    case I2CT_KC * 8 + RC: return tile(IC<I2CT_KC>{}, IC<RC>{});
    default: return false;
  }
}

// Launchers of gemm_glds_kernel, one translation unit per epilogue family; false when the
// (mode pair, kind) has no instantiation.
//   gemm_glds_plain.hip : EPI_PLAIN (rs: fused row sums, RC-mode A only)
//   gemm_glds_epi.hip   : generic EPI_FWD / EPI_BWD
//   gemm_glds_spec.hip  : specialised kinds (EPI_BIAS .. EPI_BMUL)
//   gemm_glds_pspec.hip : specialised plain kinds (EPI_P0, EPI_PR)
// (bm = the tile height, g.bm)
bool glds_launch_plain(int ma, int mb, int bnt, int prec, bool rs, dim3 grid, hipStream_t st, const GemmArgs& g,
                       const GldsArgs& x);
bool glds_launch_epi(int ma, int mb, int bnt, int prec, int epi, dim3 grid, hipStream_t st, const GemmArgs& g,
                     const GldsArgs& x);
bool glds_launch_spec(int ma, int mb, int bnt, int prec, int epi, dim3 grid, hipStream_t st, const GemmArgs& g,
                      const GldsArgs& x);
bool glds_launch_pspec(int ma, int mb, int bnt, int prec, int epi, dim3 grid, hipStream_t st, const GemmArgs& g,
                       const GldsArgs& x);
// resident blocks per CU of a launch (host side)
inline int glds_occupancy_rt(int bnt, int epi, int bm, int prec) {
  const int by_regs = bm == 256 ? 1 : bm == 64 ? 4 : (bnt == 64 && (epi == EPI_PLAIN || epi >= EPI_BIAS)) ? 3 : 2;
  const int by_lds = 163840 / glds_lds_bytes(bnt, bm == 64 || bm == 256 ? bm : BM, prec);
  return std::min(by_regs, by_lds);
}

}  // namespace espg
