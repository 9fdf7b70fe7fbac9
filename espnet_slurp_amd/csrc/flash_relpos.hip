// Flash-style relative-position self-attention (latest and legacy rel_shift), d_k = 64, fp32
// MFMA (v_mfma_f32_32x32x2_f32: exact f32 fma chains, so recomputed scores are bit-identical).
//
//   s[i][j] = (q_u[i].k[j] + bd[i][j]) / sqrt(d_k),  key mask j < klen[b],  P = softmax_j(s),
//   P_drop = dropout(P),  ctx = P_drop v                            (attention.py:64-96, 240-263)
//   latest  bd[i][j] = q_v[i].p[T-1-i+j]                                      (attention.py:240-263)
//   legacy  bd[i][j] = j <= i ? q_v[i].p[T-1-i+j] : j == i+1 ? 0 : q_v[i+1].p[j-i-2]   (:145-165)
//
// Legacy as latest: with the virtual table p_virt = [p; p[0:T-1]] (2T-1 rows, row x is p[x] or
// p[x-T]) both cases read  q_v[rho].p_virt[T-1-rho+j]  with rho = i (j <= i) or rho = i+1
// (j >= i+2), so ONE band window per 32-row block serves both (legacy needs q_v row i0+32 too).
//
// Forward (one block per (z = h*nb + b, 32 query rows)): scores are computed TRANSPOSED,
// S^T = K Q_u^T, so a lane holds one query and its registers hold keys: the row softmax is an
// in-lane reduction (+ one lane-half exchange + a 4-wave LDS exchange), and P^T in registers is
// exactly the A operand of ctx = P_drop V (an MFMA accumulator consumed as the next MFMA's
// operand without data movement).  Only ctx (B*T x D) and two floats per row (max, 1/sum) reach
// HBM: no (Z, T, T) probability tensor in the forward.
//
// Backward (one block per (z, 32 query rows)): the band window and the scores are recomputed
// (non-transposed: keys on lanes), P from the saved row statistics (bit-identical to the
// forward's), dP_drop = dctx V^T on the MFMA, dS = P (dP - D_i) / sqrt(d_k) with
// D_i = dctx_i . ctx_i.  In-kernel: dq = dS K + Dbd p_win (the band image of dS read with a
// per-row shift from LDS), the pos_bias_u / pos_bias_v column-sum partials and, for legacy,
// the carry of the block's last row into q_v row i0+32.  dS and P_drop (pitch lds) go to HBM
// for the key-side products dK = dS^T q_u and dV = P_drop^T dctx (batched GEMMs, K = T), and
// for the linear_pos gradient dp = sum_{b,i} dbd^T q_v, computed by relpos_dp_kernel straight
// from dS with skewed (diagonal) reads — the (Z, T, 2T-1) dbd tensor is never materialised.
#include <stdlib.h>

#include "common.h"

namespace {

constexpr int FR = 32, FDK = 64;

struct FlashArgs {
  const float *qu, *qv;          // (Z, T, 64) head-major, z = h*nb + b
  const float *kmat, *vmat;      // k / v rows at +(b*T + j)*ldk (ldv) + 64*head
  const float* pm;               // p rows at +row*ldpm + 64*head (latest 2T-1 rows, legacy T)
  const float *ctx, *dctx;       // (B*T, ldc) rows, head slice at 64*head (bwd)
  long ldk, ldv, ldpm, ldc;
  const int* klen;
  float* out;                    // fwd: ctx (pitch ldc); bwd: dq (pitch ldq)
  long ldq;
  float* stats;                  // (Z, T, 2): row max, 1/row sum
  float *dS, *pdrop;             // bwd: (Z, T, lds)
  long lds;
  float* bias_part;              // bwd: (Z, nqb, 2, 64) column sums of dq_u, dq_v
  float* carry;                  // bwd legacy: (Z, nqb, 64)
  int nb, T, WP, nqb, nblk, DSP;
  int band_sz;                   // bwd: floats of the band / partials region (ds follows it)
  float sqrt_dk, dscale;
  float inv_sqrt_dk;             // 1/sqrt(d_k) = 1/8 exactly for d_k = 64: x * inv == x / sqrt(d_k)
  uint32_t thr;
  uint64_t seed;
  const uint64_t* key;
};

__device__ __forceinline__ int il_of(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

// 64 d-values of a row in MFMA k-order: f[c][s] = row[32c + 16hf + s]
__device__ __forceinline__ void load_row64(const float* row, int hf, float (&f)[2][16]) {
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 v = *reinterpret_cast<const float4*>(row + 32 * c + 16 * hf + 4 * u);
      f[c][4 * u] = v.x; f[c][4 * u + 1] = v.y; f[c][4 * u + 2] = v.z; f[c][4 * u + 3] = v.w;
    }
}
// C(32x32) = sum_d A[lane row][d] B[lane row][d] over the 64 d of two row fragments
__device__ __forceinline__ f32x16 mfma_rows(const float (&a)[2][16], const float (&b)[2][16]) {
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int st = 0; st < 16; ++st) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c][st], b[c][st], acc, 0, 0, 0);
  return acc;
}

template <int REL>
__device__ __forceinline__ const float* p_virt_row(const FlashArgs& a, int x, int head) {
  const int P = REL == 2 ? a.T : 2 * a.T - 1;
  x = min(max(x, 0), 2 * a.T - 2);
  if (REL == 2 && x >= a.T) x -= a.T;
  x = min(x, P - 1);
  return a.pm + (long)x * a.ldpm + FDK * head;
}

// block -> (z, query block) with the nqb blocks of one z on one XCD (they share its k, v, p rows
// in that XCD's L2): blocks are dealt round-robin over the 8 XCDs; bijective for any count
__device__ __forceinline__ void block_task(const FlashArgs& a, int& z, int& qb) {
  const int bid = blockIdx.x, n = a.nblk;
  const int xcd = bid & 7, per = n >> 3, rem = n & 7;
  const int task = (xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per) + (bid >> 3);
  z = task / a.nqb;
  qb = task - z * a.nqb;
}

// Band window  Sbd[r][c] = q_v[i0 + r] . p_virt[kmin + c],  kmin = T - 32 - i0,  c < nbd*32,
// rows r < 32 on the MFMA (tiles dealt over the 4 waves), legacy row 32 on the VALU.
template <int REL>
__device__ __forceinline__ void band_window(const FlashArgs& a, float* sbd, int z, int head, int i0, int wave,
                                            int lane) {
  const int T = a.T, hf = lane >> 5, l32 = lane & 31;
  const int kmin = T - FR - i0;
  const int nbd = (T + FR - 1 + 31) / 32;
  float aq[2][16];
  load_row64(a.qv + ((long)z * T + min(i0 + l32, T - 1)) * FDK, hf, aq);
  for (int ct = wave; ct < nbd; ct += 4) {
    float bq[2][16];
    load_row64(p_virt_row<REL>(a, kmin + ct * 32 + l32, head), hf, bq);
    const f32x16 acc = mfma_rows(aq, bq);
#pragma unroll
    for (int r = 0; r < 16; ++r) sbd[il_of(r, hf) * a.WP + ct * 32 + l32] = acc[r];
  }
  if (REL == 2 && i0 + FR < T) {  // q_v row i0+32: only its j >= i0+33 part is read (row 31's upper triangle)
    const float* q = a.qv + ((long)z * T + i0 + FR) * FDK;
    for (int c = threadIdx.x; c < nbd * 32; c += blockDim.x) {
      const float* pr = p_virt_row<REL>(a, kmin + c, head);
      float s = 0.f;
#pragma unroll 16
      for (int d = 0; d < FDK; d += 4) {
        const float4 pv = *reinterpret_cast<const float4*>(pr + d);
        const float4 qq = *reinterpret_cast<const float4*>(q + d);
        s += qq.x * pv.x + qq.y * pv.y + qq.z * pv.z + qq.w * pv.w;
      }
      sbd[FR * a.WP + c] = s;
    }
  }
}

// rel_shift gather of the band for (query i = i0 + rr, key j): own row rr, or row rr+1 (legacy
// upper triangle), zero at legacy j == i+1
template <int REL>
__device__ __forceinline__ float band_at(const float* sbd, int WP, int rr, int i, int j) {
  if (REL == 1 || j <= i) return sbd[rr * WP + j - rr + 31];
  if (j == i + 1) return 0.f;
  return sbd[(rr + 1) * WP + j - rr + 30];
}

// ============================================================================ forward
template <int REL, int NTA>
__global__ __launch_bounds__(256, 2) void relpos_flash_fwd_kernel(FlashArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sbd = smem;                           // band window [32(+1)][WP], later ctx partials [4][32][68]
  float* red = smem + a.DSP;                   // [2][4][32] row max / sum exchange (DSP = region size here)
  int z, qb;
  block_task(a, z, qb);
  const int T = a.T, i0 = qb * FR;
  const int head = z / a.nb, b = z - head * a.nb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hf = lane >> 5, l32 = lane & 31;
  const int nac = (T + 31) / 32;
  const uint64_t seed = esp::keyed(a.seed, a.key);

  band_window<REL>(a, sbd, z, head, i0, wave, lane);
  int kl = a.klen ? a.klen[b] : T;
  kl = min(kl, T);
  float bq[2][16];  // q_u row of this lane's query (B operand of every S^T tile)
  load_row64(a.qu + ((long)z * T + min(i0 + l32, T - 1)) * FDK, hf, bq);
  __syncthreads();

  // S^T tiles: key rows on registers (il), query on the lane
  const int i = i0 + l32;
  f32x16 sc[NTA];
  float kf[2][16];  // k rows of the current tile; the next tile's are requested after its MFMAs
  if (wave < nac) load_row64(a.kmat + ((long)b * T + min(wave * 32 + l32, T - 1)) * a.ldk + FDK * head, hf, kf);
#pragma unroll
  for (int t = 0; t < NTA; ++t) {
    const int ct = wave + 4 * t;
    if (ct < nac) {
      const f32x16 acc = mfma_rows(kf, bq);
      if (t + 1 < NTA && ct + 4 < nac)
        load_row64(a.kmat + ((long)b * T + min((ct + 4) * 32 + l32, T - 1)) * a.ldk + FDK * head, hf, kf);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = ct * 32 + il_of(r, hf);
        sc[t][r] = j < kl ? (acc[r] + band_at<REL>(sbd, a.WP, l32, i, j)) * a.inv_sqrt_dk : -INFINITY;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[t][r] = -INFINITY;
    }
  }
  // v rows of the first tile fly during the softmax reductions
  float vv[2][16];
  auto load_v = [&](int ct) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float* vr = a.vmat + ((long)b * T + min(ct * 32 + il_of(r, hf), T - 1)) * a.ldv + FDK * head + l32;
      vv[0][r] = vr[0];
      vv[1][r] = vr[32];
    }
  };
  if (wave < nac) load_v(wave);
  // row softmax of query i: in-lane over (t, r), across the lane halves, across the 4 waves
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < NTA; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) m = fmaxf(m, sc[t][r]);
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  if (hf == 0) red[wave * FR + l32] = m;
  __syncthreads();  // also: every band read is done (sbd becomes the ctx partial buffer)
  m = fmaxf(fmaxf(red[l32], red[FR + l32]), fmaxf(red[2 * FR + l32], red[3 * FR + l32]));
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < NTA; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = sc[t][r] == -INFINITY ? 0.f : expf(sc[t][r] - m);
      sc[t][r] = e;
      s += e;
    }
  s += __shfl_xor(s, 32, 64);
  if (hf == 0) red[4 * FR + wave * FR + l32] = s;
  __syncthreads();
  const float tot = (red[4 * FR + l32] + red[5 * FR + l32]) + (red[6 * FR + l32] + red[7 * FR + l32]);
  const float inv = tot > 0.f ? 1.0f / tot : 0.f;

  // ctx partial = P_drop V over this wave's key tiles: P^T (registers) is the A operand as is
  f32x16 cacc[2];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) cacc[c][r] = 0.f;
  const uint64_t rowbase = ((uint64_t)z * T + (uint64_t)min(i, T - 1)) * (uint64_t)T;
#pragma unroll
  for (int t = 0; t < NTA; ++t) {
    const int ct = wave + 4 * t;
    if (ct >= nac) continue;
    float pe[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      pe[r] = sc[t][r] * inv;
      if (a.thr) {
        const int j = ct * 32 + il_of(r, hf);
        pe[r] = esp::keep_elem(seed, rowbase + (uint64_t)j, a.thr) ? pe[r] * a.dscale : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      cacc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(pe[r], vv[0][r], cacc[0], 0, 0, 0);
      cacc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(pe[r], vv[1][r], cacc[1], 0, 0, 0);
    }
    if (t + 1 < NTA && ct + 4 < nac) load_v(ct + 4);
  }
  // fixed-order sum of the 4 waves' partials through LDS, float4 stores of the ctx rows
  constexpr int PP = FDK + 4;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) sbd[(wave * FR + il_of(r, hf)) * PP + 32 * c + l32] = cacc[c][r];
  __syncthreads();
  {
    const int q = threadIdx.x >> 3, d8 = (threadIdx.x & 7) * 8;
    if (i0 + q < T) {
      float* o = a.out + ((long)b * T + i0 + q) * a.ldc + FDK * head + d8;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float4 v = *reinterpret_cast<const float4*>(sbd + q * PP + d8 + 4 * u);
#pragma unroll
        for (int w = 1; w < 4; ++w) {
          const float4 x = *reinterpret_cast<const float4*>(sbd + (w * FR + q) * PP + d8 + 4 * u);
          v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w;
        }
        *reinterpret_cast<float4*>(o + 4 * u) = v;
      }
    }
  }
  if (wave == 0 && hf == 0 && i < T) {
    a.stats[((long)z * T + i) * 2] = m;
    a.stats[((long)z * T + i) * 2 + 1] = inv;
  }
}

// ============================================================================ backward
// 8 waves (2 per SIMD, one block per CU: ~122 KB LDS).  The block's q_u and dctx rows are staged
// in LDS (row pitch 68: ds_read_b128 of 16 rows conflict-free), so a key tile's MFMA chains hold
// only the k / v fragments of that tile.
constexpr int BW_WAVES = 8, BW_NT = 64 * BW_WAVES, RP = FDK + 4;
template <int REL>
__global__ __launch_bounds__(BW_NT, 1) void relpos_flash_bwd_kernel(FlashArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int T = a.T;
  const int nbd = (T + FR - 1 + 31) / 32;
  float* sbd = smem;                                 // band window [33][WP]; later the dq partials [8][32][36]
  float* ds = smem + a.band_sz;                      // dS rows of the block [32][DSP] (keys >= T zero)
  float* qs = ds + FR * a.DSP;                       // q_u rows [32][RP]
  float* gs = qs + FR * RP;                          // dctx rows [32][RP]
  float* qst = gs + FR * RP;                         // [3][32] row max, 1/sum, D_i
  int z, qb;
  block_task(a, z, qb);
  const int i0 = qb * FR;
  const int head = z / a.nb, b = z - head * a.nb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hf = lane >> 5, l32 = lane & 31;
  const int nac = (T + 31) / 32;
  const uint64_t seed = esp::keyed(a.seed, a.key);

  // stage q_u / dctx rows; row statistics and D_i = dctx_i . ctx_i (16 threads per row)
  {
    const int q = threadIdx.x >> 4, part = threadIdx.x & 15;
    const int iq = min(i0 + q, T - 1);
    const float4 u4 = *reinterpret_cast<const float4*>(a.qu + ((long)z * T + iq) * FDK + 4 * part);
    const float4 g4 = *reinterpret_cast<const float4*>(a.dctx + ((long)b * T + iq) * a.ldc + FDK * head + 4 * part);
    const float4 c4 = *reinterpret_cast<const float4*>(a.ctx + ((long)b * T + iq) * a.ldc + FDK * head + 4 * part);
    *reinterpret_cast<float4*>(qs + q * RP + 4 * part) = u4;
    *reinterpret_cast<float4*>(gs + q * RP + 4 * part) = g4;
    float dsum = c4.x * g4.x + c4.y * g4.y + c4.z * g4.z + c4.w * g4.w;
    dsum += __shfl_xor(dsum, 1, 64);
    dsum += __shfl_xor(dsum, 2, 64);
    dsum += __shfl_xor(dsum, 4, 64);
    dsum += __shfl_xor(dsum, 8, 64);
    if (part == 0) {
      qst[q] = a.stats[((long)z * T + iq) * 2];
      qst[FR + q] = a.stats[((long)z * T + iq) * 2 + 1];
      qst[2 * FR + q] = dsum;
    }
  }
  {  // band window, tiles dealt over the 8 waves
    const int kmin = T - FR - i0;
    float aq[2][16];
    load_row64(a.qv + ((long)z * T + min(i0 + l32, T - 1)) * FDK, hf, aq);
    float bq[2][16];
    if (wave < nbd) load_row64(p_virt_row<REL>(a, kmin + wave * 32 + l32, head), hf, bq);
#pragma unroll 1
    for (int ct = wave; ct < nbd; ct += BW_WAVES) {
      const f32x16 acc = mfma_rows(aq, bq);
      if (ct + BW_WAVES < nbd)  // next tile's p rows fly during this tile's stores
        load_row64(p_virt_row<REL>(a, kmin + (ct + BW_WAVES) * 32 + l32, head), hf, bq);
#pragma unroll
      for (int r = 0; r < 16; ++r) sbd[il_of(r, hf) * a.WP + ct * 32 + l32] = acc[r];
    }
    if (REL == 2 && i0 + FR < T) {
      const float* q = a.qv + ((long)z * T + i0 + FR) * FDK;
      for (int c = threadIdx.x; c < nbd * 32; c += BW_NT) {
        const float* pr = p_virt_row<REL>(a, kmin + c, head);
        float s = 0.f;
#pragma unroll 16
        for (int d = 0; d < FDK; d += 4) {
          const float4 pv = *reinterpret_cast<const float4*>(pr + d);
          const float4 qq = *reinterpret_cast<const float4*>(q + d);
          s += qq.x * pv.x + qq.y * pv.y + qq.z * pv.z + qq.w * pv.w;
        }
        sbd[FR * a.WP + c] = s;
      }
    }
  }
  int kl = a.klen ? a.klen[b] : T;
  kl = min(kl, T);
  __syncthreads();

  // scores (keys on lanes), P, dP, dS per key tile (tiles 0..7 to waves 0..7, 8..15 to waves
  // 7..0: the waves with one band tile take the second score tile); dS / P_drop to HBM, dS to LDS
  const int ct0 = wave, ct1 = 2 * BW_WAVES - 1 - wave;
  float kf[2][16], vf[2][16];  // k / v rows of the current key tile; the next tile's are loaded
  if (ct0 < nac) {             // as soon as the current tile's MFMAs have consumed them
    load_row64(a.kmat + ((long)b * T + min(ct0 * 32 + l32, T - 1)) * a.ldk + FDK * head, hf, kf);
    load_row64(a.vmat + ((long)b * T + min(ct0 * 32 + l32, T - 1)) * a.ldv + FDK * head, hf, vf);
  }
#pragma unroll 1
  for (int k = 0; k < 2; ++k) {
    const int ct = k == 0 ? ct0 : ct1;
    if (ct >= nac) continue;
    const int j = ct * 32 + l32;
    const bool nxt = k == 0 && ct1 < nac;
    const int jn = min(ct1 * 32 + l32, T - 1);
    f32x16 ac, dp;
    {
      float af[2][16];
      load_row64(qs + l32 * RP, hf, af);
      ac = mfma_rows(af, kf);
      if (nxt) load_row64(a.kmat + ((long)b * T + jn) * a.ldk + FDK * head, hf, kf);
    }
    {
      float af[2][16];
      load_row64(gs + l32 * RP, hf, af);
      dp = mfma_rows(af, vf);
      if (nxt) load_row64(a.vmat + ((long)b * T + jn) * a.ldv + FDK * head, hf, vf);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = il_of(r, hf), i = i0 + rr;
      float pe = 0.f;
      if (j < kl) {
        const float sv = (ac[r] + band_at<REL>(sbd, a.WP, rr, i, j)) * a.inv_sqrt_dk;
        pe = expf(sv - qst[rr]) * qst[FR + rr];
      }
      float pd = pe, g = dp[r];
      if (a.thr) {
        const bool keep = esp::keep_elem(seed, ((uint64_t)z * T + (uint64_t)min(i, T - 1)) * (uint64_t)T + j, a.thr);
        pd = keep ? pe * a.dscale : 0.f;
        g = keep ? g * a.dscale : 0.f;
      }
      const float dsv = pe * (g - qst[2 * FR + rr]) * a.inv_sqrt_dk;
      ds[rr * a.DSP + j] = dsv;  // j < nac*32 <= DSP; zero beyond klen / T (pe == 0)
      if (i < T && j < T) {
        const long o = ((long)z * T + i) * a.lds + j;
        a.dS[o] = dsv;
        a.pdrop[o] = pd;
      }
    }
  }
  __syncthreads();  // ds complete; the band window is dead

  // waves 0-3: dq_u = dS K over half the keys; waves 4-7: dq_v = Dbd p_win over half the window;
  // wave = (job, half, c): one 32x32 partial tile each -> LDS [8][32][36]
  const int c = wave & 1, half = (wave >> 1) & 1;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  if (wave < 4) {
    const int k0 = half ? (nac + 1) / 2 : 0, k1 = half ? nac : (nac + 1) / 2;
    const float* kcol = a.kmat + (long)b * T * a.ldk + FDK * head + 32 * c + l32;
    float bf[16];  // k column slice of the chunk; the next chunk's is requested before the MFMAs
    if (k0 < k1) {
#pragma unroll
      for (int s = 0; s < 16; ++s) bf[s] = kcol[(long)min(k0 * 32 + 16 * hf + s, T - 1) * a.ldk];
    }
#pragma unroll 1
    for (int kc = k0; kc < k1; ++kc) {
      float af[16], bn[16];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(ds + l32 * a.DSP + kc * 32 + 16 * hf + 4 * u);
        af[4 * u] = v.x; af[4 * u + 1] = v.y; af[4 * u + 2] = v.z; af[4 * u + 3] = v.w;
      }
      if (kc + 1 < k1) {
#pragma unroll
        for (int s = 0; s < 16; ++s) bn[s] = kcol[(long)min((kc + 1) * 32 + 16 * hf + s, T - 1) * a.ldk];
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 16; ++s) bf[s] = bn[s];
    }
  } else {
    // Dbd[rr][x] (window column x = position kmin + x): latest dS[rr][x + rr - 31]; legacy (q_v
    // row rr): the lower part j = x + rr - 31 <= i0 + rr from dS row rr, the upper part from row rr-1
    const int p0 = half ? (nbd + 1) / 2 : 0, p1 = half ? nbd : (nbd + 1) / 2;
    const int kmin = T - FR - i0;
    float bf[16];  // p_win column slice of the chunk (next chunk requested before the MFMAs)
    if (p0 < p1) {
#pragma unroll
      for (int s = 0; s < 16; ++s) bf[s] = p_virt_row<REL>(a, kmin + p0 * 32 + 16 * hf + s, head)[32 * c + l32];
    }
#pragma unroll 1
    for (int pc = p0; pc < p1; ++pc) {
      float af[16], bn[16];
      if (pc + 1 < p1) {
#pragma unroll
        for (int s = 0; s < 16; ++s)
          bn[s] = p_virt_row<REL>(a, kmin + (pc + 1) * 32 + 16 * hf + s, head)[32 * c + l32];
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int x = pc * 32 + 16 * hf + s;
        const int jj = x + l32 - 31;
        float v = 0.f;
        if (jj >= 0 && jj < nac * 32) {
          if (REL == 1 || jj <= i0 + l32) v = ds[l32 * a.DSP + jj];
          else if (l32 >= 1 && jj >= i0 + l32 + 1) v = ds[(l32 - 1) * a.DSP + jj];
        }
        af[s] = v;
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 16; ++s) bf[s] = bn[s];
    }
  }
  constexpr int QP = 36;
  float* pt = sbd;  // [8 waves][32][QP]
#pragma unroll
  for (int r = 0; r < 16; ++r) pt[(wave * FR + il_of(r, hf)) * QP + l32] = acc[r];
  __syncthreads();
  // dq = (dq_u + dq_v) rows -> out: tile of (job, half, c) is wave 4 job + 2 half + c
  {
    const int q = threadIdx.x >> 4, d4 = (threadIdx.x & 15) * 4;
    const int cc = d4 >> 5, dd = d4 & 31;
    if (i0 + q < T) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int w = 0; w < 4; ++w) {  // u half 0, u half 1, v half 0, v half 1 (fixed order)
        const int wv = (w >> 1) * 4 + (w & 1) * 2 + cc;
        const float4 x = *reinterpret_cast<const float4*>(pt + (wv * FR + q) * QP + dd);
        v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w;
      }
      *reinterpret_cast<float4*>(a.out + ((long)b * T + i0 + q) * a.ldq + FDK * head + d4) = v;
    }
  }
  // column sums over the block's valid rows: pos_bias_u / pos_bias_v gradient partials
  if (threadIdx.x < 128) {
    const int which = threadIdx.x >> 6, d = threadIdx.x & 63;
    const int cc = d >> 5, dd = d & 31;
    const int w0 = which * 4 + cc, w1 = which * 4 + 2 + cc;
    float s0 = 0.f;
    for (int q = 0; q < FR && i0 + q < T; ++q) s0 += pt[(w0 * FR + q) * QP + dd] + pt[(w1 * FR + q) * QP + dd];
    a.bias_part[(((long)z * a.nqb + qb) * 2 + which) * FDK + d] = s0;
  }
  if (REL == 2 && a.carry) {
    // legacy: the upper triangle of the block's last row (i0+31) belongs to q_v row i0+32:
    // carry[d] = sum_x dS[31][x + 1] p_virt[kmin + x][d] over x with j = x + 1 >= i0 + 33
    // (next block's dq row i0+32 and its pos_bias_v sum; added by esp_relpos_dp)
    __syncthreads();
    float* cp = sbd;  // [8][64]
    const int d = threadIdx.x & 63, part = threadIdx.x >> 6;
    const int kmin = T - FR - i0;
    float s0 = 0.f;
    if (i0 + FR < T) {
      for (int x = part; x < nbd * 32; x += BW_WAVES) {
        const int jj = x + 1;  // x + rr - 31 with rr = 32
        if (jj >= i0 + FR + 1 && jj < T) s0 += ds[(FR - 1) * a.DSP + jj] * p_virt_row<REL>(a, kmin + x, head)[d];
      }
    }
    cp[part * FDK + d] = s0;
    __syncthreads();
    if (threadIdx.x < FDK) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < BW_WAVES; ++w) t += cp[w * FDK + threadIdx.x];
      a.carry[((long)z * a.nqb + qb) * FDK + threadIdx.x] = t;
    }
  }
}

// ============================================================================ linear_pos gradient
// dp_virt[h][x][d] = sum_b sum_rho Dbd[z][rho][x] q_v[z][rho][d],  Dbd[rho][x] = dS[rho][x - (T-1) + rho]
// (latest; legacy: the lower part from dS row rho, the upper from dS row rho-1).  One block per
// (h, 32-position tile, batch group): 4 waves = (d-tile c, rho half); the A operand reads dS
// along diagonals (32 consecutive keys per row: coalesced), B = q_v rows.  Partials per batch
// group -> dp_part[h][g][x][64] (fixed order, no atomics); relpos_dp_reduce folds the groups
// (and, for legacy, p_virt back onto p: dp[x] + dp[x + T]).
template <int REL>
__global__ __launch_bounds__(256) void relpos_dp_kernel(const float* __restrict__ dS, long lds,
                                                        const float* __restrict__ qv, int nb, int T, int bpg,
                                                        float* __restrict__ dp_part) {
  __shared__ float part[2][FR][FDK + 4];
  const int P2 = 2 * T - 1;
  const int nxt = (P2 + 31) / 32;
  const int g = blockIdx.x % ((nb + bpg - 1) / bpg);
  const int rest = blockIdx.x / ((nb + bpg - 1) / bpg);
  const int xt = rest % nxt, h = rest / nxt;
  const int ng = (nb + bpg - 1) / bpg;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hf = lane >> 5, l32 = lane & 31;
  const int c = wave & 1, half = wave >> 1;
  const int x = xt * 32 + l32;  // this lane's position row (A row)
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int nrc = (T + 31) / 32;  // rho chunks of 32 (K dimension per batch element)
  const int b0 = g * bpg, nbb = min(nb, (g + 1) * bpg) - b0;
  const int nit = nbb * ((nrc - half + 1) / 2);  // (batch, this half's rho chunks) iterations
  auto load_it = [&](int it, float (&af)[16], float (&bf)[16]) {
    const int per = (nrc - half + 1) / 2;
    const int bb = b0 + it / per, rc = half + 2 * (it % per);
    const long zrow = (long)(h * nb + bb) * T;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int rho = rc * 32 + 16 * hf + s;
      float v = 0.f;
      if (rho < T && x < P2) {
        const int jj = x - (T - 1) + rho;
        if (REL == 1) {
          if (jj >= 0 && jj < T) v = dS[(zrow + rho) * lds + jj];
        } else {
          if (jj >= 0 && jj <= rho) v = dS[(zrow + rho) * lds + jj];
          else if (rho >= 1 && jj >= rho + 1 && jj < T) v = dS[(zrow + rho - 1) * lds + jj];
        }
      }
      af[s] = v;
      bf[s] = rho < T ? qv[(zrow + rho) * FDK + 32 * c + l32] : 0.f;
    }
  };
  float af[16], bf[16];
  if (nit > 0) load_it(0, af, bf);
#pragma unroll 1
  for (int it = 0; it < nit; ++it) {
    float an[16], bn[16];
    if (it + 1 < nit) load_it(it + 1, an, bn);
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      af[s] = an[s];
      bf[s] = bn[s];
    }
  }
  // halves 0 / 1 of rho combined in fixed order
  if (half == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) part[c][il_of(r, hf)][l32] = acc[r];
  }
  __syncthreads();
  if (half == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int xr = xt * 32 + il_of(r, hf);
      if (xr < P2)
        dp_part[(((long)h * ng + g) * P2 + xr) * FDK + 32 * c + l32] = acc[r] + part[c][il_of(r, hf)][l32];
    }
  }
}

// dp[pos][64h + d] = sum_g dp_part[h][g][pos][d] (+ [pos + T] for legacy); pos_bias grads from the
// per-block column sums (+ legacy carries); writes dp (overwrite) and accumulates the bias grads
template <int REL>
__global__ __launch_bounds__(256) void relpos_dp_reduce_kernel(const float* __restrict__ dp_part, int H, int ng, int T,
                                                               float* __restrict__ dp, long ldp) {
  const int P = REL == 2 ? T : 2 * T - 1, P2 = 2 * T - 1;
  const long n = (long)H * P * FDK;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int d = (int)(e % FDK);
    const long r = e / FDK;
    const int pos = (int)(r % P), h = (int)(r / P);
    float s = 0.f;
    for (int g = 0; g < ng; ++g) {
      s += dp_part[(((long)h * ng + g) * P2 + pos) * FDK + d];
      if (REL == 2 && pos + T < P2) s += dp_part[(((long)h * ng + g) * P2 + pos + T) * FDK + d];
    }
    dp[(long)pos * ldp + FDK * h + d] = s;
  }
}

// one block per (head, u|v, d): 256 threads split the (b, query block) partials, fixed-order
// block reduction (deterministic)
__global__ __launch_bounds__(256) void relpos_bias_reduce_kernel(const float* __restrict__ bias_part,
                                                                 const float* __restrict__ carry, int nb, int nqb,
                                                                 int T, float* __restrict__ du, float* __restrict__ dv) {
  __shared__ float sh[16];
  const int d = blockIdx.x & 63, which = (blockIdx.x >> 6) & 1, h = blockIdx.x >> 7;
  const int n = nb * nqb;
  float s = 0.f;
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int bb = e / nqb, qb = e - bb * nqb;
    const long blk = (long)(h * nb + bb) * nqb + qb;
    s += bias_part[(blk * 2 + which) * FDK + d];
    if (which && carry && (qb + 1) * FR < T) s += carry[blk * FDK + d];
  }
  s = esp::block_sum(s, sh);
  if (threadIdx.x == 0) (which ? dv : du)[h * FDK + d] += s;
}

// legacy: add each block's carry to q row i0+32 of the query gradient
__global__ __launch_bounds__(64) void relpos_carry_kernel(const float* __restrict__ carry, int nb, int nqb, int T,
                                                          float* __restrict__ dq, long ldq) {
  const int zq = blockIdx.x;
  const int qb = zq % nqb, z = zq / nqb;
  const int h = z / nb, b = z - h * nb;
  const int i = (qb + 1) * FR;
  if (i >= T) return;
  dq[((long)b * T + i) * ldq + FDK * h + threadIdx.x] += carry[(long)zq * FDK + threadIdx.x];
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

// LDS bytes of the flash kernels for T (the host sizes its launches with this)
static size_t flash_fwd_lds(int T, int rel, int* WP) {
  const int nbd = (T + FR - 1 + 31) / 32;
  *WP = nbd * 32 + 4;
  const size_t band = (size_t)(rel == 2 ? FR + 1 : FR) * *WP;
  const size_t part = (size_t)4 * FR * (FDK + 4);
  return ((band > part ? band : part) + 8 * FR) * sizeof(float);
}
static size_t flash_bwd_lds(int T, int* WP, int* DSP, int* band_sz) {
  const int nbd = (T + FR - 1 + 31) / 32;
  *WP = nbd * 32 + 4;
  const int nac = (T + 31) / 32;
  *DSP = nac * 32 + 4;  // odd number of quads: ds_read_b128 of 16 rows conflict-free
  size_t band = (size_t)(FR + 1) * *WP;
  const size_t part = (size_t)BW_WAVES * FR * 36;
  if (band < part) band = part;
  if (band < (size_t)BW_WAVES * FDK) band = BW_WAVES * FDK;
  *band_sz = (int)band;
  return (band + (size_t)FR * *DSP + 2 * (size_t)FR * RP + 3 * FR) * sizeof(float);
}

ESP_API int esp_relpos_flash_fwd(const float* qu, const float* qv, const float* kmat, long ldk, const float* vmat,
                                 long ldv, const float* p, long ldp_row, int rel, int nb, int H, float sqrt_dk,
                                 const int* klen, float* ctx, long ldc, float* stats, float drop_p,
                                 unsigned long long seed, int T, void* stream) {
  ESP_ARG_CHECK(rel == 1 || rel == 2, "esp_relpos_flash_fwd: rel must be 1 (latest) or 2 (legacy)");
  ESP_ARG_CHECK(T >= 1 && T <= 512 && nb >= 1 && H >= 1, "esp_relpos_flash_fwd: bad sizes T=%d", T);
  ESP_ARG_CHECK(ldk % 4 == 0 && ldv % 4 == 0 && ldp_row % 4 == 0 && ldc % 4 == 0 && al16(qu) && al16(qv) &&
                    al16(kmat) && al16(vmat) && al16(p) && al16(ctx),
                "esp_relpos_flash_fwd: operands must be 16-B aligned with ld %% 4 == 0");
  FlashArgs a{};
  a.qu = qu; a.qv = qv; a.kmat = kmat; a.vmat = vmat; a.pm = p;
  a.ldk = ldk; a.ldv = ldv; a.ldpm = ldp_row; a.ldc = ldc;
  a.klen = klen; a.out = ctx; a.stats = stats;
  a.nb = nb; a.T = T; a.nqb = (T + FR - 1) / FR; a.nblk = nb * H * a.nqb;
  a.sqrt_dk = sqrt_dk;
  a.inv_sqrt_dk = 1.0f / sqrt_dk;
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  a.thr = esp::drop_threshold(drop_p);
  a.dscale = esp::drop_scale(a.thr);
  a.seed = seed;
  a.key = esp::rng_key_ptr();
  const size_t shm = flash_fwd_lds(T, rel, &a.WP);
  a.DSP = (int)(shm / sizeof(float)) - 8 * FR;  // offset of the softmax exchange area
  const int nta = ((T + 31) / 32 + 3) / 4;
  hipStream_t st = (hipStream_t)stream;
#define ESP_FF(R, N) hipLaunchKernelGGL((relpos_flash_fwd_kernel<R, N>), dim3(a.nblk), dim3(256), shm, st, a)
#define ESP_FF_N(R)            \
  if (nta <= 1) ESP_FF(R, 1);   \
  else if (nta == 2) ESP_FF(R, 2); \
  else if (nta == 3) ESP_FF(R, 3); \
  else ESP_FF(R, 4);
  if (rel == 1) { ESP_FF_N(1) } else { ESP_FF_N(2) }
#undef ESP_FF_N
#undef ESP_FF
  ESP_CHECK_LAUNCH("esp_relpos_flash_fwd");
  return 0;
}

ESP_API int esp_relpos_flash_bwd(const float* qu, const float* qv, const float* kmat, long ldk, const float* vmat,
                                 long ldv, const float* p, long ldp_row, int rel, int nb, int H, float sqrt_dk,
                                 const int* klen, const float* ctx, const float* dctx, long ldc, const float* stats,
                                 float drop_p, unsigned long long seed, int T, float* dq, long ldq, float* dS,
                                 float* pdrop, long lds, float* bias_part, float* carry, void* stream) {
  ESP_ARG_CHECK(rel == 1 || rel == 2, "esp_relpos_flash_bwd: rel must be 1 (latest) or 2 (legacy)");
  ESP_ARG_CHECK(T >= 1 && T <= 512 && nb >= 1 && H >= 1 && lds >= T, "esp_relpos_flash_bwd: bad sizes T=%d", T);
  ESP_ARG_CHECK(ldk % 4 == 0 && ldv % 4 == 0 && ldp_row % 4 == 0 && ldc % 4 == 0 && ldq % 4 == 0 && al16(qu) &&
                    al16(qv) && al16(kmat) && al16(vmat) && al16(p) && al16(ctx) && al16(dctx) && al16(dq),
                "esp_relpos_flash_bwd: operands must be 16-B aligned with ld %% 4 == 0");
  ESP_ARG_CHECK(rel == 1 || carry, "esp_relpos_flash_bwd: legacy needs the carry buffer");
  FlashArgs a{};
  a.qu = qu; a.qv = qv; a.kmat = kmat; a.vmat = vmat; a.pm = p; a.ctx = ctx; a.dctx = dctx;
  a.ldk = ldk; a.ldv = ldv; a.ldpm = ldp_row; a.ldc = ldc;
  a.klen = klen; a.out = dq; a.ldq = ldq; a.stats = const_cast<float*>(stats);
  a.dS = dS; a.pdrop = pdrop; a.lds = lds; a.bias_part = bias_part; a.carry = rel == 2 ? carry : nullptr;
  a.nb = nb; a.T = T; a.nqb = (T + FR - 1) / FR; a.nblk = nb * H * a.nqb;
  a.sqrt_dk = sqrt_dk;
  a.inv_sqrt_dk = 1.0f / sqrt_dk;
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  a.thr = esp::drop_threshold(drop_p);
  a.dscale = esp::drop_scale(a.thr);
  a.seed = seed;
  a.key = esp::rng_key_ptr();
  const size_t shm = flash_bwd_lds(T, &a.WP, &a.DSP, &a.band_sz);
  ESP_ARG_CHECK(shm <= 160 * 1024, "esp_relpos_flash_bwd: T=%d needs %zu B of LDS", T, shm);
  hipStream_t st = (hipStream_t)stream;
  if (rel == 1) hipLaunchKernelGGL(relpos_flash_bwd_kernel<1>, dim3(a.nblk), dim3(BW_NT), shm, st, a);
  else hipLaunchKernelGGL(relpos_flash_bwd_kernel<2>, dim3(a.nblk), dim3(BW_NT), shm, st, a);
  ESP_CHECK_LAUNCH("esp_relpos_flash_bwd");
  return 0;
}

// linear_pos gradient input dp (P x D, head h at columns 64h; P = 2T-1 latest, T legacy) from dS
// and q_v; work: (H * ceil((2T-1)/32) * ng) * 64 * 64 * 4 floats of partials, ng = ceil(nb / bpg).
// Also reduces the flash backward's pos_bias partials into du / dv (accumulated) and, for
// legacy, adds the carries into dq.
// the workspace this call uses at its preferred grouping (8 utterances per partial); it works with
// less (fewer, larger groups), down to the one-group minimum H * (2T-1) * 64 floats
ESP_API long esp_relpos_dp_workspace_bytes(int nb, int H, int T) {
  return nb <= 0 || H <= 0 || T <= 0 ? 0 : 4L * H * ((nb + 7) / 8) * (2L * T - 1) * FDK;
}
ESP_API int esp_relpos_dp(const float* dS, long lds, const float* qv, int rel, int nb, int H, int T, float* dp, long ldp,
                          const float* bias_part, const float* carry, float* du, float* dv, float* dq, long ldq,
                          float* work, long work_floats, void* stream) {
  ESP_ARG_CHECK(rel == 1 || rel == 2, "esp_relpos_dp: rel must be 1 or 2");
  ESP_ARG_CHECK(T >= 1 && nb >= 1 && H >= 1 && lds >= T, "esp_relpos_dp: bad sizes");
  const int P2 = 2 * T - 1;
  int bpg = 8;
  int ng = (nb + bpg - 1) / bpg;
  while ((long)H * ng * P2 * FDK > work_floats && bpg < nb) {
    bpg *= 2;
    ng = (nb + bpg - 1) / bpg;
  }
  ESP_ARG_CHECK((long)H * ng * P2 * FDK <= work_floats, "esp_relpos_dp: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int nxt = (P2 + 31) / 32;
  const dim3 grid((unsigned)(H * nxt * ng));
  if (rel == 1) hipLaunchKernelGGL(relpos_dp_kernel<1>, grid, dim3(256), 0, st, dS, lds, qv, nb, T, bpg, work);
  else hipLaunchKernelGGL(relpos_dp_kernel<2>, grid, dim3(256), 0, st, dS, lds, qv, nb, T, bpg, work);
  const int P = rel == 2 ? T : P2;
  long nb_red = ((long)H * P * FDK + 255) / 256;
  if (nb_red > 8192) nb_red = 8192;
  if (rel == 1) hipLaunchKernelGGL(relpos_dp_reduce_kernel<1>, dim3((unsigned)nb_red), dim3(256), 0, st, work, H, ng, T, dp, ldp);
  else hipLaunchKernelGGL(relpos_dp_reduce_kernel<2>, dim3((unsigned)nb_red), dim3(256), 0, st, work, H, ng, T, dp, ldp);
  const int nqb = (T + FR - 1) / FR;
  if (bias_part)
    hipLaunchKernelGGL(relpos_bias_reduce_kernel, dim3(H * 128), dim3(256), 0, st, bias_part, rel == 2 ? carry : nullptr, nb,
                       nqb, T, du, dv);
  if (rel == 2 && carry && dq)
    hipLaunchKernelGGL(relpos_carry_kernel, dim3(nb * H * nqb), dim3(64), 0, st, carry, nb, nqb, T, dq, ldq);
  ESP_CHECK_LAUNCH("esp_relpos_dp");
  return 0;
}
