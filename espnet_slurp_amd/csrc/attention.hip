// Attention pieces around the MFMA GEMMs (attention.py:16-308):
//   * heads_split: q + pos_bias_u / q + pos_bias_v into head-major (H,B,T,dk) layout
//     (the layout the batch-summed linear_pos gradient GEMM needs, attention.py:290-293)
//   * masked softmax with the rel-pos score assembly fused in:
//       s[i,j] = (ac[i,j] + bd_shift[i,j]) / sqrt(dk), masked_fill(min) -> softmax ->
//       masked_fill(0) -> (dropout copy)        (attention.py:64-96, 145-165, 240-263)
//     latest : bd_shift[i,j] = bd[i, j+T-1-i]                  (bd: T x (2T-1))
//     legacy : j<=i -> bd[i, j+T-1-i]; j==i+1 -> 0; j>i+1 -> bd[i+1, j-i-2]   (bd: T x T)
//     mask   : key j valid iff j < klen[b] (and j <= i when causal, subsequent_mask)
//   * softmax backward (+ attention-dropout backward) and the rel_shift adjoint (a
//     gather, so no atomics: each bd element receives at most one score gradient).
// One wave per score row; rows of <= 64*PER keys live in registers.
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace {

constexpr int RP_ROWS = 32, RP_DK = 64;  // fused rel-pos kernels: query rows per block, d_k

__global__ void heads_split_kernel(const float* __restrict__ src, long ld, int col0, int B, int T, int H, int dk,
                                   const float* __restrict__ bias, float* __restrict__ dst) {
  const long n = (long)H * B * T * dk;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int d = (int)(i % dk);
    long r = i / dk;
    const int t = (int)(r % T);
    r /= T;
    const int b = (int)(r % B);
    const int h = (int)(r / B);
    float v = src[((long)b * T + t) * ld + col0 + h * dk + d];
    if (bias) v += bias[h * dk + d];
    dst[i] = v;
  }
}

// q + pos_bias_u AND q + pos_bias_v in one pass (one read of q, two head-major writes), a float4
// per thread: thread (row = b*T + t, head h, quad d4) of the (B*T, H*dk) source block.
__global__ void heads_split2_kernel(const float* __restrict__ src, long ld, int col0, int B, int T, int H, int dk,
                                    const float* __restrict__ bias_a, float* __restrict__ dst_a,
                                    const float* __restrict__ bias_b, float* __restrict__ dst_b) {
  const int q4n = dk >> 2, perrow = H * q4n;
  const long n = (long)B * T * perrow;
  for (long g = blockIdx.x * (long)blockDim.x + threadIdx.x; g < n; g += (long)gridDim.x * blockDim.x) {
    const int row = (int)(g / perrow), rem = (int)(g - (long)row * perrow);
    const int h = rem / q4n, d = 4 * (rem - h * q4n);
    const int b = row / T, t = row - b * T;
    const float4 v = *reinterpret_cast<const float4*>(src + (long)row * ld + col0 + h * dk + d);
    const float4 ua = *reinterpret_cast<const float4*>(bias_a + h * dk + d);
    const float4 ub = *reinterpret_cast<const float4*>(bias_b + h * dk + d);
    const long o = (((long)h * B + b) * T + t) * dk + d;
    *reinterpret_cast<float4*>(dst_a + o) = make_float4(v.x + ua.x, v.y + ua.y, v.z + ua.z, v.w + ua.w);
    *reinterpret_cast<float4*>(dst_b + o) = make_float4(v.x + ub.x, v.y + ub.y, v.z + ub.z, v.w + ub.w);
  }
}

// Attention backward prep (esp_attn_bwd_prep), one wave per score row (z, i), z = h*nb + b:
//   dot[z*T + i] = dctx[b*T+i][h*dk ..] . ctx[b*T+i][h*dk ..]  (= sum_j P_drop[i][j] dP[i][j])
//   and the bd-gradient elements the score-gradient epilogue never writes set to 0:
//   latest: k < T-1-i and k >= 2T-1-i;  legacy: row 0's k < T-1.
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const float* __restrict__ dctx, long ldd,
                                                            const float* __restrict__ ctx, long ldc, int nb, int H,
                                                            int dk, int T, float* __restrict__ dot,
                                                            float* __restrict__ dbd, long ldp, int relpos) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)nb * H * T) return;
  const int i = (int)(row % T);
  const int z = (int)(row / T);
  const int h = z / nb, b = z - h * nb;
  const long src = ((long)b * T + i);
  float acc = 0.f;
  for (int d = lane; d < dk; d += 64) acc += dctx[src * ldd + h * dk + d] * ctx[src * ldc + h * dk + d];
  acc = esp::wave_sum(acc);
  if (lane == 0) dot[row] = acc;
  float* br = dbd + row * ldp;
  const int sh = T - 1 - i;
  if (relpos == 1) {
    for (int k = lane; k < sh; k += 64) br[k] = 0.f;
    for (int k = sh + T + lane; k < 2 * T - 1; k += 64) br[k] = 0.f;
  } else if (i == 0) {
    for (int k = lane; k < sh; k += 64) br[k] = 0.f;
  }
}

// y[r*ldy + c] += x[r*ldx + c]
__global__ void add2d_kernel(const float* __restrict__ x, long ldx, float* __restrict__ y, long ldy, int M, int N) {
  const long n = (long)M * N;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / N;
    const int c = (int)(i - r * N);
    y[r * ldy + c] += x[r * ldx + c];
  }
}

template <int PER>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const float* ac, const float* __restrict__ bd, int relpos,
                                                          int P, float sqrt_dk, const int* __restrict__ klen, int nb,
                                                          int causal, float* attn, float* __restrict__ pdrop,
                                                          uint32_t thr, float dscale, uint64_t seed, int Z, int Tq,
                                                          int Tk, long lds, long ldp, const uint64_t* __restrict__ key,
                                                          const int* __restrict__ tvalid) {
  seed = esp::keyed(seed, key);
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)Z * Tq) return;
  const int i = (int)(row % Tq);
  // legacy + length bucket: the rel_shift of the reference batch, length T' = *tvalid; rows
  // i >= T' are padding (their scores skip the band: finite, never read by a valid row)
  const int Ts = relpos == 2 && tvalid ? min(max(*tvalid, 1), Tq) : Tq;
  const int z = (int)(row / Tq);
  const int b = z % nb;  // z = h*nb + b
  int kl = klen ? klen[b] : Tk;
  if (kl > Tk) kl = Tk;
  const float* acr = ac + row * lds;
  const float* bdz = bd ? bd + (long)z * Tq * ldp : nullptr;
  float v[PER];
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int j = lane + 64 * e;
    float s = -INFINITY;
    if (j < Tk && j < kl && !(causal && j > i)) {
      float a = acr[j];
      if (relpos == 1) {
        a += bdz[(long)i * ldp + (j + Tq - 1 - i)];
      } else if (relpos == 2 && i < Ts) {
        if (j <= i) a += bdz[(long)i * ldp + (j + Ts - 1 - i)];
        else if (j > i + 1) a += bdz[(long)(i + 1) * ldp + (j - i - 2)];
      }
      s = a / sqrt_dk;
    }
    v[e] = s;
    mx = fmaxf(mx, s);
  }
  mx = esp::wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const float p = v[e] == -INFINITY ? 0.f : expf(v[e] - mx);
    v[e] = p;
    sum += p;
  }
  sum = esp::wave_sum(sum);
  const float inv = sum > 0.f ? 1.0f / sum : 0.f;
  float* ar = attn + row * lds;
  float* pr = pdrop ? pdrop + row * lds : nullptr;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int j = lane + 64 * e;
    if (j < Tk) {
      const float p = v[e] * inv;
      ar[j] = p;
      if (pr) pr[j] = esp::keep_elem(seed, (uint64_t)(row * Tk + j), thr) ? p * dscale : 0.f;
    }
  }
}

// dS = attn * (g - sum_j attn*g) / sqrt_dk,  g = dP * dropmask * dscale.  dS may alias dP.
template <int PER>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const float* __restrict__ attn, const float* dP, float* dS,
                                                          uint32_t thr, float dscale, uint64_t seed, float sqrt_dk,
                                                          long rows, int Tk, long lds, const uint64_t* __restrict__ key) {
  seed = esp::keyed(seed, key);
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* ar = attn + row * lds;
  const float* gr = dP + row * lds;
  float a[PER], g[PER];
  float dot = 0.f;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int j = lane + 64 * e;
    a[e] = 0.f;
    g[e] = 0.f;
    if (j < Tk) {
      a[e] = ar[j];
      float gv = gr[j];
      if (thr) gv = esp::keep_elem(seed, (uint64_t)(row * Tk + j), thr) ? gv * dscale : 0.f;
      g[e] = gv;
    }
    dot += a[e] * g[e];
  }
  dot = esp::wave_sum(dot);
  float* sr = dS + row * lds;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int j = lane + 64 * e;
    if (j < Tk) sr[j] = a[e] * (g[e] - dot) / sqrt_dk;
  }
}

// softmax backward fused with the rel_shift adjoint, so dS is not re-read by a separate relshift
// pass.  dS may alias dP.  The wave that owns score row (z, i) writes dS[i][j] and
//   latest (REL 1): the whole dbd row  dbd[i][k] = dS[i][k - (T-1-i)]  (0 outside the band);
//   legacy (REL 2): dbd[i][j + T-1-i] = dS[i][j] for j <= i (the upper part of row i) and
//                   dbd[i+1][j - i - 2] = dS[i][j] for j >= i+2 (the lower part of row i+1);
//                   row 0's lower part has no source and is zeroed by row 0's wave.
// Each dbd element has exactly one source (relshift_bwd_kernel's gather), so no atomics.
// Legacy with tvalid (a length-bucketed batch padded from T' = *tvalid to T frames): the shift
// is the reference batch's, T' - 1 - i, rows i >= T' and columns >= T' of dbd are zero, and the
// upper part only moves j < T' (the padded keys are masked: their dS is 0, and writing it would
// land on elements row i+1's lower part owns) -- the unpadded adjoint, zero-extended.
__device__ __forceinline__ int legacy_tv(const int* tvalid, int T) {
  if (!tvalid) return T;
  const int t = *tvalid;
  return t < 1 ? 1 : (t > T ? T : t);
}
template <int PER, int REL>
__global__ __launch_bounds__(256) void softmax_bwd_relpos_kernel(const float* __restrict__ attn, const float* dP,
                                                                 float* dS, float* __restrict__ dbd, long ldp,
                                                                 uint32_t thr, float dscale, uint64_t seed,
                                                                 float sqrt_dk, long rows, int T, long lds,
                                                                 const uint64_t* __restrict__ key,
                                                                 const int* __restrict__ tvalid) {
  seed = esp::keyed(seed, key);
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int i = (int)(row % T);
  const float* ar = attn + row * lds;
  const float* gr = dP + row * lds;
  float a[PER], g[PER];
  float dot = 0.f;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int j = lane + 64 * e;
    a[e] = 0.f;
    g[e] = 0.f;
    if (j < T) {
      a[e] = ar[j];
      float gv = gr[j];
      if (thr) gv = esp::keep_elem(seed, (uint64_t)(row * T + j), thr) ? gv * dscale : 0.f;
      g[e] = gv;
    }
    dot += a[e] * g[e];
  }
  dot = esp::wave_sum(dot);
  float* sr = dS + row * lds;
  float* br = dbd + row * ldp;
  const int Ts = REL == 2 ? legacy_tv(tvalid, T) : T;  // the rel_shift's length
  const bool live = REL == 1 || i < Ts;
  const int sh = Ts - 1 - i;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int j = lane + 64 * e;
    if (j < T) {
      const float v = a[e] * (g[e] - dot) / sqrt_dk;
      sr[j] = v;
      if (!live) continue;
      if (REL == 1 || j <= i) br[j + sh] = v;
      else if (j >= i + 2 && j < Ts) br[ldp + j - i - 2] = v;  // row i+1 of the same z (i + 1 < Ts here)
    }
  }
  if (REL == 1) {
    for (int k = lane; k < sh; k += 64) br[k] = 0.f;
    for (int k = sh + T + lane; k < 2 * T - 1; k += 64) br[k] = 0.f;
  } else {
    if (!live) {
      for (int k = lane; k < T; k += 64) br[k] = 0.f;
    } else {
      if (i == 0)
        for (int k = lane; k < sh; k += 64) br[k] = 0.f;
      for (int k = Ts + lane; k < T; k += 64) br[k] = 0.f;
    }
  }
}

// Rows longer than the register-resident kernels hold (Tk > 1024: utterances past ~41 s at 40 ms frames):
// the same arithmetic in passes over the row -- max, sum of exp(s - max), then the normalised write --
// with the score (ac + the rel_shift of bd, masks) recomputed from HBM on each pass, so the values equal
// softmax_fwd_kernel's (same expf arguments, same wave reductions; only the summation grouping per lane
// differs).  One wave per row, any length.
__device__ __forceinline__ float softmax_score(const float* acr, const float* bdz, int relpos, int i, int j, int Tq,
                                               int Ts, long ldp, int kl, int causal, float sqrt_dk) {
  if (j >= kl || (causal && j > i)) return -INFINITY;
  float a = acr[j];
  if (relpos == 1) {
    a += bdz[(long)i * ldp + (j + Tq - 1 - i)];
  } else if (relpos == 2 && i < Ts) {
    if (j <= i) a += bdz[(long)i * ldp + (j + Ts - 1 - i)];
    else if (j > i + 1) a += bdz[(long)(i + 1) * ldp + (j - i - 2)];
  }
  return a / sqrt_dk;
}
__global__ __launch_bounds__(256) void softmax_fwd_loop_kernel(const float* ac, const float* __restrict__ bd,
                                                               int relpos, int P, float sqrt_dk,
                                                               const int* __restrict__ klen, int nb, int causal,
                                                               float* attn, float* __restrict__ pdrop, uint32_t thr,
                                                               float dscale, uint64_t seed, int Z, int Tq, int Tk,
                                                               long lds, long ldp, const uint64_t* __restrict__ key,
                                                               const int* __restrict__ tvalid) {
  seed = esp::keyed(seed, key);
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)Z * Tq) return;
  const int i = (int)(row % Tq);
  const int Ts = relpos == 2 && tvalid ? min(max(*tvalid, 1), Tq) : Tq;
  const int z = (int)(row / Tq);
  const int b = z % nb;
  int kl = klen ? klen[b] : Tk;
  if (kl > Tk) kl = Tk;
  const float* acr = ac + row * lds;
  const float* bdz = bd ? bd + (long)z * Tq * ldp : nullptr;
  float mx = -INFINITY;
  for (int j = lane; j < Tk; j += 64) mx = fmaxf(mx, softmax_score(acr, bdz, relpos, i, j, Tq, Ts, ldp, kl, causal, sqrt_dk));
  mx = esp::wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < Tk; j += 64) {
    const float v = softmax_score(acr, bdz, relpos, i, j, Tq, Ts, ldp, kl, causal, sqrt_dk);
    sum += v == -INFINITY ? 0.f : expf(v - mx);
  }
  sum = esp::wave_sum(sum);
  const float inv = sum > 0.f ? 1.0f / sum : 0.f;
  float* ar = attn + row * lds;
  float* pr = pdrop ? pdrop + row * lds : nullptr;
  for (int j = lane; j < Tk; j += 64) {
    const float v = softmax_score(acr, bdz, relpos, i, j, Tq, Ts, ldp, kl, causal, sqrt_dk);
    const float p = (v == -INFINITY ? 0.f : expf(v - mx)) * inv;
    ar[j] = p;  // (ac may alias attn: element j was read above by this lane only)
    if (pr) pr[j] = esp::keep_elem(seed, (uint64_t)(row * Tk + j), thr) ? p * dscale : 0.f;
  }
}

// softmax backward (REL 0), + the latest (1) / legacy (2) rel_shift adjoint, for rows of any length: the
// dot pass, then the dS (and dbd) pass -- softmax_bwd_kernel / softmax_bwd_relpos_kernel's arithmetic
template <int REL>
__global__ __launch_bounds__(256) void softmax_bwd_loop_kernel(const float* __restrict__ attn, const float* dP,
                                                               float* dS, float* __restrict__ dbd, long ldp,
                                                               uint32_t thr, float dscale, uint64_t seed,
                                                               float sqrt_dk, long rows, int T, long lds,
                                                               const uint64_t* __restrict__ key,
                                                               const int* __restrict__ tvalid) {
  seed = esp::keyed(seed, key);
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* ar = attn + row * lds;
  const float* gr = dP + row * lds;
  auto gval = [&](int j) {
    float gv = gr[j];
    if (thr) gv = esp::keep_elem(seed, (uint64_t)(row * T + j), thr) ? gv * dscale : 0.f;
    return gv;
  };
  float dot = 0.f;
  for (int j = lane; j < T; j += 64) dot += ar[j] * gval(j);
  dot = esp::wave_sum(dot);
  float* sr = dS + row * lds;
  if constexpr (REL == 0) {
    for (int j = lane; j < T; j += 64) sr[j] = ar[j] * (gval(j) - dot) / sqrt_dk;
    return;
  } else {
    const int i = (int)(row % T);
    float* br = dbd + row * ldp;
    const int Ts = REL == 2 ? legacy_tv(tvalid, T) : T;
    const bool live = REL == 1 || i < Ts;
    const int sh = Ts - 1 - i;
    for (int j = lane; j < T; j += 64) {
      const float v = ar[j] * (gval(j) - dot) / sqrt_dk;
      sr[j] = v;
      if (!live) continue;
      if (REL == 1 || j <= i) br[j + sh] = v;
      else if (j >= i + 2 && j < Ts) br[ldp + j - i - 2] = v;
    }
    if (REL == 1) {
      for (int k = lane; k < sh; k += 64) br[k] = 0.f;
      for (int k = sh + T + lane; k < 2 * T - 1; k += 64) br[k] = 0.f;
    } else {
      if (!live) {
        for (int k = lane; k < T; k += 64) br[k] = 0.f;
      } else {
        if (i == 0)
          for (int k = lane; k < sh; k += 64) br[k] = 0.f;
        for (int k = Ts + lane; k < T; k += 64) br[k] = 0.f;
      }
    }
  }
}

// float4 form of softmax_bwd_relpos_kernel (lds % 4 == 0, 16-B aligned rows): lane L loads the
// quads 4L + 256q of P and dP (1 KB per wave instruction instead of 256 B), writes dS as float4
// (the pitch's padding columns get 0), and hands its 4 values through a per-wave LDS row so the
// rel_shift-adjoint dbd stores stay one contiguous 256-B run per instruction (j = lane + 64e).
// P2: sqrt(d_k) a power of two -> exact multiply by 1/sqrt(d_k).
// REL 1 latest, 2 legacy, 3 latest writing only the dbd band (row i: columns T-1-i .. 2T-2-i) into a
// buffer whose other elements are already zero (esp_attn_softmax_bwd_relpos_band: half the dbd bytes)
template <int Q, int REL, bool P2>  // Q quads per lane: 256*Q >= T
__global__ __launch_bounds__(256) void softmax_bwd_relpos4_kernel(const float* __restrict__ attn, const float* dP,
                                                                  float* dS, float* __restrict__ dbd, long ldp,
                                                                  uint32_t thr, float dscale, uint64_t seed,
                                                                  float sqrt_dk, long rows, int T, long lds,
                                                                  const uint64_t* __restrict__ key,
                                                                  const int* __restrict__ tvalid) {
  __shared__ __attribute__((aligned(16))) float stage[4][256 * Q];
  seed = esp::keyed(seed, key);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long row = (long)blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const int i = (int)(row % T);
  const float* ar = attn + row * lds;
  const float* gr = dP + row * lds;
  float a[Q][4], g[Q][4];
  float dot = 0.f;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int j0 = 4 * lane + 256 * q;
    float4 av = make_float4(0.f, 0.f, 0.f, 0.f), gv = av;
    if (j0 < T) {  // the quad stays inside the row pitch (lds >= round_up(T, 4))
      av = *reinterpret_cast<const float4*>(ar + j0);
      gv = *reinterpret_cast<const float4*>(gr + j0);
    }
    const float aa[4] = {av.x, av.y, av.z, av.w}, gg[4] = {gv.x, gv.y, gv.z, gv.w};
    bool kp[4] = {true, true, true, true};
    if (thr) {
      const uint64_t ix = (uint64_t)(row * T + j0);
      if ((T & 1) == 0) {  // row * T even: two hash pairs per quad (esp::keep_pair)
        esp::keep_pair(seed, ix, thr, kp[0], kp[1]);
        esp::keep_pair(seed, ix + 2, thr, kp[2], kp[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) kp[e] = esp::keep_elem(seed, ix + e, thr);
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = j0 + e;
      float x = j < T ? gg[e] : 0.f;
      if (thr) x = kp[e] ? x * dscale : 0.f;
      a[q][e] = j < T ? aa[e] : 0.f;
      g[q][e] = x;
      dot += a[q][e] * x;
    }
  }
  dot = esp::wave_sum(dot);
  const float inv = 1.0f / sqrt_dk;
  float* sr = dS + row * lds;
  float* st = stage[wave];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int j0 = 4 * lane + 256 * q;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = P2 ? a[q][e] * (g[q][e] - dot) * inv : a[q][e] * (g[q][e] - dot) / sqrt_dk;
    if (j0 < T) *reinterpret_cast<float4*>(sr + j0) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(st + j0) = make_float4(v[0], v[1], v[2], v[3]);
  }
  asm volatile("" ::: "memory");  // wave-private LDS row: in-order within the wave
  float* br = dbd + row * ldp;
  const int Ts = REL == 2 ? legacy_tv(tvalid, T) : T;  // the rel_shift's length (see the scalar kernel)
  const bool live = REL != 2 || i < Ts;
  const int sh = Ts - 1 - i;
  if (live) {
#pragma unroll
    for (int e = 0; e < 4 * Q; ++e) {
      const int j = lane + 64 * e;
      if (j < T) {
        const float v = st[j];
        if (REL != 2 || j <= i) br[j + sh] = v;
        else if (j >= i + 2 && j < Ts) br[ldp + j - i - 2] = v;  // row i+1 of the same z (i + 1 < Ts here)
      }
    }
  }
  if constexpr (REL == 1) {
    for (int k = lane; k < sh; k += 64) br[k] = 0.f;
    for (int k = sh + T + lane; k < 2 * T - 1; k += 64) br[k] = 0.f;
  } else if constexpr (REL == 2) {
    if (!live) {
      for (int k = lane; k < T; k += 64) br[k] = 0.f;
    } else {
      if (i == 0)
        for (int k = lane; k < sh; k += 64) br[k] = 0.f;
      for (int k = Ts + lane; k < T; k += 64) br[k] = 0.f;
    }
  }
}

// Fused latest rel-pos attention backward, one block per (32 query rows, z):
//   dP = dctx V^T on the MFMA (key tiles w, w+4, ... per wave; V rows from the fused qkv),
//   g  = dropout'(dP) (mask regenerated), dot_i = sum_j attn*g (xor shuffles + LDS exchange),
//   dS = attn*(g - dot)/sqrt(dk)  -> dS (pitch lds) and dbd[i][j + T-1-i] (pitch ldp, zero
//   outside the band).  Replaces the dctx.V^T GEMM (K = 64) + the softmax/rel_shift adjoint.
template <int NTA>
__global__ __launch_bounds__(256) void relpos_attn_bwd_kernel(
    const float* __restrict__ dctx, long ldd, const float* __restrict__ vmat, long ldv, const float* __restrict__ attn,
    float* __restrict__ dS, float* __restrict__ dbd, long ldp, int nb, float sqrt_dk, uint32_t thr, float dscale,
    uint64_t seed, int T, long lds, const uint64_t* __restrict__ key) {
  __shared__ float rdot[4][RP_ROWS];
  seed = esp::keyed(seed, key);
  const int z = blockIdx.y;
  const int i0 = blockIdx.x * RP_ROWS;
  const int head = z / nb, b = z - head * nb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hf = lane >> 5, l32 = lane & 31;
  const int nac = (T + 31) / 32;

  auto load_row32 = [&](const float* row, float (&f)[2][16]) {  // d = 32c + 16hf + s
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(row + 32 * c + 16 * hf + 4 * u);
        f[c][4 * u] = v.x; f[c][4 * u + 1] = v.y; f[c][4 * u + 2] = v.z; f[c][4 * u + 3] = v.w;
      }
  };
  float ad[2][16], bq[NTA][2][16];
  load_row32(dctx + ((long)b * T + min(i0 + l32, T - 1)) * ldd + head * RP_DK, ad);
#pragma unroll
  for (int t = 0; t < NTA; ++t)
    if (wave + 4 * t < nac)
      load_row32(vmat + ((long)b * T + min((wave + 4 * t) * 32 + l32, T - 1)) * ldv + head * RP_DK, bq[t]);

  f32x16 g[NTA], a[NTA];
  float dot[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) dot[r] = 0.f;
#pragma unroll
  for (int t = 0; t < NTA; ++t) {
    const int j = (wave + 4 * t) * 32 + l32;
    const bool jok = j < T && wave + 4 * t < nac;
#pragma unroll
    for (int r = 0; r < 16; ++r) {  // attn loads first: they fly during the MFMAs
      const int i = min(i0 + (r & 3) + 8 * (r >> 2) + 4 * hf, T - 1);
      a[t][r] = jok ? attn[((long)z * T + i) * lds + j] : 0.f;
    }
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if (wave + 4 * t < nac) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int st = 0; st < 16; ++st) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ad[c][st], bq[t][c][st], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long row = (long)z * T + min(i0 + (r & 3) + 8 * (r >> 2) + 4 * hf, T - 1);
      float gv = jok ? acc[r] : 0.f;
      if (thr && jok) gv = esp::keep_elem(seed, (uint64_t)(row * T + j), thr) ? gv * dscale : 0.f;
      g[t][r] = gv;
      dot[r] += a[t][r] * gv;
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) dot[r] += __shfl_xor(dot[r], o, 64);
  }
  if (l32 == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) rdot[wave][(r & 3) + 8 * (r >> 2) + 4 * hf] = dot[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int il = (r & 3) + 8 * (r >> 2) + 4 * hf;
    dot[r] = (rdot[0][il] + rdot[1][il]) + (rdot[2][il] + rdot[3][il]);
  }
#pragma unroll
  for (int t = 0; t < NTA; ++t) {
    const int j = (wave + 4 * t) * 32 + l32;
    if (j >= T || wave + 4 * t >= nac) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * hf;
      if (i >= T) continue;
      const long row = (long)z * T + i;
      const float v = a[t][r] * (g[t][r] - dot[r]) / sqrt_dk;
      dS[row * lds + j] = v;
      dbd[row * ldp + j + (T - 1 - i)] = v;
    }
  }
  // zero the dbd entries outside each row's band (k < T-1-i and k > 2T-2-i)
  for (int rr = wave; rr < RP_ROWS; rr += 4) {
    const int i = i0 + rr;
    if (i >= T) break;
    float* br = dbd + ((long)z * T + i) * ldp;
    const int sh = T - 1 - i;
    for (int k = lane; k < sh; k += 64) br[k] = 0.f;
    for (int k = sh + T + lane; k < 2 * T - 1; k += 64) br[k] = 0.f;
  }
}

// adjoint of the rel_shift gather: dbd (Z,T,P) [pitch ldp] from dS (Z,T,T) [pitch lds]
__global__ void relshift_bwd_kernel(const float* __restrict__ dS, long lds, float* __restrict__ dbd, long ldp,
                                    int relpos, int Z, int T, int P) {
  const long n = (long)Z * T * P;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
    const int k = (int)(idx % P);
    const long r = idx / P;
    const int i = (int)(r % T);
    const long z = r / T;
    const float* dz = dS + z * T * lds;
    float v = 0.f;
    if (relpos == 1) {
      const int j = k - (T - 1 - i);
      if (j >= 0 && j < T) v = dz[(long)i * lds + j];
    } else {
      if (k >= T - 1 - i) v = dz[(long)i * lds + (k - T + 1 + i)];
      else if (i >= 1 && k + i + 1 < T) v = dz[(long)(i - 1) * lds + (k + i + 1)];
    }
    dbd[r * ldp + k] = v;
  }
}

// ---------------------------------------------------------------- fused latest rel-pos softmax
// One block per (32 query rows, z): the bd window of the block is computed on the MFMA
//   Sbd[r][c] = q_v[z][i0 + r] . p[kmin + c],   kmin = T - 32 - i0,  c in [0, T + 31)
// (the 32 x (T+31) band of (q+v) p^T that rel_shift reads: bd_shift[i][j] = Sbd[i-i0][j-(i-i0)+31])
// into LDS, then each wave finishes 8 score rows: s = (ac + bd_shift) / sqrt(dk), key mask,
// softmax (wave shuffles), attention-dropout copy.  Replaces the (Z,T,2T-1) bd GEMM + its HBM
// round trip + the separate softmax pass.  d_k = 64; LDS = 32 x WP floats (WP = 32*ceil((T+31)/32)+4).
// MFMA operand k-order: lane half hf supplies d = 32c + 16hf + s at step (c, s) for both operands.
template <int PER>
__global__ __launch_bounds__(256) void relpos_softmax_fwd_kernel(
    const float* __restrict__ qv, const float* __restrict__ pm, long ldpm, int nb, int H, const float* ac,
    float sqrt_dk, const int* __restrict__ klen, float* attn, float* __restrict__ pdrop, uint32_t thr, float dscale,
    uint64_t seed, int T, long lds, int WP, const uint64_t* __restrict__ key) {
  extern __shared__ __attribute__((aligned(16))) float sbd[];  // [32][WP]
  seed = esp::keyed(seed, key);
  const int z = blockIdx.y;
  const int i0 = blockIdx.x * RP_ROWS;
  const int head = z / nb, b = z - head * nb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hf = lane >> 5, l32 = lane & 31;
  const int P = 2 * T - 1;
  const int kmin = T - RP_ROWS - i0;
  const int ntile = (T + RP_ROWS - 1 + 31) / 32;

  // A fragments: row i0 + l32 of q_v[z] (rows past T clamped: their scores are never used)
  float af[2][16];
  {
    const float* q = qv + ((long)z * T + min(i0 + l32, T - 1)) * RP_DK;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(q + 32 * c + 16 * hf + 4 * u);
        af[c][4 * u] = v.x; af[c][4 * u + 1] = v.y; af[c][4 * u + 2] = v.z; af[c][4 * u + 3] = v.w;
      }
  }
  for (int ct = wave; ct < ntile; ct += 4) {
    const int k = min(max(kmin + ct * 32 + l32, 0), P - 1);
    const float* pr = pm + (long)k * ldpm + head * RP_DK;
    float bfr[2][16];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(pr + 32 * c + 16 * hf + 4 * u);
        bfr[c][4 * u] = v.x; bfr[c][4 * u + 1] = v.y; bfr[c][4 * u + 2] = v.z; bfr[c][4 * u + 3] = v.w;
      }
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int st = 0; st < 16; ++st) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[c][st], bfr[c][st], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) sbd[((r & 3) + 8 * (r >> 2) + 4 * hf) * WP + ct * 32 + l32] = acc[r];
  }
  __syncthreads();

  const int* klp = klen;
  int kl = klp ? klp[b] : T;
  if (kl > T) kl = T;
  for (int rr = wave; rr < RP_ROWS; rr += 4) {
    const int i = i0 + rr;
    if (i >= T) break;
    const long row = (long)z * T + i;
    const float* acr = ac + row * lds;
    const float* sb = sbd + rr * WP + (RP_ROWS - 1 - rr);
    float v[PER];
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int j = lane + 64 * e;
      float sc = -INFINITY;
      if (j < T && j < kl) sc = (acr[j] + sb[j]) / sqrt_dk;
      v[e] = sc;
      mx = fmaxf(mx, sc);
    }
    mx = esp::wave_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const float pe = v[e] == -INFINITY ? 0.f : expf(v[e] - mx);
      v[e] = pe;
      sum += pe;
    }
    sum = esp::wave_sum(sum);
    const float inv = sum > 0.f ? 1.0f / sum : 0.f;
    float* ar = attn + row * lds;
    float* pd = pdrop ? pdrop + row * lds : nullptr;
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int j = lane + 64 * e;
      if (j < T) {
        const float pe = v[e] * inv;
        ar[j] = pe;
        if (pd) pd[j] = esp::keep_elem(seed, (uint64_t)(row * T + j), thr) ? pe * dscale : 0.f;
      }
    }
  }
}

// ---------------------------------------------------------------- fused latest rel-pos attention scores
// The whole score path of one (32 query rows, z) block in one kernel — no (Z,T,T) ac and no
// (Z,T,2T-1) bd tensor in HBM:
//   1. bd band window  Sbd[r][c] = q_v[i0+r] . p[kmin+c]     (MFMA, LDS)          as above
//   2. ac tiles        ac[r][j]  = q_u[i0+r] . k[j]          (MFMA, registers; wave w owns
//                                                            key tiles w, w+4, ...)
//   3. s = (ac + Sbd[r][j-r+31]) / sqrt(dk), key mask, row max / sum by xor-shuffles inside the
//      32-lane halves + a 4-wave LDS exchange, p = e/sum -> attn (+ dropout copy pdrop).
// k rows are read from the fused qkv projection: k[z][j] = kmat[(b*T + j)*ldk + 64*head].
// P2: sqrt(d_k) is a power of two (d_k = 64 in every configuration here), so s / sqrt(d_k) is
// computed exactly as s * (1 / sqrt(d_k)); exp(s - m) as exp2((s - m) * log2 e) on v_exp_f32
// (the score assembly and softmax are VALU-bound: ~100 instructions per score element with the
// IEEE division and the range-reduced expf, SQ_INSTS_VALU in profiles/r02h PMC passes).
template <int NTA, bool P2>  // key tiles per wave: ceil(ceil(T/32)/4) <= 4
__global__ __launch_bounds__(256) void relpos_attn_fwd_kernel(
    const float* __restrict__ qu, const float* __restrict__ qv, const float* __restrict__ kmat, long ldk,
    const float* __restrict__ pm, long ldpm, int nb, float sqrt_dk, const int* __restrict__ klen,
    float* __restrict__ attn, float* __restrict__ pdrop, uint32_t thr, float dscale, uint64_t seed, int T, long lds,
    int WP, const uint64_t* __restrict__ key) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sbd = smem;                  // [32][WP]
  float* rmax = smem + RP_ROWS * WP;  // [4 waves][32 rows]
  float* rsum = rmax + 4 * RP_ROWS;
  seed = esp::keyed(seed, key);
  const int z = blockIdx.y;
  const int i0 = blockIdx.x * RP_ROWS;
  const int head = z / nb, b = z - head * nb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hf = lane >> 5, l32 = lane & 31;
  const int P = 2 * T - 1;
  const int kmin = T - RP_ROWS - i0;
  const int nbd = (T + RP_ROWS - 1 + 31) / 32;
  const int nac = (T + 31) / 32;
  const float inv_sqrt_dk = 1.0f / sqrt_dk;

  auto load_row32 = [&](const float* row, float (&f)[2][16]) {  // d = 32c + 16hf + s
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(row + 32 * c + 16 * hf + 4 * u);
        f[c][4 * u] = v.x; f[c][4 * u + 1] = v.y; f[c][4 * u + 2] = v.z; f[c][4 * u + 3] = v.w;
      }
  };
  auto mfma_tile = [&](const float (&a)[2][16], const float (&bb)[2][16]) {
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int st = 0; st < 16; ++st) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c][st], bb[c][st], acc, 0, 0, 0);
    return acc;
  };

  // Every B fragment of a phase is requested before its first MFMA (one exposed latency per
  // phase, not per tile); phase 2's key rows are requested as phase 1's tiles retire.
  float aq[2][16], au[2][16], bq[4][2][16];
  auto p_row = [&](int ct) { return pm + (long)min(max(kmin + ct * 32 + l32, 0), P - 1) * ldpm + head * RP_DK; };
  auto k_row = [&](int ct) { return kmat + ((long)b * T + min(ct * 32 + l32, T - 1)) * ldk + head * RP_DK; };
  // 1. bd band window -> LDS  (nbd <= 15: at most 4 tiles per wave)
  load_row32(qv + ((long)z * T + min(i0 + l32, T - 1)) * RP_DK, aq);
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (wave + 4 * t < nbd) load_row32(p_row(wave + 4 * t), bq[t]);
  load_row32(qu + ((long)z * T + min(i0 + l32, T - 1)) * RP_DK, au);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ct = wave + 4 * t;
    if (ct < nbd) {
      const f32x16 acc = mfma_tile(aq, bq[t]);
      if (t < NTA && ct < nac) load_row32(k_row(ct), bq[t]);  // phase-2 key rows of the same slot
#pragma unroll
      for (int r = 0; r < 16; ++r) sbd[((r & 3) + 8 * (r >> 2) + 4 * hf) * WP + ct * 32 + l32] = acc[r];
    } else if (t < NTA && ct < nac) {
      load_row32(k_row(ct), bq[t]);
    }
  }
  int kl = klen ? klen[b] : T;
  if (kl > T) kl = T;
  __syncthreads();

  // 2. ac tiles + score assembly in registers
  f32x16 sc[NTA];
#pragma unroll
  for (int t = 0; t < NTA; ++t) {
    const int ct = wave + 4 * t;
    const int j = ct * 32 + l32;
    if (ct < nac) {
      const f32x16 acc = mfma_tile(au, bq[t]);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int il = (r & 3) + 8 * (r >> 2) + 4 * hf;
        const float sv = acc[r] + sbd[il * WP + j - il + RP_ROWS - 1];
        sc[t][r] = (j < kl) ? (P2 ? sv * inv_sqrt_dk : sv / sqrt_dk) : -INFINITY;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[t][r] = -INFINITY;
    }
  }
  // 3. row max (rows of register r: il(r)); lanes of a half share rows, differ in key
  float m[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = sc[0][r];
#pragma unroll
    for (int t = 1; t < NTA; ++t) v = fmaxf(v, sc[t][r]);
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    m[r] = v;
  }
  if (l32 == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) rmax[wave * RP_ROWS + (r & 3) + 8 * (r >> 2) + 4 * hf] = m[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int il = (r & 3) + 8 * (r >> 2) + 4 * hf;
    m[r] = fmaxf(fmaxf(rmax[il], rmax[RP_ROWS + il]), fmaxf(rmax[2 * RP_ROWS + il], rmax[3 * RP_ROWS + il]));
  }
  float sm[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = 0.f;
#pragma unroll
    for (int t = 0; t < NTA; ++t) {
      const float e = sc[t][r] == -INFINITY ? 0.f
                      : (P2 ? __builtin_amdgcn_exp2f((sc[t][r] - m[r]) * 1.4426950408889634f) : expf(sc[t][r] - m[r]));
      sc[t][r] = e;
      v += e;
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
    sm[r] = v;
  }
  if (l32 == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) rsum[wave * RP_ROWS + (r & 3) + 8 * (r >> 2) + 4 * hf] = sm[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int il = (r & 3) + 8 * (r >> 2) + 4 * hf;
    const float tot = (rsum[il] + rsum[RP_ROWS + il]) + (rsum[2 * RP_ROWS + il] + rsum[3 * RP_ROWS + il]);
    sm[r] = tot > 0.f ? 1.0f / tot : 0.f;
  }
#pragma unroll
  for (int t = 0; t < NTA; ++t) {
    const int j = (wave + 4 * t) * 32 + l32;
    if (j >= T) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * hf;
      if (i >= T) continue;
      const long row = (long)z * T + i;
      const float pe = sc[t][r] * sm[r];
      attn[row * lds + j] = pe;
      if (pdrop) pdrop[row * lds + j] = esp::keep_elem(seed, (uint64_t)(row * T + j), thr) ? pe * dscale : 0.f;
    }
  }
}

// ---------------------------------------------------------------- rel-pos attention probabilities, one wave per 16 rows
// Same result as relpos_attn_fwd_kernel, restructured so that no block-level synchronisation
// serialises the phases: each wave owns (z, 16 query rows) and walks the key tiles of 16 with
// v_mfma_f32_16x16x4_f32, holding its full score rows in registers (4 per tile per lane).
// Per key tile t:
//   ac(t)    = q_u[i0..i0+15] . k[16t..16t+15]                         (16 MFMAs, registers)
//   band(t+1)= q_v[i0..i0+15] . p[kb0+16(t+1) .. +15]                   (16 MFMAs, interleaved)
//   the band block goes to a per-wave 32-position LDS ring; the rel_shift read of tile t,
//   bd_shift[ii][jj] = band[ii][jj - ii + 15] (offset from block t), touches blocks t and t+1.
// The next tile's k / p fragments are fetched one tile ahead (64 B contiguous per lane, k order
// permuted identically in both operands: lane quarter q supplies d = 16 (c / 4) + 4 q + c % 4 at step c).
// Legacy rel_shift (attention.py:145-165): j <= i reads band rows q_v[i]; j == i+1 is 0;
// j >= i+2 reads q_v[i+1] . p[j-i-2].  In table positions k = j + T-1-i the first case is k < T,
// the last k > T with p at k - T - 1, and band block m covers T-16-16g+16m + [0,16) (g = i0/16):
// blocks m <= g lie wholly below T (A rows q_v[i]), blocks m >= g+1 wholly at or above T (A rows
// q_v[i+1], the shifted twin), so legacy selects the A operand per block and shares the ring.
// LDS: ring rows of RW_PITCH floats (row groups r and r+4 of a 32-lane half 16 banks apart).
// XS = 1 (the bf16 mode, esp_set_gemm_compute(1): every product of that step on bf16 operands): the ac
// and band products on v_mfma_f32_16x16x32_bf16 of the RNE-rounded operands with fp32 accumulation
// (torch autocast's bf16 matmul).  A lane's 16 values of a row (d = 16 q4 + [0,16)) are the two
// k-halves of the 16x16x32 operand (MFMA m takes d = 16 q4 + 8 m + [0, 8)); the output layout is the
// 16x16x4 one, so the ring, softmax and stores are shared with the f32 form (XS = 0).  (A bf16x6
// split-product form of the fp32 scores was measured slower, 441 vs 414 us at C2 B=128 -- the kernel
// is not bound by its MFMAs, DESIGN 3.4 -- and removed in round 5.)
typedef __attribute__((ext_vector_type(8))) __bf16 attn_bf16x8;
struct Frag16 {
  attn_bf16x8 v[2];  // [k-half]
};
__device__ __forceinline__ void split_frag(const float (&f)[16], Frag16& o) {
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    uint32_t h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) h[j] = esp::bf16_pair(f[8 * m + 2 * j], f[8 * m + 2 * j + 1]);
    o.v[m] = __builtin_bit_cast(attn_bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  }
}
__device__ __forceinline__ f32x4 mfma_np(const Frag16& a, const Frag16& b, f32x4 c) {
#pragma unroll
  for (int m = 0; m < 2; ++m) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v[m], b.v[m], c, 0, 0, 0);
  return c;
}

// 1 (default): T' <= 384 runs relpos_probs_lds_kernel (block-staged operands, split products); 0: the
// per-wave kernel for every T' (an A/B build: make VARIANT=_w EXTRA=-DESP_ATTN_PROBS_LDS=0)
#ifndef ESP_ATTN_PROBS_LDS
#define ESP_ATTN_PROBS_LDS 1
#endif
// staging steps in flight in relpos_probs_lds_kernel (2: 573 us per C2 B=256 launch, 1: 639)
#ifndef ESP_ATTN_PREFETCH
#define ESP_ATTN_PREFETCH 3
#endif

constexpr int RW_ROWS = 16, RW_PITCH = 37;
// store-transpose rows: 64 floats, so the float4 read-back (ds_read_b128 lane groups of 16 lanes over
// two rows, bank (a/4) mod 64) is conflict-free, with the column XOR-ed by 16 in rows 4..7 and 12..15
// so the two row groups of a ds_write_b32 half land 16 banks apart too (68: the reads conflicted 2-way)
constexpr int RW_SPITCH = 64;
// SPLIT = 2 (the bf16 mode's legacy rel_shift past 16 key tiles): a row group's keys are shared by
// two waves of the block (tiles [0, NTA) and [NTA, 2 NTA)), half the score registers each; the row
// max and sum are combined through LDS with one block barrier each.  (As an fp32 option it measured
// 398 vs 395 us at C2 B=128 and was removed in round 5.)
template <int NTA, bool P2, bool LEGACY, int SPLIT = 1, int XS = 0>  // SPLIT * NTA >= ceil(T/16) key tiles
__global__ __launch_bounds__(256, 2) void relpos_attn_fwd16_kernel(
    const float* __restrict__ qu, const float* __restrict__ qv, const float* __restrict__ kmat, long ldk,
    const float* __restrict__ pm, long ldpm, int nb, float sqrt_dk, const int* __restrict__ klen,
    float* __restrict__ attn, float* __restrict__ pdrop, uint32_t thr, float dscale, uint64_t seed, int T, long lds,
    const uint64_t* __restrict__ key, const int* __restrict__ tvalid, int nrb, int Z) {
  __shared__ float ring[4][RW_ROWS * RW_PITCH];
  __shared__ __attribute__((aligned(16))) float stage[4][RW_ROWS * RW_SPITCH];
  __shared__ float xch[2][4][RW_ROWS];  // SPLIT 2: per-wave row max / row sum partials
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // XCD-aware block order (1-D grid, blocks dealt round-robin over the 8 XCDs): the nrb row blocks of
  // one (head, utterance) z run on one XCD, so z's k rows and the head's p table are fetched into that
  // XCD's L2 once instead of once per XCD
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3, zq = jb / nrb;
  const int z = zq * 8 + xcd, bx = jb - zq * nrb;
  if (z >= Z) return;  // the whole block (nothing has synchronised yet)
  const int i0 = (SPLIT == 1 ? bx * 4 + wave : bx * 2 + (wave >> 1)) * RW_ROWS;
  const int t0 = SPLIT == 1 ? 0 : (wave & 1) * NTA;  // first key tile of this wave
  if (SPLIT == 1 && i0 >= T) return;  // the whole wave: nothing below synchronises the block
  seed = esp::keyed(seed, key);
  const int head = z / nb, b = z - head * nb;
  const int li = lane & 15, q4 = lane >> 4;
  const int g = i0 >> 4;
  // legacy rel_shift length: the reference batch's T' (tvalid) when the batch is padded to a
  // length bucket -- its table positions j + T'-1-i depend on T' (the latest ones, i - j, do not);
  // rows i >= T' are padding (finite, never read by a valid row), their positions are clamped
  const int Ts = LEGACY ? legacy_tv(tvalid, T) : T;
  const int kb0 = Ts - RW_ROWS - i0;  // table position of band block 0, column 0
  const int P = LEGACY ? T : 2 * T - 1;
  const float inv_sqrt_dk = 1.0f / sqrt_dk;
  float* ring0 = ring[wave];

  // a lane's 16 values of a row: d = 16 u + 4 q4 + (0..3) for u = 0..3, so each of the four float4
  // loads covers 64 contiguous bytes of a row across the lane quarter (16 rows x 64 B per instruction;
  // d = 16 q4 + 0..15 touched 16 rows x 4 separate 16-B pieces).  Any d order serves the MFMAs as long
  // as q, k and p share it (every operand is loaded here).
  auto ld16 = [&](const float* row, float (&f)[16]) {
    const float4* r4 = reinterpret_cast<const float4*>(row + 4 * q4);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 v = r4[4 * u];
      f[4 * u] = v.x; f[4 * u + 1] = v.y; f[4 * u + 2] = v.z; f[4 * u + 3] = v.w;
    }
  };
  auto k_row = [&](int t) { return kmat + ((long)b * T + min(t * 16 + li, T - 1)) * ldk + head * RP_DK; };
  auto p_row = [&](int m) {
    int pos = kb0 + 16 * m + li;
    if (LEGACY && pos > Ts) pos -= Ts + 1;  // the shifted band's table: p[j - i - 2]
    return pm + (long)min(max(pos, 0), P - 1) * ldpm + head * RP_DK;
  };
  float au[16], av[16], av2[16];
  ld16(qu + ((long)z * T + min(i0 + li, T - 1)) * RP_DK, au);
  ld16(qv + ((long)z * T + min(i0 + li, T - 1)) * RP_DK, av);
  if (LEGACY && !XS) ld16(qv + ((long)z * T + min(i0 + 1 + li, T - 1)) * RP_DK, av2);
  // XS: the query rows' split planes (once per wave).  Legacy: the band's A rows switch from q_v[i]
  // to q_v[i+1] once, at block g+1, and never back, so xv is re-split from the shifted rows at that
  // tile (one exposed load per wave) instead of holding both rows' planes
  Frag16 xu, xv;
  if constexpr (XS) {
    split_frag(au, xu);
    split_frag(av, xv);
  }
  int kl = klen ? klen[b] : T;
  if (kl > T) kl = T;

  auto put_band = [&](float* rg, int m, const f32x4& s) {
#pragma unroll
    for (int r = 0; r < 4; ++r) rg[(4 * q4 + r) * RW_PITCH + ((16 * m + li) & 31)] = s[r];
  };
  // fragments DEPTH tiles ahead: K(t) in kb[t % NB], band-block p rows P(m) in pb[m % NB]
  // (split: 3 waves per SIMD hide a tile less)
  constexpr int DEPTH = SPLIT == 2 ? 1 : 2, NB = DEPTH + 1;
  float kb[NB][16], pb[NB][16];  // indexed by the tile / block offset from t0
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) ld16(k_row(t0 + d), kb[d]);
#pragma unroll
  for (int d = 0; d <= DEPTH; ++d) ld16(p_row(t0 + d), pb[d]);
  {  // band block t0 (block 0 lies below T for every g: A rows q_v[i] in both variants)
    const bool shifted = LEGACY && t0 > g;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if constexpr (XS) {
      Frag16 pf6;
      split_frag(pb[0], pf6);
      if (shifted) {  // (SPLIT 2: a second-half wave whose keys all lie past the switch)
        ld16(qv + ((long)z * T + min(i0 + 1 + li, T - 1)) * RP_DK, av2);
        split_frag(av2, xv);
      }
      s = mfma_np(xv, pf6, s);
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        s = __builtin_amdgcn_mfma_f32_16x16x4f32(shifted ? av2[c] : av[c], pb[0][c], s, 0, 0, 0);
    }
    put_band(ring0, t0, s);
  }

  f32x4 sc[NTA];
#pragma unroll
  for (int tt = 0; tt < NTA; ++tt) {
    const int t = t0 + tt;
    // no `t < nt` branch: tiles past the last key are computed on clamped rows and masked
    // (j >= T > kl), which keeps every s_waitcnt vmcnt counted across the whole unrolled loop
    // (a conditional tile makes the compiler merge its counts pessimistically: vmcnt(4) at every
    // tile, i.e. the prefetched fragments waited for one tile early)
    {
      // the fragments DEPTH tiles ahead are requested first, into the buffers the previous tile
      // released, so a fetch has DEPTH whole tiles of this wave's work to arrive
      ld16(k_row(t + DEPTH), kb[(tt + DEPTH) % NB]);  // clamped rows: always safe to fetch
      ld16(p_row(t + 1 + DEPTH), pb[(tt + 1 + DEPTH) % NB]);
      const float(&kf)[16] = kb[tt % NB];
      const float(&pf)[16] = pb[(tt + 1) % NB];
      const bool shifted = LEGACY && t + 1 > g;  // legacy band block t+1 at/above table position T
      f32x4 a = {0.f, 0.f, 0.f, 0.f}, s = {0.f, 0.f, 0.f, 0.f};
      if constexpr (XS) {
        Frag16 kf6, pf6;
        split_frag(kf, kf6);
        split_frag(pf, pf6);
        if (LEGACY && t == g) {  // block t+1 = g+1: the first shifted band block
          ld16(qv + ((long)z * T + min(i0 + 1 + li, T - 1)) * RP_DK, av2);
          split_frag(av2, xv);
        }
        a = mfma_np(xu, kf6, a);
        s = mfma_np(xv, pf6, s);
      } else {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          a = __builtin_amdgcn_mfma_f32_16x16x4f32(au[c], kf[c], a, 0, 0, 0);
          s = __builtin_amdgcn_mfma_f32_16x16x4f32(shifted ? av2[c] : av[c], pf[c], s, 0, 0, 0);
        }
      }
      put_band(ring0, t + 1, s);
      asm volatile("" ::: "memory");  // ring writes before the shifted reads (LDS is in order per wave)
      const int j = t * 16 + li;
      // the four shifted band reads first, then their uses: one LDS round trip per tile (reads
      // interleaved with their uses cost a round trip each, `s_waitcnt lgkmcnt(0)` after every read)
      float bdv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = 4 * q4 + r;
        bdv[r] = ring0[ii * RW_PITCH + ((t * 16 + li - ii + 15) & 31)];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = 4 * q4 + r, i = i0 + ii;
        float bd = bdv[r];
        if (LEGACY && j == i + 1) bd = 0.f;
        const float sv = a[r] + bd;
        sc[tt][r] = j < kl ? (P2 ? sv * inv_sqrt_dk : sv / sqrt_dk) : -INFINITY;
      }
      asm volatile("" ::: "memory");  // ... and these reads before the next tile's ring writes
    }
  }

  // softmax over each row: a row's keys sit in the 16 lanes of one quarter x NTA tiles
  float nm[4], inv[4];  // -max * log2(e) (P2) or -max, and 1 / sum
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = sc[0][r];
#pragma unroll
    for (int t = 1; t < NTA; ++t) v = fmaxf(v, sc[t][r]);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    nm[r] = v;
  }
  if constexpr (SPLIT == 2) {  // combine with the partner wave's half of the keys
    if (li == 0)
#pragma unroll
      for (int r = 0; r < 4; ++r) xch[0][wave][4 * q4 + r] = nm[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) nm[r] = fmaxf(nm[r], xch[0][wave ^ 1][4 * q4 + r]);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float v = nm[r] == -INFINITY ? 0.f : nm[r];  // fully masked row: every e below is exp(-inf) = 0
    nm[r] = P2 ? -v * 1.4426950408889634f : -v;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = 0.f;
#pragma unroll
    for (int t = 0; t < NTA; ++t) {
      const float x = sc[t][r];
      const float e = P2 ? __builtin_amdgcn_exp2f(fmaf(x, 1.4426950408889634f, nm[r])) : expf(x + nm[r]);
      sc[t][r] = e;
      v += e;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
    inv[r] = v;
  }
  if constexpr (SPLIT == 2) {
    if (li == 0)
#pragma unroll
      for (int r = 0; r < 4; ++r) xch[1][wave][4 * q4 + r] = inv[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // the two halves in a fixed order (lower key half first)
      const float o = xch[1][wave ^ 1][4 * q4 + r];
      inv[r] = (wave & 1) ? o + inv[r] : inv[r] + o;
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) inv[r] = inv[r] > 0.f ? 1.0f / inv[r] : 0.f;
  // probabilities -> HBM through a per-wave LDS transpose, 64 columns (4 key tiles) at a time:
  // lane L then holds 4 consecutive columns of row 4p + (L >> 4), so one store instruction writes
  // 4 rows x 256 contiguous bytes (instead of 4 rows x 64 B from the accumulator layout).  A quad
  // that straddles T also writes the row pitch's padding columns (p = 0 there: keys >= T are
  // masked), so every store is a whole float4 and the only guard is j < T.
  float* stg = stage[wave];
  const int sr = lane >> 4, sc4 = 4 * (lane & 15);
  float* abase[4];
  float* dbase[4];
  uint64_t ibase[4];
  bool rok[4];
#pragma unroll
  for (int ps = 0; ps < 4; ++ps) {
    const int i = i0 + 4 * ps + sr;
    rok[ps] = i < T;
    const long row = (long)z * T + min(i, T - 1);
    abase[ps] = attn + row * lds + sc4;
    dbase[ps] = pdrop ? pdrop + row * lds + sc4 : nullptr;
    ibase[ps] = (uint64_t)(row * T + sc4);
  }
  const bool even_T = (T & 1) == 0;  // uniform
  // every dropout index of the launch (z*T + i)*T + j below 2^32 (uniform): 32-bit hash inputs,
  // the same masks (keep_pair32)
  const bool idx32 = (uint64_t)Z * (uint64_t)T * (uint64_t)T <= 0xffffffffull;
  auto store_rows = [&](auto drop_c) {
    constexpr bool DROP = decltype(drop_c)::value;
#pragma unroll
    for (int t4 = 0; t4 < NTA; t4 += 4) {
      if (16 * (t0 + t4) >= T) break;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) stg[(4 * q4 + r) * RW_SPITCH + ((16 * tt + li) ^ (16 * (q4 & 1)))] = sc[t4 + tt][r] * inv[r];
      asm volatile("" ::: "memory");
      const bool jok = 16 * (t0 + t4) + sc4 < T;
#pragma unroll
      for (int ps = 0; ps < 4; ++ps) {
        const float4 v = *reinterpret_cast<const float4*>(stg + (4 * ps + sr) * RW_SPITCH + (sc4 ^ (16 * (ps & 1))));
        if (rok[ps] && jok) {
          float* ar = abase[ps] + 16 * (t0 + t4);
          *reinterpret_cast<float4*>(ar) = v;
          if (DROP) {
            const uint64_t ix = ibase[ps] + 16 * (t0 + t4);
            float4 d;
            bool k0, k1, k2, k3;
            if (even_T && idx32) {  // row * T even: the quad is two hash pairs
              esp::keep_pair32(seed, (uint32_t)ix, thr, k0, k1);
              esp::keep_pair32(seed, (uint32_t)ix + 2, thr, k2, k3);
            } else if (even_T) {
              esp::keep_pair(seed, ix, thr, k0, k1);
              esp::keep_pair(seed, ix + 2, thr, k2, k3);
            } else {
              k0 = esp::keep_elem(seed, ix, thr);
              k1 = esp::keep_elem(seed, ix + 1, thr);
              k2 = esp::keep_elem(seed, ix + 2, thr);
              k3 = esp::keep_elem(seed, ix + 3, thr);
            }
            d.x = k0 ? v.x * dscale : 0.f;
            d.y = k1 ? v.y * dscale : 0.f;
            d.z = k2 ? v.z * dscale : 0.f;
            d.w = k3 ? v.w * dscale : 0.f;
            *reinterpret_cast<float4*>(dbase[ps] + 16 * (t0 + t4)) = d;
          }
        }
      }
      asm volatile("" ::: "memory");  // the reads above before the next chunk's writes
    }
  };
  if (pdrop) store_rows(std::true_type{});
  else store_rows(std::false_type{});
}

// ---------------------------------------------------------------- rel-pos probabilities, block-staged operands
// Round 5: the same result layout and softmax / dropout / store tail as relpos_attn_fwd16_kernel,
// with the per-tile operands staged ONCE per block instead of fetched by every wave:
// * a block = 4 waves = 64 consecutive query rows of one (head, utterance) z; at key tile t every
//   wave needs key tile t, and wave w the band block of table positions pbase + 16 (t - w) + [0,16)
//   (pbase = T' - i_block: the four waves' band windows are one block apart), so per step the block
//   takes in ONE key tile and ONE new band block (4 KB each: a float4 per thread), splits each value
//   once into its bf16 planes (split3_pair; the bf16 mode: the bf16 value alone) and writes them to
//   LDS rings (key tiles: 2 slots; band blocks: 5 -- the four waves read blocks t-3..t while t+1 is
//   written); one block barrier per tile;
// * the ac and band products on v_mfma_f32_16x16x32_bf16 from those planes: NP = 6 the six split
//   products of the GEMM family's fp32 arithmetic (hi.hi + hi.mid + mid.hi + hi.lo + lo.hi + mid.mid,
//   smallest first; fp32-accurate, gemm_kernels.h PREC 0), NP = 1 the bf16 mode's single product.
//   The query rows are split once per wave in registers.  Per tile and wave 24 (NP 6) MFMAs of 16
//   cycles instead of 32 f32 MFMAs of 32 cycles, and no per-wave global fragment fetch (DESIGN 3.4:
//   the fetches and the f32 MFMA issue were the kernel's two costs besides its stores).
// Plane image of a 16-row tile: row r (64 bf16 = 128 B = 8 chunks of 16 B) holds chunk c at
// c ^ swz16(r); a lane (li, q4) of MFMA m reads chunk 2 q4 + m of row li -- conflict-free ds_read_b128
// for every 16-lane group (rows of one parity take distinct chunks; the XOR only uses bits {0, 2}).
__device__ __forceinline__ int swz16(int r) { return ((r >> 1) & 1) | (r & 4); }
template <int NPL>
struct FragPl {
  attn_bf16x8 v[NPL][2];  // [plane hi, mid, lo][MFMA m: dims 16 q4 + 8 m + 0..7]
};
template <int NPL>
__device__ __forceinline__ void split_row16(const float (&f)[16], FragPl<NPL>& o) {
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    uint32_t h[4], md[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (NPL == 3) esp::split3_pair(f[8 * m + 2 * j], f[8 * m + 2 * j + 1], h[j], md[j], l[j]);
      else h[j] = esp::bf16_pair(f[8 * m + 2 * j], f[8 * m + 2 * j + 1]);
    }
    o.v[0][m] = __builtin_bit_cast(attn_bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
    if constexpr (NPL == 3) {
      o.v[1][m] = __builtin_bit_cast(attn_bf16x8, make_uint4(md[0], md[1], md[2], md[3]));
      o.v[2][m] = __builtin_bit_cast(attn_bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
    }
  }
}
template <int NPL>
__device__ __forceinline__ void read_frag_pl(const uint8_t* tile, int plane_bytes, int li, int q4, FragPl<NPL>& o) {
#pragma unroll
  for (int p = 0; p < NPL; ++p)
#pragma unroll
    for (int m = 0; m < 2; ++m)
      o.v[p][m] = *reinterpret_cast<const attn_bf16x8*>(tile + p * plane_bytes + li * 128 + (((2 * q4 + m) ^ swz16(li)) << 4));
}
// c += a . b over the 64 dims: NPL 3 the six split products smallest first per 32-dim half, NPL 1 hi.hi
template <int NPL>
__device__ __forceinline__ f32x4 mfma_pl(const FragPl<NPL>& a, const FragPl<NPL>& b, f32x4 c) {
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    if constexpr (NPL == 3) {
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v[1][m], b.v[1][m], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v[2][m], b.v[0][m], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v[0][m], b.v[2][m], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v[1][m], b.v[0][m], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v[0][m], b.v[1][m], c, 0, 0, 0);
    }
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v[0][m], b.v[0][m], c, 0, 0, 0);
  }
  return c;
}

// LDS slot schedule of relpos_probs_lds_kernel (the audit of VERDICT r5 'next' 7; PF, the register prefetch
// depth, does not touch LDS):
//   kpl[2]   key tile t lives in kpl[t & 1].  Written: tile 0 in the prologue, tile t+1 at the end of step t.
//            Readers of the slot it replaces (tile t-1): every wave in step t-1, all before the block barrier
//            that ends step t-1 -- the write comes after that barrier.  Step t reads kpl[t & 1] only.
//   ppl[5]   band block u lives in ppl[pslot(u)] = ppl[u mod 5]; wave w reads block t - w at step t
//            (u = t-3..t over the block) and block -1 - w in the prologue.  Written: blocks -4..0 in the
//            prologue, block t+1 at the end of step t into the slot of block t-4, whose readers are wave w
//            at step t-4+w (w = 0..3), i.e. steps t-4..t-1, all before the barrier ending step t-1; step t
//            reads blocks t-3..t, none in that slot.  The one reuse outside the loop: step 0 writes block 1
//            into pslot(-4), which wave 3 read in the prologue -- the block barrier after the prologue's
//            band read orders it (round-5 fix).
//   ring[w], stage[w]: per wave (LDS is in order within a wave; asm memory fences keep the compiler from
//            reordering the ring writes / reads).  Legacy: the block writes every wave's shifted-row plane
//            image into stage[w] in the prologue (thread -> row sr of all four images), the block barrier after
//            the prologue orders those writes before wave w reads its image into xv2 (before the key loop);
//            after that only wave w touches stage[w] (the store transpose after the loop).
// ESP_ATTN_SLOT_CHECK=1 (a separate build: make VARIANT=_slotchk EXTRA=-DESP_ATTN_SLOT_CHECK=1, loaded with
// ESP_LIB_VARIANT=_slotchk) checks this at run time: each slot carries a per-wave generation word in LDS --
// set to BUSY before a wave writes its rows of the slot and to the block / tile index after -- and every
// fragment read checks all four words equal the expected index before AND after the read, so a write that
// overlaps the read in any order is seen; mismatches are counted in g_attn_slot_err (vector stores only) and
// read back by esp_attn_slot_check_errors().
#ifndef ESP_ATTN_SLOT_CHECK
#define ESP_ATTN_SLOT_CHECK 0
#endif
#if ESP_ATTN_SLOT_CHECK
__device__ int g_attn_slot_err[64];
#endif
template <int NTA, bool P2, bool LEGACY, int NP>  // NTA >= ceil(T / 16) key tiles; NP 6 (fp32) or 1 (bf16)
__global__ __launch_bounds__(256, 2) void relpos_probs_lds_kernel(
    const float* __restrict__ qu, const float* __restrict__ qv, const float* __restrict__ kmat, long ldk,
    const float* __restrict__ pm, long ldpm, int nb, float sqrt_dk, const int* __restrict__ klen,
    float* __restrict__ attn, float* __restrict__ pdrop, uint32_t thr, float dscale, uint64_t seed, int T, long lds,
    const uint64_t* __restrict__ key, const int* __restrict__ tvalid, int nrb, int Z) {
  constexpr int NPL = NP == 6 ? 3 : 1;
  constexpr int PLB = RW_ROWS * 128;  // bytes of one plane of a 16-row tile
  constexpr int PSL = 5;              // band-block ring slots
  __shared__ __attribute__((aligned(16))) uint8_t kpl[2][NPL * PLB];
  __shared__ __attribute__((aligned(16))) uint8_t ppl[PSL][NPL * PLB];
  __shared__ float ring[4][RW_ROWS * RW_PITCH];
  // per wave: the store transpose after the loop; legacy: before it, the plane image of the wave's shifted
  // rows q_v[i+1] (split once in the prologue, read at step g -- a split inside the unrolled loop spilled)
  constexpr int STG = LEGACY && NPL * PLB / 4 > RW_ROWS * RW_SPITCH ? NPL * PLB / 4 : RW_ROWS * RW_SPITCH;
  __shared__ __attribute__((aligned(16))) float stage[4][STG];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware block order, as relpos_attn_fwd16_kernel: a z's row blocks on one XCD
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3, zq = jb / nrb;
  const int z = zq * 8 + xcd, bx = jb - zq * nrb;
  if (z >= Z) return;  // the whole block (nothing has synchronised yet)
  const int ib = bx * 4 * RW_ROWS;  // the block's first query row
  const int i0 = ib + wave * RW_ROWS;
  // (a wave whose rows all lie past T still stages and synchronises with the block; it stores nothing)
  seed = esp::keyed(seed, key);
  const int head = z / nb, b = z - head * nb;
  const int li = lane & 15, q4 = lane >> 4;
  const int g = i0 >> 4;
  const int Ts = LEGACY ? legacy_tv(tvalid, T) : T;
  const int P = LEGACY ? T : 2 * T - 1;
  const int pbase = Ts - ib;  // band block u: table positions pbase + 16 u + [0, 16)
  const float inv_sqrt_dk = 1.0f / sqrt_dk;
  float* ring0 = ring[wave];
  auto pslot = [](int u) { return ((u % PSL) + PSL) % PSL; };
#if ESP_ATTN_SLOT_CHECK
  __shared__ int kgen[2][4], pgen[PSL][4];
  constexpr int BUSY = -0x7fffffff;
  auto mark = [&](int* gw, int v) {  // this wave's generation word of a slot (before / after its rows)
    asm volatile("" ::: "memory");
    if (lane == 0) gw[wave] = v;
    asm volatile("" ::: "memory");
  };
  auto check = [&](const int* gw, int v, int where) {
    asm volatile("" ::: "memory");
    bool bad = false;
#pragma unroll
    for (int w = 0; w < 4; ++w) bad |= gw[w] != v;
    asm volatile("" ::: "memory");
    if (bad) g_attn_slot_err[lane] = 1 + where;  // (vector store; no printf: it multiplies the unrolled code)
  };
#define ESP_SLOT_MARK(g, v) mark(g, v)
#define ESP_SLOT_CHECK(g, v, w) check(g, v, w)
#else
#define ESP_SLOT_MARK(g, v) ((void)0)
#define ESP_SLOT_CHECK(g, v, w) ((void)0)
#endif

  // staging: thread -> row sr of the tile, dims sd..sd+3 (one float4; 16 threads per 256-B row)
  const int sr = tid >> 4, sd = 4 * (tid & 15);
  const int woff = sr * 128 + (((sd >> 3) ^ swz16(sr)) << 4) + ((sd >> 2) & 1) * 8;
  auto k_src = [&](int t) {
    return reinterpret_cast<const float4*>(kmat + ((long)b * T + min(t * 16 + sr, T - 1)) * ldk + head * RP_DK + sd);
  };
  auto p_src = [&](int u) {
    int pos = pbase + 16 * u + sr;
    if (LEGACY && pos > Ts) pos -= Ts + 1;  // the shifted band's table: p[j - i - 2]
    return reinterpret_cast<const float4*>(pm + (long)min(max(pos, 0), P - 1) * ldpm + head * RP_DK + sd);
  };
  auto put_tile = [&](uint8_t* dst, const float4 v) {
    if constexpr (NPL == 3) {
      uint32_t h0, m0, l0, h1, m1, l1;
      esp::split3_pair(v.x, v.y, h0, m0, l0);
      esp::split3_pair(v.z, v.w, h1, m1, l1);
      *reinterpret_cast<uint2*>(dst + woff) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(dst + PLB + woff) = make_uint2(m0, m1);
      *reinterpret_cast<uint2*>(dst + 2 * PLB + woff) = make_uint2(l0, l1);
    } else {
      *reinterpret_cast<uint2*>(dst + woff) = make_uint2(esp::bf16_pair(v.x, v.y), esp::bf16_pair(v.z, v.w));
    }
  };
  {  // prologue: band blocks u = -4..0 (wave w starts at u = -1 - w) and key tile 0
    float4 pv[PSL];
#pragma unroll
    for (int s = 0; s < PSL; ++s) pv[s] = *p_src(s - 4);
    const float4 kv = *k_src(0);
#pragma unroll
    for (int s = 0; s < PSL; ++s) {
      ESP_SLOT_MARK(pgen[pslot(s - 4)], BUSY);
      put_tile(ppl[pslot(s - 4)], pv[s]);
      ESP_SLOT_MARK(pgen[pslot(s - 4)], s - 4);
    }
    ESP_SLOT_MARK(kgen[0], BUSY);
    put_tile(kpl[0], kv);
    ESP_SLOT_MARK(kgen[0], 0);
    if constexpr (LEGACY) {  // wave w's shifted rows q_v[ib + 16 w + 1 + r] as a plane image in stage[w]
      float4 sv[4];
#pragma unroll
      for (int w = 0; w < 4; ++w)
        sv[w] = *reinterpret_cast<const float4*>(qv + ((long)z * T + min(ib + 16 * w + 1 + sr, T - 1)) * RP_DK + sd);
#pragma unroll
      for (int w = 0; w < 4; ++w) put_tile(reinterpret_cast<uint8_t*>(stage[w]), sv[w]);
    }
  }
  // the wave's query rows (d = 16 q4 + 0..15, contiguous: the plane images' order), split once
  auto ld16c = [&](const float* row, float (&f)[16]) {
    const float4* r4 = reinterpret_cast<const float4*>(row + 16 * q4);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 v = r4[u];
      f[4 * u] = v.x; f[4 * u + 1] = v.y; f[4 * u + 2] = v.z; f[4 * u + 3] = v.w;
    }
  };
  FragPl<NPL> xu, xv;
  {
    float f[16];
    ld16c(qu + ((long)z * T + min(i0 + li, T - 1)) * RP_DK, f);
    split_row16(f, xu);
    ld16c(qv + ((long)z * T + min(i0 + li, T - 1)) * RP_DK, f);
    split_row16(f, xv);
  }
  int kl = klen ? klen[b] : T;
  if (kl > T) kl = T;
  auto put_band = [&](float* rg, int m, const f32x4& s) {
#pragma unroll
    for (int r = 0; r < 4; ++r) rg[(4 * q4 + r) * RW_PITCH + ((16 * m + li) & 31)] = s[r];
  };
  __syncthreads();
  {  // band block 0 of this wave (u = -1 - w; below T for every g: A rows q_v[i] in both variants)
    FragPl<NPL> pf;
    ESP_SLOT_CHECK(pgen[pslot(-1 - wave)], -1 - wave, 0);
    read_frag_pl(ppl[pslot(-1 - wave)], PLB, li, q4, pf);
    ESP_SLOT_CHECK(pgen[pslot(-1 - wave)], -1 - wave, 1);
    put_band(ring0, 0, mfma_pl(xv, pf, f32x4{0.f, 0.f, 0.f, 0.f}));
  }
  // wave 3 read block -4 here, whose slot (pslot(-4) == pslot(1)) step 0 refills with block 1: every
  // wave's prologue read completes before any wave's step-0 ring write (without this barrier a wave
  // that ran ahead could overwrite it while wave 3 still read it -- rare, order-dependent bd errors on
  // the block's last 16 rows at key tile 0)
  __syncthreads();

  FragPl<NPL> xv2;  // legacy: the shifted rows' fragment, from the stage image
  if constexpr (LEGACY) read_frag_pl(reinterpret_cast<const uint8_t*>(stage[wave]), PLB, li, q4, xv2);
  f32x4 sc[NTA];
  // key tiles / band blocks PF steps ahead in registers (slot s % PF holds step s's): a step's loads
  // have PF steps of work to arrive before they are split into LDS
  // (legacy at depth 2: 651 vs 618 us with the spilling loop, profiles/r06f_kernel_summary_legacy_b256_pf2_nobits.txt)
  constexpr int PF = ESP_ATTN_PREFETCH;
  float4 nk[PF], np[PF];
#pragma unroll
  for (int s = 1; s < PF; ++s)
    if (s < NTA) {
      nk[s % PF] = *k_src(s);
      np[s % PF] = *p_src(s);
    }
#pragma unroll
  for (int t = 0; t < NTA; ++t) {
    if (t + PF < NTA) {
      nk[t % PF] = *k_src(t + PF);
      np[t % PF] = *p_src(t + PF);
    }
    FragPl<NPL> kf, pf;
    ESP_SLOT_CHECK(kgen[t & 1], t, 2);
    ESP_SLOT_CHECK(pgen[pslot(t - wave)], t - wave, 3);
    read_frag_pl(kpl[t & 1], PLB, li, q4, kf);
    read_frag_pl(ppl[pslot(t - wave)], PLB, li, q4, pf);
    ESP_SLOT_CHECK(kgen[t & 1], t, 4);
    ESP_SLOT_CHECK(pgen[pslot(t - wave)], t - wave, 5);
    const f32x4 a = mfma_pl(xu, kf, f32x4{0.f, 0.f, 0.f, 0.f});
    f32x4 s;
    if constexpr (LEGACY) {
      // band blocks t+1 >= g+1 (the shifted part) take the A rows q_v[i+1]: a per-step select, branch-free
      // (a branch at t == g in the unrolled loop split it into 24 scheduling regions: 42 VGPRs spilled, 618
      // vs 521 us; re-reading the fragment from LDS every step and selecting it: 596 vs 581 us microbench,
      // profiles/r06g_probs.log)
      FragPl<NPL> xa;
      const bool sw = t >= g;
#pragma unroll
      for (int p_ = 0; p_ < NPL; ++p_)
#pragma unroll
        for (int m_ = 0; m_ < 2; ++m_) xa.v[p_][m_] = sw ? xv2.v[p_][m_] : xv.v[p_][m_];
      s = mfma_pl(xa, pf, f32x4{0.f, 0.f, 0.f, 0.f});
    } else {
      s = mfma_pl(xv, pf, f32x4{0.f, 0.f, 0.f, 0.f});
    }
    put_band(ring0, t + 1, s);
    asm volatile("" ::: "memory");  // ring writes before the shifted reads (LDS is in order per wave)
    const int j = t * 16 + li;
    float bdv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = 4 * q4 + r;
      bdv[r] = ring0[ii * RW_PITCH + ((t * 16 + li - ii + 15) & 31)];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = 4 * q4 + r, i = i0 + ii;
      float bd = bdv[r];
      if (LEGACY && j == i + 1) bd = 0.f;
      const float sv = a[r] + bd;
      sc[t][r] = j < kl ? (P2 ? sv * inv_sqrt_dk : sv / sqrt_dk) : -INFINITY;
    }
    asm volatile("" ::: "memory");  // ... and these reads before the next tile's ring writes
    if (t + 1 < NTA) {
      ESP_SLOT_MARK(kgen[(t + 1) & 1], BUSY);
      put_tile(kpl[(t + 1) & 1], nk[(t + 1) % PF]);
      ESP_SLOT_MARK(kgen[(t + 1) & 1], t + 1);
      ESP_SLOT_MARK(pgen[pslot(t + 1)], BUSY);
      put_tile(ppl[pslot(t + 1)], np[(t + 1) % PF]);
      ESP_SLOT_MARK(pgen[pslot(t + 1)], t + 1);
      __syncthreads();  // step t+1's planes written; every wave done reading the slots they replaced
    }
  }

  // softmax over each row: a row's keys sit in the 16 lanes of one quarter x NTA tiles
  float nm[4], inv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = sc[0][r];
#pragma unroll
    for (int t = 1; t < NTA; ++t) v = fmaxf(v, sc[t][r]);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    v = v == -INFINITY ? 0.f : v;  // fully masked row: every e below is exp(-inf) = 0
    nm[r] = P2 ? -v * 1.4426950408889634f : -v;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = 0.f;
#pragma unroll
    for (int t = 0; t < NTA; ++t) {
      const float x = sc[t][r];
      const float e = P2 ? __builtin_amdgcn_exp2f(fmaf(x, 1.4426950408889634f, nm[r])) : expf(x + nm[r]);
      sc[t][r] = e;
      v += e;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
    inv[r] = v > 0.f ? 1.0f / v : 0.f;
  }
  // probabilities -> HBM through the per-wave LDS transpose (relpos_attn_fwd16_kernel's tail)
  float* stg = stage[wave];
  const int sr2 = lane >> 4, sc4 = 4 * (lane & 15);
  float* abase[4];
  float* dbase[4];
  uint64_t ibase[4];
  bool rok[4];
#pragma unroll
  for (int ps = 0; ps < 4; ++ps) {
    const int i = i0 + 4 * ps + sr2;
    rok[ps] = i < T;
    const long row = (long)z * T + min(i, T - 1);
    abase[ps] = attn + row * lds + sc4;
    dbase[ps] = pdrop ? pdrop + row * lds + sc4 : nullptr;
    ibase[ps] = (uint64_t)(row * T + sc4);
  }
  const bool even_T = (T & 1) == 0;
  const bool idx32 = (uint64_t)Z * (uint64_t)T * (uint64_t)T <= 0xffffffffull;
  auto store_rows = [&](auto drop_c) {
    constexpr bool DROP = decltype(drop_c)::value;
#pragma unroll
    for (int t4 = 0; t4 < NTA; t4 += 4) {
      if (16 * t4 >= T) break;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) stg[(4 * q4 + r) * RW_SPITCH + ((16 * tt + li) ^ (16 * (q4 & 1)))] = sc[t4 + tt][r] * inv[r];
      asm volatile("" ::: "memory");
      const bool jok = 16 * t4 + sc4 < T;
#pragma unroll
      for (int ps = 0; ps < 4; ++ps) {
        const float4 v = *reinterpret_cast<const float4*>(stg + (4 * ps + sr2) * RW_SPITCH + (sc4 ^ (16 * (ps & 1))));
        if (rok[ps] && jok) {
          *reinterpret_cast<float4*>(abase[ps] + 16 * t4) = v;
          if (DROP) {
            const uint64_t ix = ibase[ps] + 16 * t4;
            float4 d;
            bool k0, k1, k2, k3;
            if (even_T && idx32) {
              esp::keep_pair32(seed, (uint32_t)ix, thr, k0, k1);
              esp::keep_pair32(seed, (uint32_t)ix + 2, thr, k2, k3);
            } else if (even_T) {
              esp::keep_pair(seed, ix, thr, k0, k1);
              esp::keep_pair(seed, ix + 2, thr, k2, k3);
            } else {
              k0 = esp::keep_elem(seed, ix, thr);
              k1 = esp::keep_elem(seed, ix + 1, thr);
              k2 = esp::keep_elem(seed, ix + 2, thr);
              k3 = esp::keep_elem(seed, ix + 3, thr);
            }
            d.x = k0 ? v.x * dscale : 0.f;
            d.y = k1 ? v.y * dscale : 0.f;
            d.z = k2 ? v.z * dscale : 0.f;
            d.w = k3 ? v.w * dscale : 0.f;
            *reinterpret_cast<float4*>(dbase[ps] + 16 * t4) = d;
          }
        }
      }
      asm volatile("" ::: "memory");
    }
  };
  if (pdrop) store_rows(std::true_type{});
  else store_rows(std::false_type{});
#undef ESP_SLOT_MARK
#undef ESP_SLOT_CHECK
}

inline int gridn(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 65536 ? 65536 : (b < 1 ? 1 : b));
}

}  // namespace

// the slot-check build's mismatch count since the last call (then reset); -1 in every other build
ESP_API int esp_attn_slot_check_errors(void) {
#if ESP_ATTN_SLOT_CHECK
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  int h[64];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_attn_slot_err), sizeof h) != hipSuccess) return -2;
  int n = 0;
  for (int i = 0; i < 64; ++i) n += h[i] != 0;
  const int zeros[64] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_attn_slot_err), zeros, sizeof zeros) != hipSuccess) return -2;
  return n;
#else
  return -1;
#endif
}

ESP_API int esp_heads_split(const float* src, long ld, int col0, int B, int T, int H, int dk, const float* bias,
                            float* dst, void* stream) {
  hipLaunchKernelGGL(heads_split_kernel, dim3(gridn((long)H * B * T * dk)), dim3(256), 0, (hipStream_t)stream, src, ld,
                     col0, B, T, H, dk, bias, dst);
  ESP_CHECK_LAUNCH("esp_heads_split");
  return 0;
}

ESP_API int esp_heads_split2(const float* src, long ld, int col0, int B, int T, int H, int dk, const float* bias_a,
                             float* dst_a, const float* bias_b, float* dst_b, void* stream) {
  ESP_ARG_CHECK(dk % 4 == 0 && ld % 4 == 0 && col0 % 4 == 0 && ((uintptr_t)src & 15) == 0 &&
                    ((uintptr_t)dst_a & 15) == 0 && ((uintptr_t)dst_b & 15) == 0 && ((uintptr_t)bias_a & 15) == 0 &&
                    ((uintptr_t)bias_b & 15) == 0,
                "esp_heads_split2: 16-B aligned operands with dk, ld, col0 multiples of 4 required");
  hipLaunchKernelGGL(heads_split2_kernel, dim3(gridn((long)H * B * T * dk / 4)), dim3(256), 0, (hipStream_t)stream,
                     src, ld, col0, B, T, H, dk, bias_a, dst_a, bias_b, dst_b);
  ESP_CHECK_LAUNCH("esp_heads_split2");
  return 0;
}

ESP_API int esp_attn_bwd_prep(const float* dctx, long ldd, const float* ctx, long ldc, int nb, int H, int dk, int T,
                              float* dot, float* dbd, long ldp, int relpos, void* stream) {
  ESP_ARG_CHECK(relpos == 1 || relpos == 2, "esp_attn_bwd_prep: relpos must be 1 or 2");
  ESP_ARG_CHECK(T >= 1 && nb >= 1 && H >= 1 && dk >= 1 && ldp >= (relpos == 1 ? 2 * T - 1 : T),
                "esp_attn_bwd_prep: bad sizes");
  const long rows = (long)nb * H * T;
  hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, dctx,
                     ldd, ctx, ldc, nb, H, dk, T, dot, dbd, ldp, relpos);
  ESP_CHECK_LAUNCH("esp_attn_bwd_prep");
  return 0;
}

ESP_API int esp_add2d(const float* x, long ldx, float* y, long ldy, int M, int N, void* stream) {
  hipLaunchKernelGGL(add2d_kernel, dim3(gridn((long)M * N)), dim3(256), 0, (hipStream_t)stream, x, ldx, y, ldy, M, N);
  ESP_CHECK_LAUNCH("esp_add2d");
  return 0;
}

// relpos: 0 none, 1 latest (P=2T-1), 2 legacy (P=T). ac may alias attn (in-place).
// lds: row pitch of ac/attn/pdrop (>= Tk), ldp: row pitch of bd (>= P).
ESP_API int esp_attn_softmax_fwd(const float* ac, const float* bd, int relpos, int P, float sqrt_dk, const int* klen,
                                 int nb, int causal, float* attn, float* pdrop, float drop_p, unsigned long long seed,
                                 int Z, int Tq, int Tk, long lds, long ldp, const int* tvalid, void* stream) {
  ESP_ARG_CHECK(Tk >= 1, "esp_attn_softmax_fwd: Tk=%d", Tk);
  ESP_ARG_CHECK(relpos == 0 || (Tq == Tk && bd), "esp_attn_softmax_fwd: rel-pos needs Tq==Tk and bd");
  ESP_ARG_CHECK(relpos != 1 || P == 2 * Tq - 1, "esp_attn_softmax_fwd: latest rel-pos needs P=2T-1");
  ESP_ARG_CHECK(relpos != 2 || P == Tq, "esp_attn_softmax_fwd: legacy rel-pos needs P=T");
  ESP_ARG_CHECK(lds >= Tk && (relpos == 0 || ldp >= P), "esp_attn_softmax_fwd: pitch < row length");
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  if (!thr) pdrop = nullptr;
  const float ds = esp::drop_scale(thr);
  const long rows = (long)Z * Tq;
  dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
#define ESP_SM(PER)                                                                                                 \
  hipLaunchKernelGGL(softmax_fwd_kernel<PER>, grid, dim3(256), 0, st, ac, bd, relpos, P, sqrt_dk, klen, nb, causal, \
                     attn, pdrop, thr, ds, (uint64_t)seed, Z, Tq, Tk, lds, ldp, esp::rng_key_ptr(), tvalid)
  if (Tk <= 64) ESP_SM(1);
  else if (Tk <= 128) ESP_SM(2);
  else if (Tk <= 256) ESP_SM(4);
  else if (Tk <= 512) ESP_SM(8);
  else if (Tk <= 1024) ESP_SM(16);
  else
    hipLaunchKernelGGL(softmax_fwd_loop_kernel, grid, dim3(256), 0, st, ac, bd, relpos, P, sqrt_dk, klen, nb, causal,
                       attn, pdrop, thr, ds, (uint64_t)seed, Z, Tq, Tk, lds, ldp, esp::rng_key_ptr(), tvalid);
#undef ESP_SM
  ESP_CHECK_LAUNCH("esp_attn_softmax_fwd");
  return 0;
}

ESP_API int esp_attn_softmax_bwd(const float* attn, const float* dP, float* dS, float drop_p, unsigned long long seed,
                                 float sqrt_dk, long rows, int Tk, long lds, void* stream) {
  ESP_ARG_CHECK(Tk >= 1, "esp_attn_softmax_bwd: Tk=%d", Tk);
  ESP_ARG_CHECK(lds >= Tk, "esp_attn_softmax_bwd: pitch < Tk");
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  const float ds = esp::drop_scale(thr);
  dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
#define ESP_SB(PER) \
  hipLaunchKernelGGL(softmax_bwd_kernel<PER>, grid, dim3(256), 0, st, attn, dP, dS, thr, ds, (uint64_t)seed, sqrt_dk, rows, Tk, lds, esp::rng_key_ptr())
  if (Tk <= 64) ESP_SB(1);
  else if (Tk <= 128) ESP_SB(2);
  else if (Tk <= 256) ESP_SB(4);
  else if (Tk <= 512) ESP_SB(8);
  else if (Tk <= 1024) ESP_SB(16);
  else
    hipLaunchKernelGGL(softmax_bwd_loop_kernel<0>, grid, dim3(256), 0, st, attn, dP, dS, nullptr, 0L, thr, ds,
                       (uint64_t)seed, sqrt_dk, rows, Tk, lds, esp::rng_key_ptr(), nullptr);
#undef ESP_SB
  ESP_CHECK_LAUNCH("esp_attn_softmax_bwd");
  return 0;
}

ESP_API int esp_relshift_bwd(const float* dS, long lds, float* dbd, long ldp, int relpos, int Z, int T, int P,
                             void* stream) {
  ESP_ARG_CHECK(relpos == 1 || relpos == 2, "esp_relshift_bwd: relpos must be 1 or 2");
  ESP_ARG_CHECK(lds >= T && ldp >= P, "esp_relshift_bwd: pitch < row length");
  hipLaunchKernelGGL(relshift_bwd_kernel, dim3(gridn((long)Z * T * P)), dim3(256), 0, (hipStream_t)stream, dS, lds,
                     dbd, ldp, relpos, Z, T, P);
  ESP_CHECK_LAUNCH("esp_relshift_bwd");
  return 0;
}

// Fused latest rel-pos scores + softmax: q_v (Z,T,64) head-major (z = h*nb + b), p rows of
// length ldpm with head h at column 64h (P = 2T-1 rows), ac (Z,T) pitch lds -> attn (may
// alias ac) [+ dropout copy pdrop].
ESP_API int esp_relpos_softmax_fwd(const float* qv, const float* p, long ldp_row, int nb, int H, const float* ac,
                                   float sqrt_dk, const int* klen, float* attn, float* pdrop, float drop_p,
                                   unsigned long long seed, int T, long lds, void* stream) {
  ESP_ARG_CHECK(T >= 1 && T <= 1024 && lds >= T && nb >= 1 && H >= 1, "esp_relpos_softmax_fwd: bad sizes T=%d", T);
  ESP_ARG_CHECK(ldp_row % 4 == 0 && ((uintptr_t)p & 15) == 0 && ((uintptr_t)qv & 15) == 0,
                "esp_relpos_softmax_fwd: q_v / p must be 16-B aligned with ld %% 4 == 0");
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  if (!thr) pdrop = nullptr;
  const float ds = esp::drop_scale(thr);
  const int ntile = (T + RP_ROWS - 1 + 31) / 32;
  const int WP = ntile * 32 + 4;
  const size_t shm = (size_t)RP_ROWS * WP * sizeof(float);
  ESP_ARG_CHECK(shm <= 65536, "esp_relpos_softmax_fwd: T=%d needs %zu B of LDS (> 64 KB)", T, shm);
  dim3 grid((unsigned)((T + RP_ROWS - 1) / RP_ROWS), (unsigned)(nb * H));
  hipStream_t st = (hipStream_t)stream;
#define ESP_RP(PER)                                                                                              \
  hipLaunchKernelGGL(relpos_softmax_fwd_kernel<PER>, grid, dim3(256), shm, st, qv, p, ldp_row, nb, H, ac, sqrt_dk, \
                     klen, attn, pdrop, thr, ds, (uint64_t)seed, T, lds, WP, esp::rng_key_ptr())
  if (T <= 64) ESP_RP(1);
  else if (T <= 128) ESP_RP(2);
  else if (T <= 256) ESP_RP(4);
  else if (T <= 512) ESP_RP(8);
  else ESP_RP(16);
#undef ESP_RP
  ESP_CHECK_LAUNCH("esp_relpos_softmax_fwd");
  return 0;
}

// Fully fused latest rel-pos attention probabilities: ac = q_u k^T and the bd band both on the
// MFMA inside the kernel, softmax + dropout copy -> attn / pdrop (pitch lds).  q_u, q_v (Z,T,64)
// head-major; k rows at kmat + (b*T + j)*ldk + 64*head; p as in esp_relpos_softmax_fwd.
ESP_API int esp_relpos_attn_fwd(const float* qu, const float* qv, const float* kmat, long ldk, const float* p,
                                long ldp_row, int nb, int H, float sqrt_dk, const int* klen, float* attn, float* pdrop,
                                float drop_p, unsigned long long seed, int T, long lds, void* stream) {
  ESP_ARG_CHECK(T >= 1 && lds >= T && nb >= 1 && H >= 1, "esp_relpos_attn_fwd: bad sizes T=%d", T);
  ESP_ARG_CHECK(ldp_row % 4 == 0 && ldk % 4 == 0 && ((uintptr_t)p & 15) == 0 && ((uintptr_t)qv & 15) == 0 &&
                    ((uintptr_t)qu & 15) == 0 && ((uintptr_t)kmat & 15) == 0,
                "esp_relpos_attn_fwd: operands must be 16-B aligned with ld %% 4 == 0");
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  if (!thr) pdrop = nullptr;
  const float ds = esp::drop_scale(thr);
  const int nbd = (T + RP_ROWS - 1 + 31) / 32;
  const int WP = nbd * 32 + 4;
  const size_t shm = ((size_t)RP_ROWS * WP + 8 * RP_ROWS) * sizeof(float);
  ESP_ARG_CHECK(shm <= 65536, "esp_relpos_attn_fwd: T=%d needs %zu B of LDS (> 64 KB)", T, shm);
  const int nta = ((T + 31) / 32 + 3) / 4;
  dim3 grid((unsigned)((T + RP_ROWS - 1) / RP_ROWS), (unsigned)(nb * H));
  hipStream_t st = (hipStream_t)stream;
  const bool p2 = sqrt_dk > 0.f && (__builtin_bit_cast(uint32_t, sqrt_dk) & 0x7fffffu) == 0;
#define ESP_RA(N)                                                                                                    \
  do {                                                                                                               \
    if (p2)                                                                                                          \
      hipLaunchKernelGGL((relpos_attn_fwd_kernel<N, true>), grid, dim3(256), shm, st, qu, qv, kmat, ldk, p, ldp_row,  \
                         nb, sqrt_dk, klen, attn, pdrop, thr, ds, (uint64_t)seed, T, lds, WP, esp::rng_key_ptr());    \
    else                                                                                                             \
      hipLaunchKernelGGL((relpos_attn_fwd_kernel<N, false>), grid, dim3(256), shm, st, qu, qv, kmat, ldk, p, ldp_row, \
                         nb, sqrt_dk, klen, attn, pdrop, thr, ds, (uint64_t)seed, T, lds, WP, esp::rng_key_ptr());    \
  } while (0)
  if (nta <= 1) ESP_RA(1);
  else if (nta == 2) ESP_RA(2);
  else if (nta == 3) ESP_RA(3);
  else ESP_RA(4);
#undef ESP_RA
  ESP_CHECK_LAUNCH("esp_relpos_attn_fwd");
  return 0;
}

// Rel-pos attention probabilities, latest (relpos 1, P = 2T-1 table rows) or legacy (relpos 2,
// P = T rows), one wave per 16 query rows (relpos_attn_fwd16_kernel).  T <= 512.
ESP_API int esp_relpos_attn_probs(const float* qu, const float* qv, const float* kmat, long ldk, const float* p,
                                  long ldp_row, int relpos, int nb, int H, float sqrt_dk, const int* klen,
                                  float* attn, float* pdrop, float drop_p, unsigned long long seed, int T, long lds,
                                  const int* tvalid, void* stream) {
  ESP_ARG_CHECK(T >= 1 && T <= 512 && lds >= T && nb >= 1 && H >= 1, "esp_relpos_attn_probs: bad sizes T=%d", T);
  ESP_ARG_CHECK(relpos == 1 || relpos == 2, "esp_relpos_attn_probs: relpos must be 1 (latest) or 2 (legacy)");
  ESP_ARG_CHECK(lds % 4 == 0 && ((uintptr_t)attn & 15) == 0 && ((uintptr_t)pdrop & 15) == 0,
                "esp_relpos_attn_probs: attn / pdrop rows must be 16-B aligned (whole float4s are written, up to "
                "the pitch lds rounded to 4)");
  ESP_ARG_CHECK(ldp_row % 4 == 0 && ldk % 4 == 0 && ((uintptr_t)p & 15) == 0 && ((uintptr_t)qv & 15) == 0 &&
                    ((uintptr_t)qu & 15) == 0 && ((uintptr_t)kmat & 15) == 0,
                "esp_relpos_attn_probs: operands must be 16-B aligned with ld %% 4 == 0");
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  if (!thr) pdrop = nullptr;
  const float ds = esp::drop_scale(thr);
  const int nt = (T + 15) / 16;
  const int Zn = nb * H;
  int nrb = (T + 4 * RW_ROWS - 1) / (4 * RW_ROWS);  // row blocks per z (4 waves x 16 rows)
  dim3 grid((unsigned)(8 * ((Zn + 7) / 8) * nrb));  // XCD-aware order (see the kernel)
  hipStream_t st = (hipStream_t)stream;
  const bool p2 = sqrt_dk > 0.f && (__builtin_bit_cast(uint32_t, sqrt_dk) & 0x7fffffu) == 0;
  if (ESP_ATTN_PROBS_LDS && nt <= 24) {
    // block-staged operands, split products (relpos_probs_lds_kernel): fp32-accurate six products in
    // the fp32 mode, the single bf16 product in the bf16 mode (like every other product of its step)
    const bool b16 = esp_get_gemm_compute() == 1;
#define ESP_RL(N, P2_, L_, NP_)                                                                                     \
  hipLaunchKernelGGL((relpos_probs_lds_kernel<N, P2_, L_, NP_>), grid, dim3(256), 0, st, qu, qv, kmat, ldk, p,     \
                     ldp_row, nb, sqrt_dk, klen, attn, pdrop, thr, ds, (uint64_t)seed, T, lds, esp::rng_key_ptr(), \
                     tvalid, nrb, Zn)
#define ESP_RLN(N, P2_, L_)          \
  do {                               \
    if (b16) ESP_RL(N, P2_, L_, 1);  \
    else ESP_RL(N, P2_, L_, 6);      \
  } while (0)
#define ESP_RLT(N)                                 \
  do {                                             \
    if (relpos == 2) {                             \
      if (p2) ESP_RLN(N, true, true);              \
      else ESP_RLN(N, false, true);                \
    } else {                                       \
      if (p2) ESP_RLN(N, true, false);             \
      else ESP_RLN(N, false, false);               \
    }                                              \
  } while (0)
    if (nt <= 8) ESP_RLT(8);
    else if (nt <= 16) ESP_RLT(16);
    else ESP_RLT(24);
#undef ESP_RLT
#undef ESP_RLN
#undef ESP_RL
    ESP_CHECK_LAUNCH("esp_relpos_attn_probs");
    return 0;
  }
  // the bf16 mode computes the scores on bf16 operands like every other product of its step
  if (esp_get_gemm_compute() == 1) {
#define ESP_RX(N, P2_, L_)                                                                                         \
  hipLaunchKernelGGL((relpos_attn_fwd16_kernel<N, P2_, L_, 1, 1>), grid, dim3(256), 0, st, qu, qv, kmat, ldk, p, \
                     ldp_row, nb, sqrt_dk, klen, attn, pdrop, thr, ds, (uint64_t)seed, T, lds, esp::rng_key_ptr(),   \
                     tvalid, nrb, Zn)
#define ESP_RXN(N)                      \
  do {                                  \
    if (relpos == 2) {                  \
      if (p2) ESP_RX(N, true, true);    \
      else ESP_RX(N, false, true);      \
    } else {                            \
      if (p2) ESP_RX(N, true, false);   \
      else ESP_RX(N, false, false);     \
    }                                   \
  } while (0)
    if (nt <= 8) ESP_RXN(8);
    else if (nt <= 16) ESP_RXN(16);
    else if (relpos == 2) {
      // legacy: the row-shift re-split leaves no registers for 24+ score tiles per wave; two waves
      // share a row group's keys (SPLIT 2, half the score registers each)
      nrb = (T + 2 * RW_ROWS - 1) / (2 * RW_ROWS);
      grid.x = (unsigned)(8 * ((Zn + 7) / 8) * nrb);
      if (p2)
        hipLaunchKernelGGL((relpos_attn_fwd16_kernel<16, true, true, 2, 1>), grid, dim3(256), 0, st, qu, qv, kmat, ldk,
                           p, ldp_row, nb, sqrt_dk, klen, attn, pdrop, thr, ds, (uint64_t)seed, T, lds,
                           esp::rng_key_ptr(), tvalid, nrb, Zn);
      else
        hipLaunchKernelGGL((relpos_attn_fwd16_kernel<16, false, true, 2, 1>), grid, dim3(256), 0, st, qu, qv, kmat, ldk,
                           p, ldp_row, nb, sqrt_dk, klen, attn, pdrop, thr, ds, (uint64_t)seed, T, lds,
                           esp::rng_key_ptr(), tvalid, nrb, Zn);
    } else if (nt <= 24) ESP_RXN(24);
    else ESP_RXN(32);
#undef ESP_RXN
#undef ESP_RX
    ESP_CHECK_LAUNCH("esp_relpos_attn_probs");
    return 0;
  }
#define ESP_RW3(N, P2_, L_)                                                                                         \
  hipLaunchKernelGGL((relpos_attn_fwd16_kernel<N, P2_, L_>), grid, dim3(256), 0, st, qu, qv, kmat, ldk, p, ldp_row, \
                     nb, sqrt_dk, klen, attn, pdrop, thr, ds, (uint64_t)seed, T, lds, esp::rng_key_ptr(), tvalid, nrb, Zn)
#define ESP_RW(N)                             \
  do {                                        \
    if (relpos == 2) {                        \
      if (p2) ESP_RW3(N, true, true);         \
      else ESP_RW3(N, false, true);           \
    } else {                                  \
      if (p2) ESP_RW3(N, true, false);        \
      else ESP_RW3(N, false, false);          \
    }                                         \
  } while (0)
  if (nt <= 4) ESP_RW(4);
  else if (nt <= 8) ESP_RW(8);
  else if (nt <= 12) ESP_RW(12);
  else if (nt <= 16) ESP_RW(16);
  else if (nt <= 20) ESP_RW(20);
  else if (nt <= 24) ESP_RW(24);
  else if (nt <= 28) ESP_RW(28);
  else ESP_RW(32);
#undef ESP_RW
#undef ESP_RW3
  ESP_CHECK_LAUNCH("esp_relpos_attn_probs");
  return 0;
}

// softmax backward + latest rel_shift adjoint in one pass (see softmax_bwd_relpos_kernel)
// latest rel_shift, dbd written only on its band: dbd's other elements must already be 0 (a buffer kept
// for this use, zeroed once: the kernel never writes outside the band)
ESP_API int esp_attn_softmax_bwd_relpos_band(const float* attn, const float* dP, float* dS, float* dbd, long ldp,
                                             float drop_p, unsigned long long seed, float sqrt_dk, long rows, int T,
                                             long lds, void* stream) {
  ESP_ARG_CHECK(T >= 1 && T <= 1024 && lds >= T && lds % 4 == 0 && ldp >= 2 * T - 1 && rows % T == 0,
                "esp_attn_softmax_bwd_relpos_band: bad sizes");
  ESP_ARG_CHECK(((uintptr_t)attn & 15) == 0 && ((uintptr_t)dP & 15) == 0 && ((uintptr_t)dS & 15) == 0,
                "esp_attn_softmax_bwd_relpos_band: attn / dP / dS must be 16-B aligned");
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  const float ds = esp::drop_scale(thr);
  dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  const bool p2 = sqrt_dk > 0.f && (__builtin_bit_cast(uint32_t, sqrt_dk) & 0x7fffffu) == 0;
#define ESP_SBB(Q)                                                                                                 \
  do {                                                                                                             \
    if (p2)                                                                                                        \
      hipLaunchKernelGGL((softmax_bwd_relpos4_kernel<Q, 3, true>), grid, dim3(256), 0, st, attn, dP, dS, dbd, ldp,  \
                         thr, ds, (uint64_t)seed, sqrt_dk, rows, T, lds, esp::rng_key_ptr(), nullptr);             \
    else                                                                                                           \
      hipLaunchKernelGGL((softmax_bwd_relpos4_kernel<Q, 3, false>), grid, dim3(256), 0, st, attn, dP, dS, dbd, ldp, \
                         thr, ds, (uint64_t)seed, sqrt_dk, rows, T, lds, esp::rng_key_ptr(), nullptr);             \
  } while (0)
  if (T <= 256) ESP_SBB(1);
  else if (T <= 512) ESP_SBB(2);
  else ESP_SBB(4);
#undef ESP_SBB
  ESP_CHECK_LAUNCH("esp_attn_softmax_bwd_relpos_band");
  return 0;
}

ESP_API int esp_attn_softmax_bwd_relpos(const float* attn, const float* dP, float* dS, float* dbd, long ldp,
                                        int relpos, float drop_p, unsigned long long seed, float sqrt_dk, long rows,
                                        int T, long lds, const int* tvalid, void* stream) {
  ESP_ARG_CHECK(relpos == 1 || relpos == 2, "esp_attn_softmax_bwd_relpos: relpos must be 1 or 2");
  ESP_ARG_CHECK(T >= 1 && lds >= T && ldp >= (relpos == 1 ? 2 * T - 1 : T) && rows % T == 0,
                "esp_attn_softmax_bwd_relpos: bad sizes");
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  const float ds = esp::drop_scale(thr);
  dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  const bool p2 = sqrt_dk > 0.f && (__builtin_bit_cast(uint32_t, sqrt_dk) & 0x7fffffu) == 0;
  if (T <= 1024 && lds % 4 == 0 && ((uintptr_t)attn & 15) == 0 && ((uintptr_t)dP & 15) == 0 &&
      ((uintptr_t)dS & 15) == 0) {
#define ESP_SB4(Q, R)                                                                                             \
  do {                                                                                                            \
    if (p2)                                                                                                       \
      hipLaunchKernelGGL((softmax_bwd_relpos4_kernel<Q, R, true>), grid, dim3(256), 0, st, attn, dP, dS, dbd, ldp, \
                         thr, ds, (uint64_t)seed, sqrt_dk, rows, T, lds, esp::rng_key_ptr(), tvalid);                     \
    else                                                                                                          \
      hipLaunchKernelGGL((softmax_bwd_relpos4_kernel<Q, R, false>), grid, dim3(256), 0, st, attn, dP, dS, dbd,     \
                         ldp, thr, ds, (uint64_t)seed, sqrt_dk, rows, T, lds, esp::rng_key_ptr(), tvalid);                \
  } while (0)
#define ESP_SB4R(Q)              \
  do {                           \
    if (relpos == 1) ESP_SB4(Q, 1); \
    else ESP_SB4(Q, 2);          \
  } while (0)
    if (T <= 256) ESP_SB4R(1);
    else if (T <= 512) ESP_SB4R(2);
    else ESP_SB4R(4);
#undef ESP_SB4R
#undef ESP_SB4
    ESP_CHECK_LAUNCH("esp_attn_softmax_bwd_relpos");
    return 0;
  }
#define ESP_SBR(PER)                                                                                         \
  do {                                                                                                       \
    if (relpos == 1)                                                                                         \
      hipLaunchKernelGGL((softmax_bwd_relpos_kernel<PER, 1>), grid, dim3(256), 0, st, attn, dP, dS, dbd, ldp, \
                         thr, ds, (uint64_t)seed, sqrt_dk, rows, T, lds, esp::rng_key_ptr(), tvalid);                \
    else                                                                                                     \
      hipLaunchKernelGGL((softmax_bwd_relpos_kernel<PER, 2>), grid, dim3(256), 0, st, attn, dP, dS, dbd, ldp, \
                         thr, ds, (uint64_t)seed, sqrt_dk, rows, T, lds, esp::rng_key_ptr(), tvalid);                \
  } while (0)
  if (T <= 64) ESP_SBR(1);
  else if (T <= 128) ESP_SBR(2);
  else if (T <= 256) ESP_SBR(4);
  else if (T <= 512) ESP_SBR(8);
  else if (T <= 1024) ESP_SBR(16);
  else if (relpos == 1)
    hipLaunchKernelGGL(softmax_bwd_loop_kernel<1>, grid, dim3(256), 0, st, attn, dP, dS, dbd, ldp, thr, ds,
                       (uint64_t)seed, sqrt_dk, rows, T, lds, esp::rng_key_ptr(), tvalid);
  else
    hipLaunchKernelGGL(softmax_bwd_loop_kernel<2>, grid, dim3(256), 0, st, attn, dP, dS, dbd, ldp, thr, ds,
                       (uint64_t)seed, sqrt_dk, rows, T, lds, esp::rng_key_ptr(), tvalid);
#undef ESP_SBR
  ESP_CHECK_LAUNCH("esp_attn_softmax_bwd_relpos");
  return 0;
}

// Fused latest rel-pos attention backward (see relpos_attn_bwd_kernel): dctx rows at
// dctx + (b*T + i)*ldd + 64h, V rows at vmat + (b*T + j)*ldv + 64h; attn/dS pitch lds, dbd pitch ldp.
ESP_API int esp_relpos_attn_bwd(const float* dctx, long ldd, const float* vmat, long ldv, const float* attn,
                                float* dS, float* dbd, long ldp, int nb, int H, float sqrt_dk, float drop_p,
                                unsigned long long seed, int T, long lds, void* stream) {
  ESP_ARG_CHECK(T >= 1 && T <= 512 && lds >= T && ldp >= 2 * T - 1 && nb >= 1 && H >= 1,
                "esp_relpos_attn_bwd: bad sizes T=%d", T);
  ESP_ARG_CHECK(ldd % 4 == 0 && ldv % 4 == 0 && ((uintptr_t)dctx & 15) == 0 && ((uintptr_t)vmat & 15) == 0,
                "esp_relpos_attn_bwd: dctx / v must be 16-B aligned with ld %% 4 == 0");
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  const float ds = esp::drop_scale(thr);
  const int nta = ((T + 31) / 32 + 3) / 4;
  dim3 grid((unsigned)((T + RP_ROWS - 1) / RP_ROWS), (unsigned)(nb * H));
  hipStream_t st = (hipStream_t)stream;
#define ESP_RB(N)                                                                                                  \
  hipLaunchKernelGGL(relpos_attn_bwd_kernel<N>, grid, dim3(256), 0, st, dctx, ldd, vmat, ldv, attn, dS, dbd, ldp, nb, \
                     sqrt_dk, thr, ds, (uint64_t)seed, T, lds, esp::rng_key_ptr())
  if (nta <= 1) ESP_RB(1);
  else if (nta == 2) ESP_RB(2);
  else if (nta == 3) ESP_RB(3);
  else ESP_RB(4);
#undef ESP_RB
  ESP_CHECK_LAUNCH("esp_relpos_attn_bwd");
  return 0;
}
