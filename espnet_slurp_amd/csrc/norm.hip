// Normalisation / reduction kernels (HBM-bound): LayerNorm fwd/bwd (eps 1e-12,
// layer_norm.py:12-38), deterministic column sums (bias grads), the Conformer
// ConvolutionModule's GLU + depthwise Conv1d(k, pad (k-1)/2) + BatchNorm1d (training
// statistics over all B*T' rows, padded frames included) + Swish, fwd and bwd
// (conformer/convolution.py:56-79).  Row-major [rows][channels] everywhere; one wave per
// row for row reductions; column reductions go through per-block partials and a fixed-
// order finalize, so every result is bitwise reproducible run to run.
#include <initializer_list>

#include "common.h"

namespace {

constexpr int MAXD = 2048;  // max feature dim for LayerNorm (per-lane registers: MAXD/64)

// ----------------------------------------------------------------------------- LayerNorm
template <int PER>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, float* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + (long)row * D;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < D ? xr[c] : 0.f;
    s += v[i];
  }
  const float mean = esp::wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const float d = c < D ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float var = esp::wave_sum(q) / (float)D;
  const float rstd = 1.0f / sqrtf(var + eps);
  float* yr = y + (long)row * D;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    if (c < D) yr[c] = (v[i] - mean) * rstd * w[c] + b[c];
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// The same LayerNorm with y written as bf16 planes (n = 3: the exact split, esp::split3_pair; n = 1:
// bf16(y)) for the GEMMs that are its only readers (kernels.Planes).  A lane owns float4 quads
// (D % 4 == 0); y values, mean and rstd are those of ln_fwd_kernel (same sums, same order per row:
// the wave sums run over the same per-lane partials in a different lane assignment, so they can
// differ in the last bit -- both are exact-order wave reductions of the same row).
template <int PQ>
__global__ __launch_bounds__(256) void ln_fwd_planes_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ b, uint16_t* __restrict__ y,
                                                            long ldy, long ps, int n, float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out, int M, int D, float eps,
                                                            float* __restrict__ yf) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nq = D >> 2;
  const float4* xr = reinterpret_cast<const float4*>(x + (long)row * D);
  float4 v[PQ];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PQ; ++i) {
    const int q = lane + 64 * i;
    v[i] = q < nq ? xr[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = esp::wave_sum(s) / (float)D;
  float qs = 0.f;
#pragma unroll
  for (int i = 0; i < PQ; ++i) {
    const int q = lane + 64 * i;
    if (q < nq) {
      const float a = v[i].x - mean, bb = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
      qs += (a * a + bb * bb) + (c * c + d * d);
    }
  }
  const float var = esp::wave_sum(qs) / (float)D;
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < PQ; ++i) {
    const int q = lane + 64 * i;
    if (q >= nq) continue;
    const float4 wq = reinterpret_cast<const float4*>(w)[q], bq = reinterpret_cast<const float4*>(b)[q];
    const float4 o = make_float4((v[i].x - mean) * rstd * wq.x + bq.x, (v[i].y - mean) * rstd * wq.y + bq.y,
                                 (v[i].z - mean) * rstd * wq.z + bq.z, (v[i].w - mean) * rstd * wq.w + bq.w);
    esp::store_planes4(y, (long)row * ldy + 4 * q, ps, n, o.x, o.y, o.z, o.w);
    if (yf) reinterpret_cast<float4*>(yf + (long)row * D)[q] = o;  // (esp_layernorm_fwd_dual: y in fp32 too)
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx (+)= rstd * (g - mean(g) - xhat*mean(g*xhat)), g = dy*w; partial dw/db per block.
// A wave owns LN_RB consecutive rows per pass (their loads are all in flight before the first
// reduction: row-level ILP), float4 along the row (D % 4 == 0); a block covers
// LN_BWD_ROWS rows so that ~M/32 blocks keep every CU busy (the HBM roofline needs many
// rows in flight, a wave walking 16 rows one by one is latency-bound).
constexpr int LN_RB = 4, LN_BWD_ROWS = 32;
template <int PQ>  // float4 quads per lane: D <= 256 * PQ
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                     const float* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, float* __restrict__ dx,
                                                     int accumulate, float* __restrict__ part, int M, int D) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nq = D >> 2;
  __shared__ float4 sh[4][64];
  float4 pw[PQ], pb[PQ], wq[PQ];
#pragma unroll
  for (int i = 0; i < PQ; ++i) {
    pw[i] = pb[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int q = lane + 64 * i;
    wq[i] = q < nq ? reinterpret_cast<const float4*>(w)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int r0 = blockIdx.x * LN_BWD_ROWS;
  const int r1 = min(M, r0 + LN_BWD_ROWS);
  const float invD = 1.0f / (float)D;
  for (int base = r0 + wv * LN_RB; base < r1; base += 4 * LN_RB) {
    float4 xh[LN_RB][PQ], g[LN_RB][PQ];
    float s1[LN_RB], s2[LN_RB], rs[LN_RB];
#pragma unroll
    for (int j = 0; j < LN_RB; ++j) {
      const int row = base + j;
      const bool ok = row < r1;
      const float mu = ok ? mean_in[row] : 0.f;
      rs[j] = ok ? rstd_in[row] : 0.f;
      s1[j] = s2[j] = 0.f;
#pragma unroll
      for (int i = 0; i < PQ; ++i) {
        const int q = lane + 64 * i;
        float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), d = xv;
        if (ok && q < nq) {
          xv = reinterpret_cast<const float4*>(x + (long)row * D)[q];
          d = reinterpret_cast<const float4*>(dy + (long)row * D)[q];
        }
        float4 h;
        h.x = (xv.x - mu) * rs[j]; h.y = (xv.y - mu) * rs[j]; h.z = (xv.z - mu) * rs[j]; h.w = (xv.w - mu) * rs[j];
        float4 gg;
        gg.x = d.x * wq[i].x; gg.y = d.y * wq[i].y; gg.z = d.z * wq[i].z; gg.w = d.w * wq[i].w;
        pw[i].x += d.x * h.x; pw[i].y += d.y * h.y; pw[i].z += d.z * h.z; pw[i].w += d.w * h.w;
        pb[i].x += d.x; pb[i].y += d.y; pb[i].z += d.z; pb[i].w += d.w;
        s1[j] += (gg.x + gg.y) + (gg.z + gg.w);
        s2[j] += (gg.x * h.x + gg.y * h.y) + (gg.z * h.z + gg.w * h.w);
        xh[j][i] = h;
        g[j][i] = gg;
      }
    }
#pragma unroll
    for (int j = 0; j < LN_RB; ++j) {
      s1[j] = esp::wave_sum(s1[j]) * invD;
      s2[j] = esp::wave_sum(s2[j]) * invD;
    }
#pragma unroll
    for (int j = 0; j < LN_RB; ++j) {
      const int row = base + j;
      if (row >= r1) continue;
      float4* dxr = reinterpret_cast<float4*>(dx + (long)row * D);
#pragma unroll
      for (int i = 0; i < PQ; ++i) {
        const int q = lane + 64 * i;
        if (q >= nq) continue;
        float4 v;
        v.x = rs[j] * (g[j][i].x - s1[j] - xh[j][i].x * s2[j]);
        v.y = rs[j] * (g[j][i].y - s1[j] - xh[j][i].y * s2[j]);
        v.z = rs[j] * (g[j][i].z - s1[j] - xh[j][i].z * s2[j]);
        v.w = rs[j] * (g[j][i].w - s1[j] - xh[j][i].w * s2[j]);
        if (accumulate) {
          const float4 o = dxr[q];
          v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        dxr[q] = v;
      }
    }
  }
  // combine the 4 waves' column partials in fixed order: part[blk][0:D] = dw, [D:2D] = db
  float* pr = part + (long)blockIdx.x * 2 * D;
#pragma unroll
  for (int i = 0; i < PQ; ++i) {
    const int q = lane + 64 * i;
#pragma unroll
    for (int which = 0; which < 2; ++which) {
      __syncthreads();
      sh[wv][lane] = which ? pb[i] : pw[i];
      __syncthreads();
      if (wv == 0 && q < nq) {
        const float4 a = sh[0][lane], b = sh[1][lane], c = sh[2][lane], e = sh[3][lane];
        float4 t;
        t.x = ((a.x + b.x) + c.x) + e.x; t.y = ((a.y + b.y) + c.y) + e.y;
        t.z = ((a.z + b.z) + c.z) + e.z; t.w = ((a.w + b.w) + c.w) + e.w;
        reinterpret_cast<float4*>(pr + which * D)[q] = t;
      }
    }
  }
}

// out[c] (+)= sum_{p<nb} part[p*stride + c]   for c < N.  Block = 16 columns x 64 row groups (1024
// threads, grid N / 16: 4x the blocks of a 64-column block, each thread a quarter of the rows); a
// group sums rows g, g+64, ... into four interleaved accumulators (four loads in flight), combined in
// fixed order, then the 64 groups in fixed order (deterministic).  These are ~10-us latency-bound
// launches (80 + 48 per C2 step): with 64-column blocks a thread walked nb/16 dependent loads.
constexpr int FC_COLS = 16, FC_GROUPS = 64;
template <typename T>
__device__ __forceinline__ T fc_sum_rows(const T* __restrict__ part, int nb, long stride, int c, int g) {
  T s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int p = g;
  for (; p + 3 * FC_GROUPS < nb; p += 4 * FC_GROUPS) {
    s0 += part[(long)p * stride + c];
    s1 += part[(long)(p + FC_GROUPS) * stride + c];
    s2 += part[(long)(p + 2 * FC_GROUPS) * stride + c];
    s3 += part[(long)(p + 3 * FC_GROUPS) * stride + c];
  }
  for (; p < nb; p += FC_GROUPS) s0 += part[(long)p * stride + c];
  return (s0 + s1) + (s2 + s3);
}
template <typename T>
__device__ __forceinline__ T fc_block_sum(T s, int cl, int g, T (&sh)[FC_GROUPS][FC_COLS]) {
  sh[g][cl] = s;
  __syncthreads();
  T t = 0;
  if (g == 0)
    for (int k = 0; k < FC_GROUPS; ++k) t += sh[k][cl];
  return t;
}

template <typename T>
__global__ __launch_bounds__(1024) void finalize_cols_kernel(const T* __restrict__ part, int nb, long stride, int N,
                                                             float* __restrict__ out, int accumulate) {
  __shared__ T sh[FC_GROUPS][FC_COLS];
  const int cl = threadIdx.x % FC_COLS, g = threadIdx.x / FC_COLS;
  const int c = blockIdx.x * FC_COLS + cl;
  const T s = c < N ? fc_sum_rows(part, nb, stride, c, g) : (T)0;
  const T t = fc_block_sum(s, cl, g, sh);
  if (g == 0 && c < N) out[c] = accumulate ? out[c] + (float)t : (float)t;
}

// the same over 2*D columns of [nb][2D] partials, accumulated into out0 (c < D) / out1 (c >= D)
__global__ __launch_bounds__(1024) void finalize_cols2_kernel(const float* __restrict__ part, int nb, long stride, int D,
                                                              float* __restrict__ out0, float* __restrict__ out1) {
  __shared__ float sh[FC_GROUPS][FC_COLS];
  const int cl = threadIdx.x % FC_COLS, g = threadIdx.x / FC_COLS;
  const int c = blockIdx.x * FC_COLS + cl;
  const float s = c < 2 * D ? fc_sum_rows(part, nb, stride, c, g) : 0.f;
  const float t = fc_block_sum(s, cl, g, sh);
  if (g == 0 && c < 2 * D) {
    if (c < D) out0[c] += t;
    else out1[c - D] += t;
  }
}

// column partial sums of a [M][N] (ld) matrix: block = CS_ROWS rows x 256 columns; lane =
// column quad (float4 when vec), 4 waves interleave the rows, combined in fixed order.
constexpr int CS_ROWS = 32;
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ x, int M, int N, long ld, int vec,
                                                          float* __restrict__ part) {
  __shared__ float4 sh[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = (blockIdx.y * 64 + lane) * 4;
  const int r0 = blockIdx.x * CS_ROWS, r1 = min(M, r0 + CS_ROWS);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < N) {
    if (vec) {
#pragma unroll 4
      for (int r = r0 + wv; r < r1; r += 4) {
        const float4 v = *reinterpret_cast<const float4*>(x + (long)r * ld + c);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
    } else {
      for (int r = r0 + wv; r < r1; r += 4) {
        const float* xr = x + (long)r * ld + c;
        s.x += xr[0];
        if (c + 1 < N) s.y += xr[1];
        if (c + 2 < N) s.z += xr[2];
        if (c + 3 < N) s.w += xr[3];
      }
    }
  }
  sh[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && c < N) {
    const float4 a = sh[0][lane], b = sh[1][lane], d = sh[2][lane], e = sh[3][lane];
    float* pr = part + (long)blockIdx.x * N + c;
    pr[0] = ((a.x + b.x) + d.x) + e.x;
    if (c + 1 < N) pr[1] = ((a.y + b.y) + d.y) + e.y;
    if (c + 2 < N) pr[2] = ((a.z + b.z) + d.z) + e.z;
    if (c + 3 < N) pr[3] = ((a.w + b.w) + d.w) + e.w;
  }
}

// ----------------------------------------------------------------------------- conv module
// g = a * sigmoid(b), u = [a | b] (rows x 2D)   (F.glu(dim=channels))
__global__ void glu_fwd_kernel(const float* __restrict__ u, float* __restrict__ g, long rows, int D) {
  const long n = rows * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / D;
    const int c = (int)(i - r * D);
    const float a = u[r * 2 * D + c], b = u[r * 2 * D + D + c];
    g[i] = a * esp::fast_sigmoid(b);
  }
}

// float4 forms (D % 4 == 0, 16-B aligned, rows*D/4 < 2^31): one 32-bit division per 4 elements
// instead of a 64-bit division per element, hardware exp2 / rcp sigmoid
__global__ void glu_fwd4_kernel(const float* __restrict__ u, float* __restrict__ g, int rows, int D) {
  const int nq = D >> 2, n = rows * nq;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = i / nq, c = 4 * (i - r * nq);
    const float4 a = *reinterpret_cast<const float4*>(u + (long)r * 2 * D + c);
    const float4 b = *reinterpret_cast<const float4*>(u + (long)r * 2 * D + D + c);
    *reinterpret_cast<float4*>(g + (long)r * D + c) =
        make_float4(a.x * esp::fast_sigmoid(b.x), a.y * esp::fast_sigmoid(b.y), a.z * esp::fast_sigmoid(b.z),
                    a.w * esp::fast_sigmoid(b.w));
  }
}
__global__ void glu_bwd4_kernel(const float* __restrict__ u, const float* __restrict__ dg, float* __restrict__ du,
                                int rows, int D) {
  const int nq = D >> 2, n = rows * nq;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = i / nq, c = 4 * (i - r * nq);
    const float4 a = *reinterpret_cast<const float4*>(u + (long)r * 2 * D + c);
    const float4 b = *reinterpret_cast<const float4*>(u + (long)r * 2 * D + D + c);
    const float4 d = *reinterpret_cast<const float4*>(dg + (long)r * D + c);
    const float sx = esp::fast_sigmoid(b.x), sy = esp::fast_sigmoid(b.y), sz = esp::fast_sigmoid(b.z),
                sw = esp::fast_sigmoid(b.w);
    *reinterpret_cast<float4*>(du + (long)r * 2 * D + c) = make_float4(d.x * sx, d.y * sy, d.z * sz, d.w * sw);
    *reinterpret_cast<float4*>(du + (long)r * 2 * D + D + c) =
        make_float4(d.x * a.x * sx * (1.0f - sx), d.y * a.y * sy * (1.0f - sy), d.z * a.z * sz * (1.0f - sz),
                    d.w * a.w * sw * (1.0f - sw));
  }
}

// du written as bf16 planes (row pitch 2D, n = 3 exact split / 1 bf16) for pointwise_conv1's weight- and
// input-gradient GEMMs, its only readers (kernels.Planes)
__global__ void glu_bwd4_planes_kernel(const float* __restrict__ u, const float* __restrict__ dg,
                                       uint16_t* __restrict__ du, long ps, int np, int rows, int D) {
  const int nq = D >> 2, n = rows * nq;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = i / nq, c = 4 * (i - r * nq);
    const float4 a = *reinterpret_cast<const float4*>(u + (long)r * 2 * D + c);
    const float4 b = *reinterpret_cast<const float4*>(u + (long)r * 2 * D + D + c);
    const float4 d = *reinterpret_cast<const float4*>(dg + (long)r * D + c);
    const float sx = esp::fast_sigmoid(b.x), sy = esp::fast_sigmoid(b.y), sz = esp::fast_sigmoid(b.z),
                sw = esp::fast_sigmoid(b.w);
    esp::store_planes4(du, (long)r * 2 * D + c, ps, np, d.x * sx, d.y * sy, d.z * sz, d.w * sw);
    esp::store_planes4(du, (long)r * 2 * D + D + c, ps, np, d.x * a.x * sx * (1.0f - sx), d.y * a.y * sy * (1.0f - sy),
                       d.z * a.z * sz * (1.0f - sz), d.w * a.w * sw * (1.0f - sw));
  }
}

__global__ void glu_bwd_kernel(const float* __restrict__ u, const float* __restrict__ dg, float* __restrict__ du,
                               long rows, int D) {
  const long n = rows * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / D;
    const int c = (int)(i - r * D);
    const float a = u[r * 2 * D + c], b = u[r * 2 * D + D + c];
    const float s = esp::fast_sigmoid(b);
    const float d = dg[i];
    du[r * 2 * D + c] = d * s;
    du[r * 2 * D + D + c] = d * a * s * (1.0f - s);
  }
}

// Valid-frame bound of a length-bucketed batch (HIP-graph trainer): a batch padded to T frames
// per utterance whose true padded length is *tvalid < T.  The frames t >= *tvalid do not exist
// in the reference batch: the depthwise convolution reads them as its zero padding and writes
// 0 there, BatchNorm statistics and gradients exclude them (their gradient is 0).  NULL: all
// T frames are real.
__device__ __forceinline__ int valid_T(const int* tvalid, int T) { return tvalid ? min(T, *tvalid) : T; }

// y[b,t,c] = bias[c] + sum_k W[c,k] * x[b, t + k - pad, c]   (flip=0, forward)
// y[b,t,c] = sum_k W[c,k] * x[b, t - k + pad, c]             (flip=1, input grad)
// Block = 64 channels x DW_TT time steps; the input window (DW_TT + K - 1 rows) and the
// 64 filters are staged in LDS; a thread owns one channel and DW_TT/4 consecutive steps.
constexpr int DW_TT = 32, DW_KMAX = 64;
__global__ __launch_bounds__(256) void dwconv_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                     const float* __restrict__ bias, float* __restrict__ y, int Bn,
                                                     int T, int D, int K, int flip, const int* __restrict__ tvalid) {
  __shared__ float xs[DW_TT + DW_KMAX][64];
  const int Tv = valid_T(tvalid, T);
  __shared__ float ws[64][DW_KMAX + 1];
  const int c0 = blockIdx.x * 64, t0 = blockIdx.y * DW_TT, b = blockIdx.z;
  const int pad = (K - 1) / 2;
  const int cl = threadIdx.x & 63, tg = threadIdx.x >> 6;
  const int c = c0 + cl;
  const float* xb = x + (long)b * T * D;
  const int rows = DW_TT + K - 1;
  for (int r = tg; r < rows; r += 4) {
    const int t = t0 - pad + r;
    xs[r][cl] = (c < D && t >= 0 && t < Tv) ? xb[(long)t * D + c] : 0.f;
  }
  for (int e = threadIdx.x; e < 64 * K; e += 256) {
    const int cc = e / K, k = e - cc * K;
    ws[cc][k] = (c0 + cc < D) ? W[(long)(c0 + cc) * K + (flip ? (K - 1 - k) : k)] : 0.f;
  }
  __syncthreads();
  if (c >= D) return;
  constexpr int PT = DW_TT / 4;
  float acc[PT];
  const float bv = bias ? bias[c] : 0.f;
#pragma unroll
  for (int j = 0; j < PT; ++j) acc[j] = bv;
  const int base = tg * PT;
  for (int k = 0; k < K; ++k) {
    const float wk = ws[cl][k];
#pragma unroll
    for (int j = 0; j < PT; ++j) acc[j] += wk * xs[base + j + k][cl];
  }
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    const int t = t0 + base + j;
    if (t < T) y[((long)b * T + t) * D + c] = t < Tv ? acc[j] : 0.f;
  }
}

// dW[c,k] partials over a DWW_TCH-step time chunk: sum_t dy[b,t,c] * x[b,t+k-pad,c].
// Block = 64 channels; 4 tap groups (k = kg, kg+4, ...); dy and x windows in LDS.
constexpr int DWW_TCH = 64;
__global__ __launch_bounds__(256) void dwconv_wgrad_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                           float* __restrict__ part, int T, int D, int K,
                                                           const int* __restrict__ tvalid) {
  __shared__ float xs[DWW_TCH + DW_KMAX][64];
  const int Tv = valid_T(tvalid, T);
  __shared__ float gs[DWW_TCH][64];
  const int c0 = blockIdx.x * 64, ch = blockIdx.y, b = blockIdx.z, nch = gridDim.y;
  const int t0 = ch * DWW_TCH;
  const int pad = (K - 1) / 2;
  const int cl = threadIdx.x & 63, kg = threadIdx.x >> 6;
  const int c = c0 + cl;
  const float* xb = x + (long)b * T * D;
  const float* db = dy + (long)b * T * D;
  for (int r = kg; r < DWW_TCH + K - 1; r += 4) {
    const int t = t0 - pad + r;
    xs[r][cl] = (c < D && t >= 0 && t < Tv) ? xb[(long)t * D + c] : 0.f;
  }
  for (int r = kg; r < DWW_TCH; r += 4) {
    const int t = t0 + r;
    gs[r][cl] = (c < D && t < Tv) ? db[(long)t * D + c] : 0.f;
  }
  __syncthreads();
  if (c >= D) return;
  constexpr int KPT = DW_KMAX / 4;  // taps per thread (k = kg + 4i)
  float acc[KPT];
#pragma unroll
  for (int i = 0; i < KPT; ++i) acc[i] = 0.f;
  for (int t = 0; t < DWW_TCH; ++t) {
    const float g = gs[t][cl];
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int k = kg + 4 * i;
      if (k < K) acc[i] += g * xs[t + k][cl];
    }
  }
  float* pr = part + ((long)(b * nch + ch) * D + c) * K;
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    const int k = kg + 4 * i;
    if (k < K) pr[k] = acc[i];
  }
}

// Register-blocked variants for the common kernel sizes (cnn_module_kernel 31 / 15): a thread's
// PT outputs need PT + K - 1 inputs, read ONCE from LDS into a register window (the LDS-tiled
// kernels above read K*PT values per thread), filters in registers.
constexpr int DWR_PT = 16, DWR_TT = 4 * DWR_PT;  // outputs per thread, time steps per block
// rows t_lo .. t_lo + DWR_TT + KT - 2 of channels c0 .. c0+63 into LDS (zero outside [0,T) x [0,D)),
// float4 per lane: 16 lanes per row, 16 rows per pass of the 256-thread block
template <int KT>
__device__ __forceinline__ void dw_stage(float (*xs)[64], const float* __restrict__ xb, int t_lo, int T, int D,
                                         int c0) {
  const int q = threadIdx.x & 15, r0 = threadIdx.x >> 4;
  const int c = c0 + 4 * q;
  const bool vec = (D & 3) == 0 && c + 4 <= D;
  for (int r = r0; r < DWR_TT + KT - 1; r += 16) {
    const int t = t_lo + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t >= 0 && t < T) {
      const float* src = xb + (long)t * D + c;
      if (vec) {
        v = *reinterpret_cast<const float4*>(src);
      } else {
        if (c < D) v.x = src[0];
        if (c + 1 < D) v.y = src[1];
        if (c + 2 < D) v.z = src[2];
        if (c + 3 < D) v.w = src[3];
      }
    }
    *reinterpret_cast<float4*>(&xs[r][4 * q]) = v;
  }
}
template <int KT>
__global__ __launch_bounds__(256) void dwconv_rb_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                        const float* __restrict__ bias, float* __restrict__ y, int T,
                                                        int D, int flip, const int* __restrict__ tvalid) {
  __shared__ __attribute__((aligned(16))) float xs[DWR_TT + KT - 1][64];
  const int Tv = valid_T(tvalid, T);
  __shared__ float ws[KT][64];
  constexpr int pad = (KT - 1) / 2;
  const int c0 = blockIdx.x * 64, t0 = blockIdx.y * DWR_TT, b = blockIdx.z;
  const int cl = threadIdx.x & 63, tg = threadIdx.x >> 6;
  const int c = c0 + cl;
  const float* xb = x + (long)b * T * D;
  // the block's 64 x KT weights are contiguous in W: coalesced load, transposed into LDS
  const int nw = min(64, D - c0) * KT;
  for (int i = threadIdx.x; i < nw; i += 256) {
    const int cc = i / KT, kk = i - cc * KT;
    ws[flip ? (KT - 1 - kk) : kk][cc] = W[(long)c0 * KT + i];
  }
  dw_stage<KT>(xs, xb, t0 - pad, Tv, D, c0);
  __syncthreads();
  if (c >= D) return;
  float w[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) w[k] = ws[k][cl];
  float win[DWR_PT + KT - 1];
#pragma unroll
  for (int i = 0; i < DWR_PT + KT - 1; ++i) win[i] = xs[tg * DWR_PT + i][cl];
  const float bv = bias ? bias[c] : 0.f;
#pragma unroll
  for (int j = 0; j < DWR_PT; ++j) {
    float a = bv;
#pragma unroll
    for (int k = 0; k < KT; ++k) a += w[k] * win[j + k];
    const int t = t0 + tg * DWR_PT + j;
    if (t < T) y[((long)b * T + t) * D + c] = t < Tv ? a : 0.f;
  }
}

// dW[c,k] partials over a DWR_TT-step chunk: thread (channel, time group) accumulates all K taps
// over its 16 steps from a register window, the 4 time groups are summed in LDS (fixed order).
template <int KT>
__global__ __launch_bounds__(256) void dwconv_wgrad_rb_kernel(const float* __restrict__ dy,
                                                              const float* __restrict__ x,
                                                              float* __restrict__ part, int T, int D,
                                                              const int* __restrict__ tvalid) {
  __shared__ __attribute__((aligned(16))) float xs[DWR_TT + KT - 1][64];
  __shared__ float red[3][KT][64];
  const int Tv = valid_T(tvalid, T);
  constexpr int pad = (KT - 1) / 2;
  const int c0 = blockIdx.x * 64, ch = blockIdx.y, b = blockIdx.z, nch = gridDim.y;
  const int t0 = ch * DWR_TT;
  const int cl = threadIdx.x & 63, tg = threadIdx.x >> 6;
  const int c = c0 + cl;
  const float* xb = x + (long)b * T * D;
  const float* db = dy + (long)b * T * D;
  dw_stage<KT>(xs, xb, t0 - pad, Tv, D, c0);
  float g[DWR_PT];
#pragma unroll
  for (int j = 0; j < DWR_PT; ++j) {
    const int t = t0 + tg * DWR_PT + j;
    g[j] = (c < D && t < Tv) ? db[(long)t * D + c] : 0.f;
  }
  __syncthreads();
  float win[DWR_PT + KT - 1];
#pragma unroll
  for (int i = 0; i < DWR_PT + KT - 1; ++i) win[i] = xs[tg * DWR_PT + i][cl];
  float acc[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < DWR_PT; ++j) a += g[j] * win[j + k];
    acc[k] = a;
  }
  if (tg > 0) {
#pragma unroll
    for (int k = 0; k < KT; ++k) red[tg - 1][k][cl] = acc[k];
  }
  __syncthreads();
  if (tg == 0 && c < D) {
    float* pr = part + ((long)(b * nch + ch) * D + c) * KT;
#pragma unroll
    for (int k = 0; k < KT; ++k) pr[k] = ((acc[k] + red[0][k][cl]) + red[1][k][cl]) + red[2][k][cl];
  }
}

// BatchNorm statistics, stage 1: per row-chunk partial sums (double) of x and, given a
// mean, of (x-mean)^2.  mode 0: sum x ; mode 1: sum (x-mean)^2
// (rows r = b*T + t; with tvalid only t < *tvalid count)
__global__ void bn_part_kernel(const float* __restrict__ x, int M, int D, int rows_per_block,
                               const float* __restrict__ mean, int mode, double* __restrict__ part, int T,
                               const int* __restrict__ tvalid) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= D) return;
  const int Tv = valid_T(tvalid, T);
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  double s = 0.0;
  const float mu = mode ? mean[c] : 0.f;
  int t = r0 % T;
  for (int r = r0; r < r1; ++r, t = (t + 1 == T ? 0 : t + 1)) {
    if (t >= Tv) continue;
    const float v = x[(long)r * D + c];
    if (mode) {
      const double d = (double)v - (double)mu;
      s += d * d;
    } else {
      s += v;
    }
  }
  part[(long)blockIdx.x * D + c] = s;
}

// fixed-order sum of nb partial rows for 64 columns: 16 groups of 64 lanes
__device__ __forceinline__ double sum_parts16(const double* __restrict__ part, int nb, long stride, int c, bool ok,
                                              double (*sh)[64]) {
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  double s = 0.0;
  if (ok)
    for (int p = g; p < nb; p += 16) s += part[(long)p * stride + c];
  sh[g][cl] = s;
  __syncthreads();
  double t = 0.0;
  for (int k = 0; k < 16; ++k) t += sh[k][cl];
  return t;
}

// fixed-order sum of nb partial rows for 16 columns: 64 groups of 16 lanes (the BatchNorm
// statistics have up to BN_CHUNKS partial rows per column, so the rows, not the columns, need
// the parallelism)
constexpr int BNF_COLS = 16, BNF_GROUPS = 64;
__device__ __forceinline__ double sum_parts_rows(const double* __restrict__ part, int nb, long stride, int c, bool ok,
                                                 double (*sh)[BNF_COLS]) {
  const int cl = threadIdx.x % BNF_COLS, g = threadIdx.x / BNF_COLS;
  double s = 0.0;
  if (ok)
    for (int p = g; p < nb; p += BNF_GROUPS) s += part[(long)p * stride + c];
  sh[g][cl] = s;
  __syncthreads();
  double t = 0.0;
  for (int k = 0; k < BNF_GROUPS; ++k) t += sh[k][cl];
  return t;
}

// finalize: mode 0 -> mean[c] = S/M ; mode 1 -> rstd[c], running stats update
__global__ __launch_bounds__(1024) void bn_finalize_kernel(const double* __restrict__ part, int nb, int D, int M, int mode,
                                                           float* __restrict__ mean, float* __restrict__ rstd,
                                                           float* __restrict__ run_mean, float* __restrict__ run_var,
                                                           float momentum, float eps, int T,
                                                           const int* __restrict__ tvalid) {
  __shared__ double sh[BNF_GROUPS][BNF_COLS];
  if (tvalid) M = (M / T) * valid_T(tvalid, T);  // B * T' rows of the reference batch
  const int c = blockIdx.x * BNF_COLS + threadIdx.x % BNF_COLS;
  const double s = sum_parts_rows(part, nb, D, c, c < D, sh);
  if (threadIdx.x / BNF_COLS != 0 || c >= D) return;
  if (mode == 0) {
    mean[c] = (float)(s / M);
  } else {
    const double var = s / M;
    rstd[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (run_mean) {
      const double unb = M > 1 ? s / (M - 1) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean[c];
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
    }
  }
}

// s = swish(gamma*(y-mean)*rstd + beta), float4 form (D % 4 == 0, 16-B aligned, M*D/4 < 2^31)
__global__ void bn_swish_fwd4_kernel(const float* __restrict__ y, const float* __restrict__ mean,
                                     const float* __restrict__ rstd, const float* __restrict__ gamma,
                                     const float* __restrict__ beta, float* __restrict__ s, int n4, int D) {
  const int nq = D >> 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const int c = 4 * (i % nq);
    const float4 v = reinterpret_cast<const float4*>(y)[i];
    const float4 mu = *reinterpret_cast<const float4*>(mean + c), rs = *reinterpret_cast<const float4*>(rstd + c);
    const float4 ga = *reinterpret_cast<const float4*>(gamma + c), be = *reinterpret_cast<const float4*>(beta + c);
    const float zx = (v.x - mu.x) * rs.x * ga.x + be.x, zy = (v.y - mu.y) * rs.y * ga.y + be.y;
    const float zz = (v.z - mu.z) * rs.z * ga.z + be.z, zw = (v.w - mu.w) * rs.w * ga.w + be.w;
    reinterpret_cast<float4*>(s)[i] = make_float4(zx * esp::fast_sigmoid(zx), zy * esp::fast_sigmoid(zy),
                                                  zz * esp::fast_sigmoid(zz), zw * esp::fast_sigmoid(zw));
  }
}

// the same, s written as bf16 planes (n = 3 exact split, 1 = bf16) for pointwise_conv2, its only
// reader (kernels.Planes); row pitch ld (bf16 elements), plane stride ps
__global__ void bn_swish_fwd4_planes_kernel(const float* __restrict__ y, const float* __restrict__ mean,
                                            const float* __restrict__ rstd, const float* __restrict__ gamma,
                                            const float* __restrict__ beta, uint16_t* __restrict__ s, long ld, long ps,
                                            int n, int n4, int D) {
  const int nq = D >> 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const int r = i / nq, c = 4 * (i - r * nq);
    const float4 v = reinterpret_cast<const float4*>(y)[i];
    const float4 mu = *reinterpret_cast<const float4*>(mean + c), rs = *reinterpret_cast<const float4*>(rstd + c);
    const float4 ga = *reinterpret_cast<const float4*>(gamma + c), be = *reinterpret_cast<const float4*>(beta + c);
    const float zx = (v.x - mu.x) * rs.x * ga.x + be.x, zy = (v.y - mu.y) * rs.y * ga.y + be.y;
    const float zz = (v.z - mu.z) * rs.z * ga.z + be.z, zw = (v.w - mu.w) * rs.w * ga.w + be.w;
    esp::store_planes4(s, (long)r * ld + c, ps, n, zx * esp::fast_sigmoid(zx), zy * esp::fast_sigmoid(zy),
                       zz * esp::fast_sigmoid(zz), zw * esp::fast_sigmoid(zw));
  }
}

// s = swish(gamma*(y-mean)*rstd + beta)
__global__ void bn_swish_fwd_kernel(const float* __restrict__ y, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, const float* __restrict__ gamma,
                                    const float* __restrict__ beta, float* __restrict__ s, long n, int D) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % D);
    const float z = (y[i] - mean[c]) * rstd[c] * gamma[c] + beta[c];
    s[i] = z * esp::fast_sigmoid(z);
  }
}

// stage 1 of BN backward: dz = ds * swish'(z) written to dz; partials of sum dz, sum dz*xhat
__global__ void bn_swish_bwd_part_kernel(const float* __restrict__ ds, const float* __restrict__ y,
                                         const float* __restrict__ mean, const float* __restrict__ rstd,
                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                         float* __restrict__ dz, int M, int D, int rows_per_block,
                                         double* __restrict__ part, int T, const int* __restrict__ tvalid) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= D) return;
  const int Tv = valid_T(tvalid, T);
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const float mu = mean[c], rs = rstd[c], ga = gamma[c], be = beta[c];
  double s1 = 0.0, s2 = 0.0;
  int t = r0 % T;
  for (int r = r0; r < r1; ++r, t = (t + 1 == T ? 0 : t + 1)) {
    const long i = (long)r * D + c;
    if (t >= Tv) {  // not a frame of the reference batch: zero gradient, not in the sums
      dz[i] = 0.f;
      continue;
    }
    const float xh = (y[i] - mu) * rs;
    const float z = xh * ga + be;
    const float sg = esp::fast_sigmoid(z);
    const float d = ds[i] * (sg * (1.0f + z * (1.0f - sg)));
    dz[i] = d;
    s1 += d;
    s2 += (double)d * xh;
  }
  part[((long)blockIdx.x * 2) * D + c] = s1;
  part[((long)blockIdx.x * 2) * D + D + c] = s2;
}

__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(const double* __restrict__ part, int nb, int D,
                                                               float* __restrict__ sums, float* __restrict__ dgamma,
                                                               float* __restrict__ dbeta) {
  __shared__ double sh[BNF_GROUPS][BNF_COLS];
  const int c = blockIdx.x * BNF_COLS + threadIdx.x % BNF_COLS;
  const double s1 = sum_parts_rows(part, nb, 2L * D, c, c < D, sh);
  __syncthreads();
  const double s2 = sum_parts_rows(part + D, nb, 2L * D, c, c < D, sh);
  if (threadIdx.x / BNF_COLS != 0 || c >= D) return;
  sums[c] = (float)s1;
  sums[D + c] = (float)s2;
  dbeta[c] += (float)s1;
  dgamma[c] += (float)s2;
}

// float4 form of bn_bwd_apply_kernel (D % 4 == 0, 16-B aligned, M*D/4 < 2^31): 32-bit index
// math, 1/M hoisted (the scalar form divides per element)
__global__ void bn_bwd_apply4_kernel(float* __restrict__ dz, const float* __restrict__ y,
                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                     const float* __restrict__ gamma, const float* __restrict__ sums, int n4, int D,
                                     int M, int T, const int* __restrict__ tvalid) {
  const int Tv = valid_T(tvalid, T);
  if (tvalid) M = (M / T) * Tv;
  const float invM = 1.0f / (float)M;
  const int nq = D >> 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const int row = i / nq, c = 4 * (i - row * nq);
    if (tvalid && row % T >= Tv) continue;  // stays 0 (bn_swish_bwd_part_kernel)
    const float4 d4 = reinterpret_cast<const float4*>(dz)[i], y4 = reinterpret_cast<const float4*>(y)[i];
    const float dv[4] = {d4.x, d4.y, d4.z, d4.w}, yv[4] = {y4.x, y4.y, y4.z, y4.w};
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float rs = rstd[c + e];
      const float xh = (yv[e] - mean[c + e]) * rs;
      o[e] = gamma[c + e] * rs * (dv[e] - sums[c + e] * invM - xh * sums[D + c + e] * invM);
    }
    reinterpret_cast<float4*>(dz)[i] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// dy = gamma*rstd*(dz - S1/M - xhat*S2/M)   (in place over dz)
__global__ void bn_bwd_apply_kernel(float* __restrict__ dz, const float* __restrict__ y, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, const float* __restrict__ gamma,
                                    const float* __restrict__ sums, long n, int D, int M, int T,
                                    const int* __restrict__ tvalid) {
  const int Tv = valid_T(tvalid, T);
  if (tvalid) M = (M / T) * Tv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % D);
    if (tvalid && (int)((i / D) % T) >= Tv) continue;  // stays 0 (bn_swish_bwd_part_kernel)
    const float xh = (y[i] - mean[c]) * rstd[c];
    dz[i] = gamma[c] * rstd[c] * (dz[i] - sums[c] / M - xh * sums[D + c] / M);
  }
}

inline int gridn(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 65536 ? 65536 : (b < 1 ? 1 : b));
}
inline int nchunks(int M, int target_rows) { return (M + target_rows - 1) / target_rows; }
// rows per block so that about 1536 blocks share the rows: each thread walks its channel down
// the chunk serially, so the statistics passes are latency-bound unless every CU holds several
// blocks (384 chunks measured 1.2 TB/s on 47872 x 256; the workspace bound is BN_CHUNKS)
constexpr int BN_CHUNKS = 1536;
inline int rows_per_block(int M) {
  int r = (M + BN_CHUNKS - 1) / BN_CHUNKS;
  return r < 8 ? 8 : r;
}
inline dim3 fin_grid(int N) { return dim3((N + FC_COLS - 1) / FC_COLS); }
inline dim3 bnf_grid(int D) { return dim3((D + BNF_COLS - 1) / BNF_COLS); }

}  // namespace

// --------------------------------------------------------------------------- C-ABI
ESP_API int esp_layernorm_fwd(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd,
                              int M, int D, float eps, void* stream) {
  ESP_ARG_CHECK(D <= MAXD, "esp_layernorm_fwd: D=%d > %d", D, MAXD);
  dim3 grid((M + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
  const int per = (D + 63) / 64;
  if (per <= 4) hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, dim3(256), 0, st, x, w, b, y, mean, rstd, M, D, eps);
  else if (per <= 8) hipLaunchKernelGGL(ln_fwd_kernel<8>, grid, dim3(256), 0, st, x, w, b, y, mean, rstd, M, D, eps);
  else hipLaunchKernelGGL(ln_fwd_kernel<32>, grid, dim3(256), 0, st, x, w, b, y, mean, rstd, M, D, eps);
  ESP_CHECK_LAUNCH("esp_layernorm_fwd");
  return 0;
}

static int layernorm_fwd_planes_impl(const float* x, const float* w, const float* b, void* y, long ldy, long pstride,
                                     int nplanes, float* mean, float* rstd, int M, int D, float eps, float* yf,
                                     void* stream) {
  ESP_ARG_CHECK(D <= MAXD && D % 4 == 0, "esp_layernorm_fwd_planes: D=%d must be a multiple of 4 and <= %d", D, MAXD);
  ESP_ARG_CHECK((nplanes == 1 || nplanes == 3) && ldy >= D && ldy % 4 == 0 && (nplanes == 1 || pstride >= (long)M * ldy) &&
                    ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 7) == 0 && ((uintptr_t)w & 15) == 0 &&
                    ((uintptr_t)b & 15) == 0 && pstride % 4 == 0,
                "esp_layernorm_fwd_planes/_dual: bad planes layout (nplanes %d, ldy %ld, pstride %ld) or alignment", nplanes,
                ldy, pstride);
  if (M <= 0) return 0;
  dim3 grid((M + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
  const int pq = (D / 4 + 63) / 64;
  uint16_t* yp = (uint16_t*)y;
  if (pq <= 1)
    hipLaunchKernelGGL(ln_fwd_planes_kernel<1>, grid, dim3(256), 0, st, x, w, b, yp, ldy, pstride, nplanes, mean, rstd, M, D, eps, yf);
  else if (pq <= 2)
    hipLaunchKernelGGL(ln_fwd_planes_kernel<2>, grid, dim3(256), 0, st, x, w, b, yp, ldy, pstride, nplanes, mean, rstd, M, D, eps, yf);
  else
    hipLaunchKernelGGL(ln_fwd_planes_kernel<8>, grid, dim3(256), 0, st, x, w, b, yp, ldy, pstride, nplanes, mean, rstd, M, D, eps, yf);
  ESP_CHECK_LAUNCH("esp_layernorm_fwd_planes");
  return 0;
}

// workspace: 2*D*ceil(M/32) floats (esp_layernorm_bwd_workspace_bytes).  dw/db are accumulated (+=).
ESP_API int esp_layernorm_fwd_planes(const float* x, const float* w, const float* b, void* y, long ldy, long pstride,
                                     int nplanes, float* mean, float* rstd, int M, int D, float eps, void* stream) {
  return layernorm_fwd_planes_impl(x, w, b, y, ldy, pstride, nplanes, mean, rstd, M, D, eps, nullptr, stream);
}

// y in fp32 (row pitch D) AND as planes: the LayerNorm outputs that feed a Linear forward (fp32 A, weight
// planes B) and its weight gradient (B = the planes: no split of B in that GEMM's k-loop)
ESP_API int esp_layernorm_fwd_dual(const float* x, const float* w, const float* b, float* yf, void* y, long ldy,
                                   long pstride, int nplanes, float* mean, float* rstd, int M, int D, float eps,
                                   void* stream) {
  ESP_ARG_CHECK(yf && ((uintptr_t)yf & 15) == 0, "esp_layernorm_fwd_dual: y (fp32) must be 16-B aligned");
  return layernorm_fwd_planes_impl(x, w, b, y, ldy, pstride, nplanes, mean, rstd, M, D, eps, yf, stream);
}

ESP_API long esp_layernorm_bwd_workspace_bytes(int M, int D) {
  return M <= 0 || D <= 0 ? 0 : 4L * 2 * D * ((M + LN_BWD_ROWS - 1) / LN_BWD_ROWS);
}
ESP_API int esp_layernorm_bwd(const float* dy, const float* x, const float* w, const float* mean, const float* rstd,
                              float* dx, int accumulate, float* dw, float* db, int M, int D, float* work,
                              long work_bytes, void* stream) {
  ESP_ARG_CHECK(D <= MAXD && D % 4 == 0, "esp_layernorm_bwd: D=%d must be a multiple of 4 and <= %d", D, MAXD);
  const long need__ = esp_layernorm_bwd_workspace_bytes(M, D);
  ESP_ARG_CHECK(work_bytes >= need__, "esp_layernorm_bwd: workspace %ld B < %ld B required (esp_layernorm_bwd_workspace_bytes)", work_bytes, need__);
  if (M <= 0) return 0;
  const int nb = (M + LN_BWD_ROWS - 1) / LN_BWD_ROWS;
  hipStream_t st = (hipStream_t)stream;
  const int pq = (D / 4 + 63) / 64;
  if (pq <= 1)
    hipLaunchKernelGGL(ln_bwd_kernel<1>, dim3(nb), dim3(256), 0, st, dy, x, w, mean, rstd, dx, accumulate, work, M, D);
  else if (pq <= 2)
    hipLaunchKernelGGL(ln_bwd_kernel<2>, dim3(nb), dim3(256), 0, st, dy, x, w, mean, rstd, dx, accumulate, work, M, D);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<8>, dim3(nb), dim3(256), 0, st, dy, x, w, mean, rstd, dx, accumulate, work, M, D);
  hipLaunchKernelGGL(finalize_cols2_kernel, fin_grid(2 * D), dim3(1024), 0, st, work, nb, (long)2 * D, D, dw, db);
  ESP_CHECK_LAUNCH("esp_layernorm_bwd");
  return 0;
}

// out[c] (+)= sum_r x[r*ld + c].  workspace: N*ceil(M/32) floats (esp_colsum_workspace_bytes)
ESP_API long esp_colsum_workspace_bytes(int M, int N) {
  return M <= 0 || N <= 0 ? 0 : 4L * N * ((M + CS_ROWS - 1) / CS_ROWS);
}
ESP_API int esp_colsum(const float* x, int M, int N, long ld, float* out, int accumulate, float* work, long work_bytes,
                       void* stream) {
  const long need__ = esp_colsum_workspace_bytes(M, N);
  ESP_ARG_CHECK(work_bytes >= need__, "esp_colsum: workspace %ld B < %ld B required (esp_colsum_workspace_bytes)", work_bytes, need__);
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) {
    if (!accumulate) (void)hipMemsetAsync(out, 0, sizeof(float) * N, st);
    return 0;
  }
  const int nb = (M + CS_ROWS - 1) / CS_ROWS;
  const int vec = ((uintptr_t)x % 16 == 0) && ld % 4 == 0 && N % 4 == 0;
  hipLaunchKernelGGL(colsum_part_kernel, dim3(nb, (N + 255) / 256), dim3(256), 0, st, x, M, N, ld, vec, work);
  hipLaunchKernelGGL(finalize_cols_kernel<float>, fin_grid(N), dim3(1024), 0, st, work, nb, (long)N, N, out, accumulate);
  ESP_CHECK_LAUNCH("esp_colsum");
  return 0;
}

static bool vec4_ok(long n, int D, std::initializer_list<const void*> ps) {
  if (D % 4 || n / 4 >= (1L << 31)) return false;
  for (const void* p : ps)
    if ((uintptr_t)p & 15) return false;
  return true;
}

ESP_API int esp_glu_fwd(const float* u, float* g, long rows, int D, void* stream) {
  if (vec4_ok(rows * 2 * D, D, {u, g}))
    hipLaunchKernelGGL(glu_fwd4_kernel, dim3(gridn(rows * D / 4)), dim3(256), 0, (hipStream_t)stream, u, g,
                       (int)rows, D);
  else
    hipLaunchKernelGGL(glu_fwd_kernel, dim3(gridn(rows * D)), dim3(256), 0, (hipStream_t)stream, u, g, rows, D);
  ESP_CHECK_LAUNCH("esp_glu_fwd");
  return 0;
}

ESP_API int esp_glu_bwd_planes(const float* u, const float* dg, void* du, long pstride, int nplanes, long rows, int D,
                               void* stream) {
  ESP_ARG_CHECK((nplanes == 1 || nplanes == 3) && vec4_ok(rows * 2 * D, D, {u, dg}) && ((uintptr_t)du & 7) == 0 &&
                    pstride % 4 == 0 && (nplanes == 1 || pstride >= rows * 2 * D),
                "esp_glu_bwd_planes: D %% 4 == 0, aligned operands, nplanes 1 or 3");
  hipLaunchKernelGGL(glu_bwd4_planes_kernel, dim3(gridn(rows * D / 4)), dim3(256), 0, (hipStream_t)stream, u, dg,
                     (uint16_t*)du, pstride, nplanes, (int)rows, D);
  ESP_CHECK_LAUNCH("esp_glu_bwd_planes");
  return 0;
}
ESP_API int esp_glu_bwd(const float* u, const float* dg, float* du, long rows, int D, void* stream) {
  if (vec4_ok(rows * 2 * D, D, {u, dg, du}))
    hipLaunchKernelGGL(glu_bwd4_kernel, dim3(gridn(rows * D / 4)), dim3(256), 0, (hipStream_t)stream, u, dg, du,
                       (int)rows, D);
  else
    hipLaunchKernelGGL(glu_bwd_kernel, dim3(gridn(rows * D)), dim3(256), 0, (hipStream_t)stream, u, dg, du, rows, D);
  ESP_CHECK_LAUNCH("esp_glu_bwd");
  return 0;
}

// flip=0: y = dwconv(x) + bias ; flip=1: input-gradient (bias ignored)
ESP_API int esp_dwconv1d(const float* x, const float* W, const float* bias, float* y, int Bn, int T, int D, int K,
                         int flip, const int* tvalid, void* stream) {
  ESP_ARG_CHECK(K % 2 == 1 && K <= 64, "esp_dwconv1d: K must be odd and <= 64");
  if (K == 31 || K == 15) {
    dim3 g2((D + 63) / 64, (T + DWR_TT - 1) / DWR_TT, Bn);
    if (K == 31)
      hipLaunchKernelGGL(dwconv_rb_kernel<31>, g2, dim3(256), 0, (hipStream_t)stream, x, W, flip ? nullptr : bias, y, T,
                         D, flip, tvalid);
    else
      hipLaunchKernelGGL(dwconv_rb_kernel<15>, g2, dim3(256), 0, (hipStream_t)stream, x, W, flip ? nullptr : bias, y, T,
                         D, flip, tvalid);
    ESP_CHECK_LAUNCH("esp_dwconv1d");
    return 0;
  }
  dim3 grid((D + 63) / 64, (T + DW_TT - 1) / DW_TT, Bn);
  hipLaunchKernelGGL(dwconv_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, W, flip ? nullptr : bias, y, Bn, T, D, K,
                     flip, tvalid);
  ESP_CHECK_LAUNCH("esp_dwconv1d");
  return 0;
}

// dW[c,k] += sum_{b,t} dy[b,t,c]*x[b,t+k-pad,c].  workspace: Bn * (time chunks) * D * K floats
// (esp_dwconv1d_wgrad_workspace_bytes)
static int dww_chunks(int T, int K) {
  return (K == 31 || K == 15) ? (T + DWR_TT - 1) / DWR_TT : (T + DWW_TCH - 1) / DWW_TCH;
}
ESP_API long esp_dwconv1d_wgrad_workspace_bytes(int Bn, int T, int D, int K) {
  return Bn <= 0 || T <= 0 || D <= 0 || K <= 0 ? 0 : 4L * Bn * dww_chunks(T, K) * D * K;
}
ESP_API int esp_dwconv1d_wgrad(const float* dy, const float* x, float* dW, int Bn, int T, int D, int K, float* work,
                               long work_bytes, const int* tvalid, void* stream) {
  ESP_ARG_CHECK(K % 2 == 1 && K <= 64, "esp_dwconv1d_wgrad: K must be odd and <= 64");
  const long need__ = esp_dwconv1d_wgrad_workspace_bytes(Bn, T, D, K);
  ESP_ARG_CHECK(work_bytes >= need__, "esp_dwconv1d_wgrad: workspace %ld B < %ld B required (esp_dwconv1d_wgrad_workspace_bytes)", work_bytes, need__);
  const int nch = dww_chunks(T, K);
  hipStream_t st = (hipStream_t)stream;
  if (K == 31)
    hipLaunchKernelGGL(dwconv_wgrad_rb_kernel<31>, dim3((D + 63) / 64, nch, Bn), dim3(256), 0, st, dy, x, work, T, D,
                       tvalid);
  else if (K == 15)
    hipLaunchKernelGGL(dwconv_wgrad_rb_kernel<15>, dim3((D + 63) / 64, nch, Bn), dim3(256), 0, st, dy, x, work, T, D,
                       tvalid);
  else
    hipLaunchKernelGGL(dwconv_wgrad_kernel, dim3((D + 63) / 64, nch, Bn), dim3(256), 0, st, dy, x, work, T, D, K,
                       tvalid);
  hipLaunchKernelGGL(finalize_cols_kernel<float>, fin_grid(D * K), dim3(1024), 0, st, work, Bn * nch, (long)D * K,
                     D * K, dW, 1);
  ESP_CHECK_LAUNCH("esp_dwconv1d_wgrad");
  return 0;
}

// BatchNorm1d training forward + Swish. mean/rstd (D) outputs; running stats updated when
// run_mean != NULL.  workspace: D doubles per row chunk (esp_bn_swish_fwd_workspace_bytes; at
// most BN_CHUNKS chunks of rows_per_block rows)
ESP_API long esp_bn_swish_fwd_workspace_bytes(int M, int D) {
  return M <= 0 || D <= 0 ? 0 : 8L * D * nchunks(M, rows_per_block(M));
}
static int bn_swish_fwd_impl(const float* y, const float* gamma, const float* beta, float* s, void* s_planes, long lds,
                             long pstride, int nplanes, float* mean, float* rstd, float* run_mean, float* run_var,
                             float momentum, float eps, int M, int D, double* work, long work_bytes, int T,
                             const int* tvalid, void* stream) {
  ESP_ARG_CHECK(!tvalid || (T > 0 && M % T == 0), "esp_bn_swish_fwd: M must be a multiple of T with tvalid");
  const long need__ = esp_bn_swish_fwd_workspace_bytes(M, D);
  ESP_ARG_CHECK(work_bytes >= need__, "esp_bn_swish_fwd: workspace %ld B < %ld B required (esp_bn_swish_fwd_workspace_bytes)", work_bytes, need__);
  if (!tvalid) T = M > 0 ? M : 1;
  const int rpb = rows_per_block(M), nb = nchunks(M, rpb);
  hipStream_t st = (hipStream_t)stream;
  dim3 g1(nb, (D + 255) / 256), gf((D + 255) / 256);
  hipLaunchKernelGGL(bn_part_kernel, g1, dim3(256), 0, st, y, M, D, rpb, nullptr, 0, work, T, tvalid);
  hipLaunchKernelGGL(bn_finalize_kernel, bnf_grid(D), dim3(1024), 0, st, work, nb, D, M, 0, mean, rstd, nullptr,
                     nullptr, momentum, eps, T, tvalid);
  hipLaunchKernelGGL(bn_part_kernel, g1, dim3(256), 0, st, y, M, D, rpb, mean, 1, work, T, tvalid);
  hipLaunchKernelGGL(bn_finalize_kernel, bnf_grid(D), dim3(1024), 0, st, work, nb, D, M, 1, mean, rstd, run_mean,
                     run_var, momentum, eps, T, tvalid);
  if (s_planes) {
    hipLaunchKernelGGL(bn_swish_fwd4_planes_kernel, dim3(gridn((long)M * D / 4)), dim3(256), 0, st, y, mean, rstd,
                       gamma, beta, (uint16_t*)s_planes, lds, pstride, nplanes, (int)((long)M * D / 4), D);
  } else if (vec4_ok((long)M * D, D, {y, mean, rstd, gamma, beta, s})) {
    hipLaunchKernelGGL(bn_swish_fwd4_kernel, dim3(gridn((long)M * D / 4)), dim3(256), 0, st, y, mean, rstd, gamma,
                       beta, s, (int)((long)M * D / 4), D);
  } else {
    hipLaunchKernelGGL(bn_swish_fwd_kernel, dim3(gridn((long)M * D)), dim3(256), 0, st, y, mean, rstd, gamma, beta,
                       s, (long)M * D, D);
  }
  ESP_CHECK_LAUNCH("esp_bn_swish_fwd");
  return 0;
}
ESP_API int esp_bn_swish_fwd(const float* y, const float* gamma, const float* beta, float* s, float* mean, float* rstd,
                             float* run_mean, float* run_var, float momentum, float eps, int M, int D, double* work,
                             long work_bytes, int T, const int* tvalid, void* stream) {
  return bn_swish_fwd_impl(y, gamma, beta, s, nullptr, 0, 0, 0, mean, rstd, run_mean, run_var, momentum, eps, M, D,
                           work, work_bytes, T, tvalid, stream);
}
ESP_API int esp_bn_swish_fwd_planes(const float* y, const float* gamma, const float* beta, void* s_planes, long lds,
                                    long pstride, int nplanes, float* mean, float* rstd, float* run_mean,
                                    float* run_var, float momentum, float eps, int M, int D, double* work,
                                    long work_bytes, int T, const int* tvalid, void* stream) {
  ESP_ARG_CHECK(s_planes && (nplanes == 1 || nplanes == 3) && D % 4 == 0 && lds % 4 == 0 && lds >= D &&
                    pstride % 4 == 0 && ((uintptr_t)s_planes & 7) == 0 &&
                    vec4_ok((long)M * D, D, {y, mean, rstd, gamma, beta}),
                "esp_bn_swish_fwd_planes: D, ld, pstride %% 4 == 0, aligned operands needed");
  return bn_swish_fwd_impl(y, gamma, beta, nullptr, s_planes, lds, pstride, nplanes, mean, rstd, run_mean, run_var,
                           momentum, eps, M, D, work, work_bytes, T, tvalid, stream);
}

// eval mode (BatchNorm1d with track_running_stats, convolution.py:56-79 under model.eval()):
// mean / rstd from the running statistics, then the same fused BN + Swish
__global__ void bn_running_kernel(const float* __restrict__ rm, const float* __restrict__ rv, float eps, int D,
                                  float* __restrict__ mean, float* __restrict__ rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < D) {
    mean[c] = rm[c];
    rstd[c] = 1.0f / sqrtf(rv[c] + eps);
  }
}
ESP_API int esp_bn_swish_eval(const float* y, const float* gamma, const float* beta, float* s, const float* run_mean,
                              const float* run_var, float eps, int M, int D, float* mean, float* rstd, void* stream) {
  ESP_ARG_CHECK(M >= 0 && D >= 1, "esp_bn_swish_eval: bad sizes M=%d D=%d", M, D);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_running_kernel, dim3((D + 255) / 256), dim3(256), 0, st, run_mean, run_var, eps, D, mean, rstd);
  if ((long)M * D > 0)
    hipLaunchKernelGGL(bn_swish_fwd_kernel, dim3(gridn((long)M * D)), dim3(256), 0, st, y, mean, rstd, gamma, beta, s,
                       (long)M * D, D);
  ESP_CHECK_LAUNCH("esp_bn_swish_eval");
  return 0;
}

// given ds = dL/ds, writes dy (grad wrt BN input) into `dy`; dgamma/dbeta accumulated.
// workspace: 2*D doubles per row chunk (esp_bn_swish_bwd_workspace_bytes) + 2*D floats (sums)
// passed separately
ESP_API long esp_bn_swish_bwd_workspace_bytes(int M, int D) {
  return M <= 0 || D <= 0 ? 0 : 8L * 2 * D * nchunks(M, rows_per_block(M));
}
ESP_API int esp_bn_swish_bwd(const float* ds, const float* y, const float* mean, const float* rstd, const float* gamma,
                             const float* beta, float* dy, float* dgamma, float* dbeta, int M, int D, double* work,
                             long work_bytes, float* sums, int T, const int* tvalid, void* stream) {
  ESP_ARG_CHECK(!tvalid || (T > 0 && M % T == 0), "esp_bn_swish_bwd: M must be a multiple of T with tvalid");
  const long need__ = esp_bn_swish_bwd_workspace_bytes(M, D);
  ESP_ARG_CHECK(work_bytes >= need__, "esp_bn_swish_bwd: workspace %ld B < %ld B required (esp_bn_swish_bwd_workspace_bytes)", work_bytes, need__);
  if (!tvalid) T = M > 0 ? M : 1;
  const int rpb = rows_per_block(M), nb = nchunks(M, rpb);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_swish_bwd_part_kernel, dim3(nb, (D + 255) / 256), dim3(256), 0, st, ds, y, mean, rstd, gamma,
                     beta, dy, M, D, rpb, work, T, tvalid);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, bnf_grid(D), dim3(1024), 0, st, work, nb, D, sums, dgamma, dbeta);
  if (vec4_ok((long)M * D, D, {dy, y}))
    hipLaunchKernelGGL(bn_bwd_apply4_kernel, dim3(gridn((long)M * D / 4)), dim3(256), 0, st, dy, y, mean, rstd, gamma,
                       sums, (int)((long)M * D / 4), D, M, T, tvalid);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(gridn((long)M * D)), dim3(256), 0, st, dy, y, mean, rstd, gamma, sums,
                     (long)M * D, D, M, T, tvalid);
  ESP_CHECK_LAUNCH("esp_bn_swish_bwd");
  return 0;
}
