// Normalisation / reduction kernels (HBM-bound): LayerNorm fwd/bwd (eps 1e-12,
// layer_norm.py:12-38), deterministic column sums (bias grads), the Conformer
// ConvolutionModule's GLU + depthwise Conv1d(k, pad (k-1)/2) + BatchNorm1d (training
// statistics over all B*T' rows, padded frames included) + Swish, fwd and bwd
// (conformer/convolution.py:56-79).  Row-major [rows][channels] everywhere; one wave per
// row for row reductions; column reductions go through per-block partials and a fixed-
// order finalize, so every result is bitwise reproducible run to run.
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

// dx (+)= rstd * (g - mean(g) - xhat*mean(g*xhat)), g = dy*w; partial dw/db per block.
template <int PER>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                     const float* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, float* __restrict__ dx,
                                                     int accumulate, float* __restrict__ part, int M, int D,
                                                     int rows_per_block) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ float sh[4][2][64];
  float pw[PER], pb[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) pw[i] = pb[i] = 0.f;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  for (int row = r0 + wv; row < r1; row += 4) {
    const float* xr = x + (long)row * D;
    const float* dyr = dy + (long)row * D;
    const float mu = mean_in[row], rs = rstd_in[row];
    float xh[PER], g[PER];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        xh[i] = (xr[c] - mu) * rs;
        const float d = dyr[c];
        g[i] = d * w[c];
        pw[i] += d * xh[i];
        pb[i] += d;
      } else {
        xh[i] = g[i] = 0.f;
      }
      s1 += g[i];
      s2 += g[i] * xh[i];
    }
    s1 = esp::wave_sum(s1) / (float)D;
    s2 = esp::wave_sum(s2) / (float)D;
    float* dxr = dx + (long)row * D;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        const float v = rs * (g[i] - s1 - xh[i] * s2);
        dxr[c] = accumulate ? dxr[c] + v : v;
      }
    }
  }
  // combine the 4 waves' column partials in fixed order
  float* pr = part + (long)blockIdx.x * 2 * D;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    __syncthreads();
    if (c < D) {
      sh[wv][0][lane] = pw[i];
      sh[wv][1][lane] = pb[i];
    }
    __syncthreads();
    if (wv == 0 && c < D) {
      pr[c] = sh[0][0][lane] + sh[1][0][lane] + sh[2][0][lane] + sh[3][0][lane];
      pr[D + c] = sh[0][1][lane] + sh[1][1][lane] + sh[2][1][lane] + sh[3][1][lane];
    }
  }
}

// out[c] (+)= sum_{p<nb} part[p*stride + c]   for c < N.  Block = 64 columns x 16 row
// groups (1024 threads); each group sums rows g, g+16, ...; groups combined in fixed order.
template <typename T>
__global__ __launch_bounds__(1024) void finalize_cols_kernel(const T* __restrict__ part, int nb, long stride, int N,
                                                             float* __restrict__ out, int accumulate) {
  __shared__ T sh[16][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  T s = 0;
  if (c < N) {
#pragma unroll 4
    for (int p = g; p < nb; p += 16) s += part[(long)p * stride + c];
  }
  sh[g][cl] = s;
  __syncthreads();
  if (g == 0 && c < N) {
    T t = 0;
    for (int k = 0; k < 16; ++k) t += sh[k][cl];
    out[c] = accumulate ? out[c] + (float)t : (float)t;
  }
}

// column partial sums of a [M][N] (ld) matrix: block = chunk of rows, thread = column
__global__ void colsum_part_kernel(const float* __restrict__ x, int M, int N, long ld, int rows_per_block,
                                   float* __restrict__ part) {
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (int c = blockIdx.y * blockDim.x + threadIdx.x; c < N; c += gridDim.y * blockDim.x) {
    float s = 0.f;
    for (int r = r0; r < r1; ++r) s += x[(long)r * ld + c];
    part[(long)blockIdx.x * N + c] = s;
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
    g[i] = a * (1.0f / (1.0f + expf(-b)));
  }
}

__global__ void glu_bwd_kernel(const float* __restrict__ u, const float* __restrict__ dg, float* __restrict__ du,
                               long rows, int D) {
  const long n = rows * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / D;
    const int c = (int)(i - r * D);
    const float a = u[r * 2 * D + c], b = u[r * 2 * D + D + c];
    const float s = 1.0f / (1.0f + expf(-b));
    const float d = dg[i];
    du[r * 2 * D + c] = d * s;
    du[r * 2 * D + D + c] = d * a * s * (1.0f - s);
  }
}

// y[b,t,c] = bias[c] + sum_k W[c,k] * x[b, t + k - pad, c]   (flip=0, forward)
// y[b,t,c] = sum_k W[c,k] * x[b, t - k + pad, c]             (flip=1, input grad)
// Block = 64 channels x DW_TT time steps; the input window (DW_TT + K - 1 rows) and the
// 64 filters are staged in LDS; a thread owns one channel and DW_TT/4 consecutive steps.
constexpr int DW_TT = 32, DW_KMAX = 64;
__global__ __launch_bounds__(256) void dwconv_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                     const float* __restrict__ bias, float* __restrict__ y, int Bn,
                                                     int T, int D, int K, int flip) {
  __shared__ float xs[DW_TT + DW_KMAX][64];
  __shared__ float ws[64][DW_KMAX + 1];
  const int c0 = blockIdx.x * 64, t0 = blockIdx.y * DW_TT, b = blockIdx.z;
  const int pad = (K - 1) / 2;
  const int cl = threadIdx.x & 63, tg = threadIdx.x >> 6;
  const int c = c0 + cl;
  const float* xb = x + (long)b * T * D;
  const int rows = DW_TT + K - 1;
  for (int r = tg; r < rows; r += 4) {
    const int t = t0 - pad + r;
    xs[r][cl] = (c < D && t >= 0 && t < T) ? xb[(long)t * D + c] : 0.f;
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
    if (t < T) y[((long)b * T + t) * D + c] = acc[j];
  }
}

// dW[c,k] partials over a DWW_TCH-step time chunk: sum_t dy[b,t,c] * x[b,t+k-pad,c].
// Block = 64 channels; 4 tap groups (k = kg, kg+4, ...); dy and x windows in LDS.
constexpr int DWW_TCH = 64;
__global__ __launch_bounds__(256) void dwconv_wgrad_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                           float* __restrict__ part, int T, int D, int K) {
  __shared__ float xs[DWW_TCH + DW_KMAX][64];
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
    xs[r][cl] = (c < D && t >= 0 && t < T) ? xb[(long)t * D + c] : 0.f;
  }
  for (int r = kg; r < DWW_TCH; r += 4) {
    const int t = t0 + r;
    gs[r][cl] = (c < D && t < T) ? db[(long)t * D + c] : 0.f;
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

// BatchNorm statistics, stage 1: per row-chunk partial sums (double) of x and, given a
// mean, of (x-mean)^2.  mode 0: sum x ; mode 1: sum (x-mean)^2
__global__ void bn_part_kernel(const float* __restrict__ x, int M, int D, int rows_per_block,
                               const float* __restrict__ mean, int mode, double* __restrict__ part) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= D) return;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  double s = 0.0;
  const float mu = mode ? mean[c] : 0.f;
  for (int r = r0; r < r1; ++r) {
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

// finalize: mode 0 -> mean[c] = S/M ; mode 1 -> rstd[c], running stats update
__global__ __launch_bounds__(1024) void bn_finalize_kernel(const double* __restrict__ part, int nb, int D, int M, int mode,
                                                           float* __restrict__ mean, float* __restrict__ rstd,
                                                           float* __restrict__ run_mean, float* __restrict__ run_var,
                                                           float momentum, float eps) {
  __shared__ double sh[16][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const double s = sum_parts16(part, nb, D, c, c < D, sh);
  if ((threadIdx.x >> 6) != 0 || c >= D) return;
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

// s = swish(gamma*(y-mean)*rstd + beta)
__global__ void bn_swish_fwd_kernel(const float* __restrict__ y, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, const float* __restrict__ gamma,
                                    const float* __restrict__ beta, float* __restrict__ s, long n, int D) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % D);
    const float z = (y[i] - mean[c]) * rstd[c] * gamma[c] + beta[c];
    s[i] = z / (1.0f + expf(-z));
  }
}

// stage 1 of BN backward: dz = ds * swish'(z) written to dz; partials of sum dz, sum dz*xhat
__global__ void bn_swish_bwd_part_kernel(const float* __restrict__ ds, const float* __restrict__ y,
                                         const float* __restrict__ mean, const float* __restrict__ rstd,
                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                         float* __restrict__ dz, int M, int D, int rows_per_block,
                                         double* __restrict__ part) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= D) return;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const float mu = mean[c], rs = rstd[c], ga = gamma[c], be = beta[c];
  double s1 = 0.0, s2 = 0.0;
  for (int r = r0; r < r1; ++r) {
    const long i = (long)r * D + c;
    const float xh = (y[i] - mu) * rs;
    const float z = xh * ga + be;
    const float sg = 1.0f / (1.0f + expf(-z));
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
  __shared__ double sh[16][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const double s1 = sum_parts16(part, nb, 2L * D, c, c < D, sh);
  __syncthreads();
  const double s2 = sum_parts16(part + D, nb, 2L * D, c, c < D, sh);
  if ((threadIdx.x >> 6) != 0 || c >= D) return;
  sums[c] = (float)s1;
  sums[D + c] = (float)s2;
  dbeta[c] += (float)s1;
  dgamma[c] += (float)s2;
}

// dy = gamma*rstd*(dz - S1/M - xhat*S2/M)   (in place over dz)
__global__ void bn_bwd_apply_kernel(float* __restrict__ dz, const float* __restrict__ y, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, const float* __restrict__ gamma,
                                    const float* __restrict__ sums, long n, int D, int M) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % D);
    const float xh = (y[i] - mean[c]) * rstd[c];
    dz[i] = gamma[c] * rstd[c] * (dz[i] - sums[c] / M - xh * sums[D + c] / M);
  }
}

inline int gridn(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 65536 ? 65536 : (b < 1 ? 1 : b));
}
inline int nchunks(int M, int target_rows) { return (M + target_rows - 1) / target_rows; }
// rows per block so that about 384 blocks share the rows (fills 256 CUs, bounded partials)
inline int rows_per_block(int M) {
  int r = (M + 383) / 384;
  return r < 8 ? 8 : r;
}
inline dim3 fin_grid(int N) { return dim3((N + 63) / 64); }

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

// workspace: >= 2*D*ceil(M/64) floats.  dw/db are accumulated (+=).
ESP_API int esp_layernorm_bwd(const float* dy, const float* x, const float* w, const float* mean, const float* rstd,
                              float* dx, int accumulate, float* dw, float* db, int M, int D, float* work,
                              void* stream) {
  ESP_ARG_CHECK(D <= MAXD, "esp_layernorm_bwd: D too large");
  const int rpb = rows_per_block(M);
  const int nb = nchunks(M, rpb);
  hipStream_t st = (hipStream_t)stream;
  const int per = (D + 63) / 64;
  if (per <= 4)
    hipLaunchKernelGGL(ln_bwd_kernel<4>, dim3(nb), dim3(256), 0, st, dy, x, w, mean, rstd, dx, accumulate, work, M, D, rpb);
  else if (per <= 8)
    hipLaunchKernelGGL(ln_bwd_kernel<8>, dim3(nb), dim3(256), 0, st, dy, x, w, mean, rstd, dx, accumulate, work, M, D, rpb);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<32>, dim3(nb), dim3(256), 0, st, dy, x, w, mean, rstd, dx, accumulate, work, M, D, rpb);
  hipLaunchKernelGGL(finalize_cols_kernel<float>, fin_grid(D), dim3(1024), 0, st, work, nb, (long)2 * D, D, dw, 1);
  hipLaunchKernelGGL(finalize_cols_kernel<float>, fin_grid(D), dim3(1024), 0, st, work + D, nb, (long)2 * D, D, db, 1);
  ESP_CHECK_LAUNCH("esp_layernorm_bwd");
  return 0;
}

// out[c] (+)= sum_r x[r*ld + c].  workspace: >= N*ceil(M/64) floats
ESP_API int esp_colsum(const float* x, int M, int N, long ld, float* out, int accumulate, float* work, void* stream) {
  const int rpb = rows_per_block(M);
  const int nb = nchunks(M, rpb);
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) {
    if (!accumulate) (void)hipMemsetAsync(out, 0, sizeof(float) * N, st);
    return 0;
  }
  const int ty = (N + 255) / 256;
  hipLaunchKernelGGL(colsum_part_kernel, dim3(nb, ty), dim3(256), 0, st, x, M, N, ld, rpb, work);
  hipLaunchKernelGGL(finalize_cols_kernel<float>, fin_grid(N), dim3(1024), 0, st, work, nb, (long)N, N, out, accumulate);
  ESP_CHECK_LAUNCH("esp_colsum");
  return 0;
}

ESP_API int esp_glu_fwd(const float* u, float* g, long rows, int D, void* stream) {
  hipLaunchKernelGGL(glu_fwd_kernel, dim3(gridn(rows * D)), dim3(256), 0, (hipStream_t)stream, u, g, rows, D);
  ESP_CHECK_LAUNCH("esp_glu_fwd");
  return 0;
}

ESP_API int esp_glu_bwd(const float* u, const float* dg, float* du, long rows, int D, void* stream) {
  hipLaunchKernelGGL(glu_bwd_kernel, dim3(gridn(rows * D)), dim3(256), 0, (hipStream_t)stream, u, dg, du, rows, D);
  ESP_CHECK_LAUNCH("esp_glu_bwd");
  return 0;
}

// flip=0: y = dwconv(x) + bias ; flip=1: input-gradient (bias ignored)
ESP_API int esp_dwconv1d(const float* x, const float* W, const float* bias, float* y, int Bn, int T, int D, int K,
                         int flip, void* stream) {
  ESP_ARG_CHECK(K % 2 == 1 && K <= 64, "esp_dwconv1d: K must be odd and <= 64");
  dim3 grid((D + 63) / 64, (T + DW_TT - 1) / DW_TT, Bn);
  hipLaunchKernelGGL(dwconv_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, W, flip ? nullptr : bias, y, Bn, T, D, K,
                     flip);
  ESP_CHECK_LAUNCH("esp_dwconv1d");
  return 0;
}

// dW[c,k] += sum_{b,t} dy[b,t,c]*x[b,t+k-pad,c].  workspace >= Bn*ceil(T/64)*D*K floats
ESP_API int esp_dwconv1d_wgrad(const float* dy, const float* x, float* dW, int Bn, int T, int D, int K, float* work,
                               void* stream) {
  ESP_ARG_CHECK(K % 2 == 1 && K <= 64, "esp_dwconv1d_wgrad: K must be odd and <= 64");
  const int nch = (T + DWW_TCH - 1) / DWW_TCH;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(dwconv_wgrad_kernel, dim3((D + 63) / 64, nch, Bn), dim3(256), 0, st, dy, x, work, T, D, K);
  hipLaunchKernelGGL(finalize_cols_kernel<float>, fin_grid(D * K), dim3(1024), 0, st, work, Bn * nch, (long)D * K,
                     D * K, dW, 1);
  ESP_CHECK_LAUNCH("esp_dwconv1d_wgrad");
  return 0;
}

// BatchNorm1d training forward + Swish. mean/rstd (D) outputs; running stats updated when
// run_mean != NULL.  workspace: >= D*ceil(M/64) doubles
ESP_API int esp_bn_swish_fwd(const float* y, const float* gamma, const float* beta, float* s, float* mean, float* rstd,
                             float* run_mean, float* run_var, float momentum, float eps, int M, int D, double* work,
                             void* stream) {
  const int rpb = rows_per_block(M), nb = nchunks(M, rpb);
  hipStream_t st = (hipStream_t)stream;
  dim3 g1(nb, (D + 255) / 256), gf((D + 255) / 256);
  hipLaunchKernelGGL(bn_part_kernel, g1, dim3(256), 0, st, y, M, D, rpb, nullptr, 0, work);
  hipLaunchKernelGGL(bn_finalize_kernel, fin_grid(D), dim3(1024), 0, st, work, nb, D, M, 0, mean, rstd, nullptr,
                     nullptr, momentum, eps);
  hipLaunchKernelGGL(bn_part_kernel, g1, dim3(256), 0, st, y, M, D, rpb, mean, 1, work);
  hipLaunchKernelGGL(bn_finalize_kernel, fin_grid(D), dim3(1024), 0, st, work, nb, D, M, 1, mean, rstd, run_mean,
                     run_var, momentum, eps);
  hipLaunchKernelGGL(bn_swish_fwd_kernel, dim3(gridn((long)M * D)), dim3(256), 0, st, y, mean, rstd, gamma, beta, s,
                     (long)M * D, D);
  ESP_CHECK_LAUNCH("esp_bn_swish_fwd");
  return 0;
}

// given ds = dL/ds, writes dy (grad wrt BN input) into `dy`; dgamma/dbeta accumulated.
// workspace: >= 2*D*ceil(M/64) doubles + 2*D floats (sums) passed separately
ESP_API int esp_bn_swish_bwd(const float* ds, const float* y, const float* mean, const float* rstd, const float* gamma,
                             const float* beta, float* dy, float* dgamma, float* dbeta, int M, int D, double* work,
                             float* sums, void* stream) {
  const int rpb = rows_per_block(M), nb = nchunks(M, rpb);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_swish_bwd_part_kernel, dim3(nb, (D + 255) / 256), dim3(256), 0, st, ds, y, mean, rstd, gamma,
                     beta, dy, M, D, rpb, work);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, fin_grid(D), dim3(1024), 0, st, work, nb, D, sums, dgamma, dbeta);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(gridn((long)M * D)), dim3(256), 0, st, dy, y, mean, rstd, gamma, sums,
                     (long)M * D, D, M);
  ESP_CHECK_LAUNCH("esp_bn_swish_bwd");
  return 0;
}
