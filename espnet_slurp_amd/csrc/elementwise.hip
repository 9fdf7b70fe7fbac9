// Memory-bound element-wise kernels: activation/dropout backward, residual scaling,
// embedding, positional scaling, SpecAugment (time warp + masks), utterance MVN,
// fused Adam over the flat parameter buffer, global grad-norm, and library errors.
// All are HBM-bound: float4 loads/stores where the layout allows, grid-stride loops.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace esp {
static thread_local char g_err[512] = "";
static const uint64_t* g_rng_key = nullptr;
const uint64_t* rng_key_ptr() { return g_rng_key; }
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace esp

ESP_API const char* esp_last_error(void) { return esp::g_err; }
ESP_API int esp_abi_version(void) { return 32; }
ESP_API int esp_set_rng_key(const unsigned long long* key) {
  esp::g_rng_key = (const uint64_t*)key;
  return 0;
}

namespace {


inline int grid_for(long n, int per_thread = 1) {
  long b = (n / per_thread + 255) / 256;
  if (b > 65536) b = 65536;
  return (int)(b < 1 ? 1 : b);
}

// dx = dy * keep*scale * act'(h)        (act: 0 none, 1 relu, 2 swish)
__global__ void act_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ h,
                               float* __restrict__ dx, long n, int act, uint32_t thr, float scale,
                               uint64_t seed, long idx_off, const uint64_t* __restrict__ key) {
  seed = esp::keyed(seed, key);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float g = dy[i];
    if (thr) g = esp::keep_elem(seed, (uint64_t)(i + idx_off), thr) ? g * scale : 0.f;
    const float x = h[i];
    if (act == 1) g = x > 0.f ? g : 0.f;
    else if (act == 2) {
      const float s = 1.0f / (1.0f + expf(-x));
      g = g * (s * (1.0f + x * (1.0f - s)));
    }
    dx[i] = g;
  }
}

// y = alpha * keep*scale * x (+ beta * r)  — dropout forward/backward on residual branches
__global__ void scale_drop_kernel(const float* __restrict__ x, float* __restrict__ y, long n, float alpha,
                                  uint32_t thr, float scale, uint64_t seed, const float* r, float beta,
                                  const uint64_t* __restrict__ key) {
  seed = esp::keyed(seed, key);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float v = x[i];
    if (thr) v = esp::keep_elem(seed, (uint64_t)i, thr) ? v * scale : 0.f;
    v *= alpha;
    if (r) v += beta * r[i];
    y[i] = v;
  }
}

// float4 form (n % 4 == 0, 16-B aligned): same element indices for the dropout hash
__global__ void scale_drop4_kernel(const float* __restrict__ x, float* __restrict__ y, long n4, float alpha,
                                   uint32_t thr, float scale, uint64_t seed, const float* __restrict__ r, float beta,
                                   const uint64_t* __restrict__ key) {
  seed = esp::keyed(seed, key);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v4 = reinterpret_cast<const float4*>(x)[i];
    float v[4] = {v4.x, v4.y, v4.z, v4.w};
    bool kp[4] = {true, true, true, true};
    if (thr) {
      esp::keep_pair(seed, (uint64_t)(4 * i), thr, kp[0], kp[1]);
      esp::keep_pair(seed, (uint64_t)(4 * i + 2), thr, kp[2], kp[3]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (thr) v[e] = kp[e] ? v[e] * scale : 0.f;
      v[e] *= alpha;
    }
    if (r) {
      const float4 r4 = reinterpret_cast<const float4*>(r)[i];
      v[0] += beta * r4.x; v[1] += beta * r4.y; v[2] += beta * r4.z; v[3] += beta * r4.w;
    }
    reinterpret_cast<float4*>(y)[i] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// the same without a residual, y written as bf16 planes (n = 3 exact split, 1 = bf16) of a matrix whose
// rows are whole planes rows (ld == cols): the backward's residual-branch gradient that only the
// branch's weight- and input-gradient GEMMs read (kernels.Planes)
__global__ void scale_drop4_planes_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, long n4, long ps,
                                          int np, float alpha, uint32_t thr, float scale, uint64_t seed,
                                          const uint64_t* __restrict__ key) {
  seed = esp::keyed(seed, key);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v4 = reinterpret_cast<const float4*>(x)[i];
    float v[4] = {v4.x, v4.y, v4.z, v4.w};
    bool kp[4] = {true, true, true, true};
    if (thr) {
      esp::keep_pair(seed, (uint64_t)(4 * i), thr, kp[0], kp[1]);
      esp::keep_pair(seed, (uint64_t)(4 * i + 2), thr, kp[2], kp[3]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (thr) v[e] = kp[e] ? v[e] * scale : 0.f;
      v[e] *= alpha;
    }
    esp::store_planes4(y, 4 * i, ps, np, v[0], v[1], v[2], v[3]);
  }
}

// encoder input of the blocks: x = drop(x * xscale); pos = drop(pos)  (embedding.py:228-244)
// decoder: x = drop(E[tok] * xscale + pe[l])                            (embedding.py:81-94)
__global__ void embed_fwd_kernel(const int64_t* __restrict__ tok, const float* __restrict__ E,
                                 const float* __restrict__ pe, float* __restrict__ y, int L, int D,
                                 float xscale, uint32_t thr, float scale, uint64_t seed, long n,
                                 const uint64_t* __restrict__ key) {
  seed = esp::keyed(seed, key);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long row = i / D;
    const int d = (int)(i - row * D);
    const int l = (int)(row % L);
    float v = E[tok[row] * (long)D + d] * xscale + pe[(long)l * D + d];
    if (thr) v = esp::keep_elem(seed, (uint64_t)i, thr) ? v * scale : 0.f;
    y[i] = v;
  }
}

// dE[v, :] += sum over rows with tok==v of dy*mask*scale*xscale.  One block per vocab row;
// the block scans the token list 256 rows at a time (coalesced), compacts the matching row
// indices into LDS in ascending order (wave ballot + per-wave prefix), then every thread
// accumulates its columns over that list.  The summation order is ascending r, fixed, so
// the result is deterministic (no atomics).
constexpr int EMB_MAXD = 1024;  // D / 256 accumulators per thread
__global__ void __launch_bounds__(256) embed_bwd_kernel(const int64_t* __restrict__ tok, const float* __restrict__ dy,
                                                        float* __restrict__ dE, int nrows, int D, float xscale,
                                                        uint32_t thr, float scale, uint64_t seed,
                                                        const uint64_t* __restrict__ key) {
  __shared__ int rows[256];
  __shared__ int wcnt[4];
  seed = esp::keyed(seed, key);
  const int v = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float acc[EMB_MAXD / 256];
#pragma unroll
  for (int j = 0; j < EMB_MAXD / 256; ++j) acc[j] = 0.f;
  bool any = false;
  for (int c = 0; c < nrows; c += 256) {
    const int r = c + tid;
    const bool hit = r < nrows && tok[r] == v;
    const uint64_t m = __ballot(hit);
    if (lane == 0) wcnt[w] = __popcll(m);
    __syncthreads();
    const int base = (w > 0 ? wcnt[0] : 0) + (w > 1 ? wcnt[1] : 0) + (w > 2 ? wcnt[2] : 0);
    const int n = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    if (hit) rows[base + __popcll(m & ((1ull << lane) - 1))] = r;
    __syncthreads();
    any |= n > 0;
    // EMB_GROUP rows' loads issued before their adds (which stay in ascending row order): a token
    // that fills most of the list (the eos padding of the decoder input) no longer waits out one
    // load latency per row: 962 -> ~500 us per launch at C2 B=256 (profiles/r04p_ vs r04r_kernel_summary_b256.txt;
    // 8- and 32-row groups measure the same -- the rest is the token scan)
    constexpr int EMB_GROUP = 32;
    int k = 0;
    for (; k + EMB_GROUP <= n; k += EMB_GROUP) {
#pragma unroll
      for (int j = 0; j < EMB_MAXD / 256; ++j) {
        const int d = tid + j * 256;
        if (j * 256 >= D) break;  // (uniform)
        float g[EMB_GROUP];
#pragma unroll
        for (int u = 0; u < EMB_GROUP; ++u) g[u] = d < D ? dy[(long)rows[k + u] * D + d] : 0.f;
#pragma unroll
        for (int u = 0; u < EMB_GROUP; ++u) {
          float x = g[u];
          if (thr) x = esp::keep_elem(seed, (uint64_t)((long)rows[k + u] * D + d), thr) ? x * scale : 0.f;
          if (d < D) acc[j] += x * xscale;
        }
      }
    }
    for (; k < n; ++k) {
      const long rb = (long)rows[k] * D;
#pragma unroll
      for (int j = 0; j < EMB_MAXD / 256; ++j) {
        const int d = tid + j * 256;
        if (d < D) {
          float g = dy[rb + d];
          if (thr) g = esp::keep_elem(seed, (uint64_t)(rb + d), thr) ? g * scale : 0.f;
          acc[j] += g * xscale;
        }
      }
    }
    __syncthreads();  // rows/wcnt reused by the next chunk
  }
  if (!any) return;
#pragma unroll
  for (int j = 0; j < EMB_MAXD / 256; ++j) {
    const int d = tid + j * 256;
    if (d < D) dE[(long)v * D + d] += acc[j];
  }
}

__global__ void scale_by_dev_kernel(float* __restrict__ x, long n, const float* __restrict__ s) {
  const float v = *s;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] *= v;
}

// ------------------------------------------------------------------------- SpecAugment
// Bicubic (A=-0.75) resampling identical to torch upsample_bicubic2d with
// align_corners=False along time only (the freq size is unchanged, so its weights are
// the identity): time_warp.py:9-46.  One launch handles a whole batch; per utterance
// (len, center, warped) describe the warp of x[b, :len] (len==T & shared params for the
// equal-length branch of TimeWarp.forward, time_warp.py:73-86).
__device__ __forceinline__ float cubic1(float x, float A) { return ((A + 2) * x - (A + 3)) * x * x + 1; }
__device__ __forceinline__ float cubic2(float x, float A) { return ((A * x - 5 * A) * x + 8 * A) * x - 4 * A; }

__device__ float bicubic_seg(const float* __restrict__ src, int F, int in_len, int out_len, int o, int f) {
  // src points at the first row of the input segment (in_len rows of F)
  const float sc = (float)in_len / (float)out_len;
  const float real = sc * (o + 0.5f) - 0.5f;
  const float fl = floorf(real);
  const int i0 = (int)fl;
  const float t = real - fl;
  const float A = -0.75f;
  const float w0 = cubic2(t + 1.0f, A), w1 = cubic1(t, A), w2 = cubic1(1.0f - t, A), w3 = cubic2(2.0f - t, A);
  auto at = [&](int i) {
    i = i < 0 ? 0 : (i > in_len - 1 ? in_len - 1 : i);
    return src[(long)i * F + f];
  };
  return at(i0 - 1) * w0 + at(i0) * w1 + at(i0 + 1) * w2 + at(i0 + 2) * w3;
}

__global__ void specaug_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int T, int F,
                               const int* __restrict__ lens, const int* __restrict__ warp /*B x2*/,
                               const int* __restrict__ fmask /*B x nf x2*/, int nf,
                               const int* __restrict__ tmask /*B x nt x2*/, int nt) {
  const long n = (long)B * T * F;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int f = (int)(i % F);
    const long bt = i / F;
    const int t = (int)(bt % T), b = (int)(bt / T);
    const float* xb = x + (long)b * T * F;
    const int len = lens[b];
    float v;
    if (warp && t >= len) {
      v = 0.f;  // per-utterance warp pads with 0.0 (time_warp.py:86, pad_list)
    } else if (warp && warp[2 * b] > 0) {
      const int center = warp[2 * b], warped = warp[2 * b + 1];
      if (t < warped) v = bicubic_seg(xb, F, center, warped, t, f);
      else v = bicubic_seg(xb + (long)center * F, F, len - center, len - warped, t - warped, f);
    } else {
      v = xb[(long)t * F + f];
    }
    bool m = false;
    for (int k = 0; k < nf; ++k) {
      const int p = fmask[(b * nf + k) * 2], w = fmask[(b * nf + k) * 2 + 1];
      m |= (f >= p && f < p + w);
    }
    for (int k = 0; k < nt; ++k) {
      const int p = tmask[(b * nt + k) * 2], w = tmask[(b * nt + k) * 2 + 1];
      m |= (t >= p && t < p + w);
    }
    y[i] = m ? 0.f : v;
  }
}

// UtteranceMVN (norm_means=True, norm_vars=False): zero the pad, subtract the per-utterance
// mean over valid frames from EVERY frame (pads become -mean), utterance_mvn.py:45-80.
// One block per (b, feature-chunk of 64); threads stride over time.
__global__ void mvn_kernel(float* __restrict__ x, int T, int F, const int* __restrict__ lens) {
  const int b = blockIdx.x;
  const int f = blockIdx.y * 64 + (threadIdx.x & 63);
  const int tg = threadIdx.x >> 6, ntg = blockDim.x >> 6;
  __shared__ double sh[16][64];
  const int len = lens[b];
  float* xb = x + (long)b * T * F;
  double s = 0.0;
  if (f < F)
    for (int t = tg; t < len; t += ntg) s += xb[(long)t * F + f];
  sh[tg][threadIdx.x & 63] = s;
  __syncthreads();
  double tot = 0.0;
  for (int k = 0; k < ntg; ++k) tot += sh[k][threadIdx.x & 63];
  const float mean = (float)(tot / (double)len);
  if (f < F)
    for (int t = tg; t < T; t += ntg) {
      const long o = (long)t * F + f;
      xb[o] = (t < len ? xb[o] : 0.f) - mean;
    }
}

// ------------------------------------------------------------------------- optimizer
// sum of squares of the flat gradient, stage 1 (per-block partial, fp64)
__global__ void sumsq_kernel(const float* __restrict__ g, long n, double* __restrict__ part) {
  __shared__ double sh[16];
  double s = 0.0;
  const long n4 = n / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = g4[i];
    s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += (double)g[i] * g[i];
  s = esp::block_sum<double>(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// stage 2: norm, clip coefficient (torch clip_grad_norm_: coef = max_norm/(norm+1e-6),
// clamped to 1) and finite flag. out[0]=norm, out[1]=coef, out[2]=finite(1/0)
__global__ void norm_finalize_kernel(const double* __restrict__ part, int nb, float max_norm,
                                     float* __restrict__ out) {
  __shared__ double sh[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[i];
  s = esp::block_sum<double>(s, sh);
  if (threadIdx.x == 0) {
    const float norm = (float)sqrt(s);
    float coef = max_norm / (norm + 1e-6f);
    coef = coef < 1.f ? coef : 1.f;
    out[0] = norm;
    out[1] = coef;
    out[2] = isfinite(norm) ? 1.f : 0.f;
  }
}

// torch.optim.Adam (L2 weight_decay added to the gradient), step `t` (1-based), applied to the flat
// buffers; grad is first multiplied by the clip coefficient.  Skips entirely when the finite flag is 0
// (trainer.py:651-667).  AMS (amsgrad=True): the denominator takes the running maximum of exp_avg_sq,
// kept in vmax (torch: max_exp_avg_sqs = maximum(max_exp_avg_sqs, exp_avg_sq)).
template <bool AMS>
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, float* __restrict__ vmax, long n, const float* __restrict__ clip,
                            float lr, float omb1, float b2, float omb2, float eps, float wd, float bc1,
                            float bc2_sqrt, const float* __restrict__ hyper) {
  if (clip[2] == 0.f) return;
  if (hyper) {  // device-resident step hyper-parameters (HIP-graph replay): {lr, bc1, sqrt(bc2)}
    lr = hyper[0];
    bc1 = hyper[1];
    bc2_sqrt = hyper[2];
  }
  const float coef = clip[1];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float gi = g[i] * coef;
    const float pi = p[i];
    if (wd != 0.f) gi += wd * pi;
    const float m0 = m[i];
    const float mi = m0 + omb1 * (gi - m0);  // torch: exp_avg.lerp_(grad, 1-beta1)
    const float vi = b2 * v[i] + omb2 * gi * gi;  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1-beta2)
    m[i] = mi;
    v[i] = vi;
    float vd = vi;
    if constexpr (AMS) {
      vd = fmaxf(vmax[i], vi);
      vmax[i] = vd;
    }
    const float denom = sqrtf(vd) / bc2_sqrt + eps;
    p[i] = pi - (lr / bc1) * (mi / denom);
  }
}

}  // namespace

ESP_API int esp_act_bwd(const float* dy, const float* h, float* dx, long n, int act, float drop_p,
                        unsigned long long seed, long idx_off, void* stream) {
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, dy, h, dx, n, act,
                     thr, esp::drop_scale(thr), (uint64_t)seed, idx_off, esp::rng_key_ptr());
  ESP_CHECK_LAUNCH("esp_act_bwd");
  return 0;
}

ESP_API int esp_scale_dropout(const float* x, float* y, long n, float alpha, float drop_p, unsigned long long seed,
                              const float* r, float beta, void* stream) {
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  if (n % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)r & 15) == 0)
    hipLaunchKernelGGL(scale_drop4_kernel, dim3(grid_for(n / 4)), dim3(256), 0, (hipStream_t)stream, x, y, n / 4,
                       alpha, thr, esp::drop_scale(thr), (uint64_t)seed, r, beta, esp::rng_key_ptr());
  else
    hipLaunchKernelGGL(scale_drop_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, y, n, alpha, thr,
                       esp::drop_scale(thr), (uint64_t)seed, r, beta, esp::rng_key_ptr());
  ESP_CHECK_LAUNCH("esp_scale_dropout");
  return 0;
}

ESP_API int esp_scale_dropout_planes(const float* x, void* y, long n, long pstride, int nplanes, float alpha,
                                     float drop_p, unsigned long long seed, void* stream) {
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  ESP_ARG_CHECK(n % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 7) == 0 && (nplanes == 1 || nplanes == 3) &&
                    pstride % 4 == 0 && (nplanes == 1 || pstride >= n),
                "esp_scale_dropout_planes: n, pstride %% 4 == 0, aligned x / y, nplanes 1 or 3");
  const uint32_t thr = esp::drop_threshold(drop_p);
  hipLaunchKernelGGL(scale_drop4_planes_kernel, dim3(grid_for(n / 4)), dim3(256), 0, (hipStream_t)stream, x,
                     (uint16_t*)y, n / 4, pstride, nplanes, alpha, thr, esp::drop_scale(thr), (uint64_t)seed,
                     esp::rng_key_ptr());
  ESP_CHECK_LAUNCH("esp_scale_dropout_planes");
  return 0;
}

// x *= *s  (s on device: the autograd grad_output, no host sync)
ESP_API int esp_scale_by_dev(float* x, long n, const float* s, void* stream) {
  hipLaunchKernelGGL(scale_by_dev_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, s);
  ESP_CHECK_LAUNCH("esp_scale_by_dev");
  return 0;
}

ESP_API int esp_embed_fwd(const long long* tok, const float* E, const float* pe, float* y, int nrows, int L, int D,
                          float xscale, float drop_p, unsigned long long seed, void* stream) {
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  const long n = (long)nrows * D;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const int64_t*)tok, E,
                     pe, y, L, D, xscale, thr, esp::drop_scale(thr), (uint64_t)seed, n, esp::rng_key_ptr());
  ESP_CHECK_LAUNCH("esp_embed_fwd");
  return 0;
}

ESP_API int esp_embed_bwd(const long long* tok, const float* dy, float* dE, int nrows, int V, int D, float xscale,
                          float drop_p, unsigned long long seed, void* stream) {
  ESP_ARG_CHECK(D <= EMB_MAXD, "esp_embed_bwd: D > 1024");
  ESP_ARG_CHECK(drop_p < 1.f, "dropout p must be < 1 (got %g)", (double)drop_p);
  const uint32_t thr = esp::drop_threshold(drop_p);
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(V), dim3(256), 0, (hipStream_t)stream, (const int64_t*)tok, dy, dE, nrows,
                     D, xscale, thr, esp::drop_scale(thr), (uint64_t)seed, esp::rng_key_ptr());
  ESP_CHECK_LAUNCH("esp_embed_bwd");
  return 0;
}

ESP_API int esp_specaug(const float* x, float* y, int B, int T, int F, const int* lens, const int* warp,
                        const int* fmask, int nf, const int* tmask, int nt, void* stream) {
  ESP_ARG_CHECK(x != y, "esp_specaug: in-place not supported");
  const long n = (long)B * T * F;
  hipLaunchKernelGGL(specaug_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, y, B, T, F, lens, warp,
                     fmask, nf, tmask, nt);
  ESP_CHECK_LAUNCH("esp_specaug");
  return 0;
}

ESP_API int esp_utterance_mvn(float* x, int B, int T, int F, const int* lens, void* stream) {
  hipLaunchKernelGGL(mvn_kernel, dim3(B, (F + 63) / 64), dim3(1024), 0, (hipStream_t)stream, x, T, F, lens);
  ESP_CHECK_LAUNCH("esp_utterance_mvn");
  return 0;
}

// workspace: 1024 doubles (esp_grad_norm_workspace_bytes); out: 3 floats (norm, clip coef, finite
// flag) on device
constexpr int GN_BLOCKS = 1024;
ESP_API long esp_grad_norm_workspace_bytes(long n) { return n < 0 ? 0 : 8L * GN_BLOCKS; }
ESP_API int esp_grad_norm(const float* g, long n, float max_norm, double* work, long work_bytes, float* out,
                          void* stream) {
  const int nb = GN_BLOCKS;
  const long need__ = esp_grad_norm_workspace_bytes(n);
  ESP_ARG_CHECK(work_bytes >= need__, "esp_grad_norm: workspace %ld B < %ld B required (esp_grad_norm_workspace_bytes)", work_bytes, need__);
  hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, g, n, work);
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, work, nb, max_norm, out);
  ESP_CHECK_LAUNCH("esp_grad_norm");
  return 0;
}

ESP_API int esp_adam(float* p, const float* g, float* m, float* v, long n, const float* clip, float lr, double b1,
                     double b2, float eps, float wd, int step, void* stream) {
  ESP_ARG_CHECK(step >= 1, "esp_adam: step must be >= 1");
  const float bc1 = (float)(1.0 - pow(b1, (double)step));  // python-float math, as torch
  const float bc2s = (float)sqrt(1.0 - pow(b2, (double)step));  // torch: (1 - beta2 ** step) ** 0.5
  hipLaunchKernelGGL(adam_kernel<false>, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, nullptr,
                     n, clip, lr, (float)(1.0 - b1), (float)b2, (float)(1.0 - b2), eps, wd, bc1, bc2s, nullptr);
  ESP_CHECK_LAUNCH("esp_adam");
  return 0;
}

ESP_API int esp_adam_amsgrad(float* p, const float* g, float* m, float* v, float* vmax, long n, const float* clip,
                             float lr, double b1, double b2, float eps, float wd, int step, void* stream) {
  ESP_ARG_CHECK(step >= 1 && vmax, "esp_adam_amsgrad: step must be >= 1 and vmax non-NULL");
  const float bc1 = (float)(1.0 - pow(b1, (double)step));
  const float bc2s = (float)sqrt(1.0 - pow(b2, (double)step));  // torch: (1 - beta2 ** step) ** 0.5
  hipLaunchKernelGGL(adam_kernel<true>, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, vmax, n,
                     clip, lr, (float)(1.0 - b1), (float)b2, (float)(1.0 - b2), eps, wd, bc1, bc2s, nullptr);
  ESP_CHECK_LAUNCH("esp_adam_amsgrad");
  return 0;
}

// ---- device-resident optimizer bookkeeping, so a whole training step can be one HIP graph.
// state[0] = Adam steps applied so far, state[1] = WarmupLR steps taken (scheduler.last_epoch).
namespace {
__global__ void opt_hyper_kernel(const double* __restrict__ state, double base_lr, double warmup, double b1, double b2,
                                 float* __restrict__ hyper) {
  const double t = state[0] + 1.0, s = state[1] + 1.0;
  double lr = base_lr;
  if (warmup > 0.0) lr = base_lr * sqrt(warmup) * fmin(1.0 / sqrt(s), s * pow(warmup, -1.5));
  hyper[0] = (float)lr;
  hyper[1] = (float)(1.0 - pow(b1, t));
  hyper[2] = (float)sqrt(1.0 - pow(b2, t));  // torch: bias_correction2_sqrt = (1 - beta2 ** step) ** 0.5
}
__global__ void opt_advance_kernel(double* __restrict__ state, const float* __restrict__ clip) {
  if (clip[2] != 0.f) {
    state[0] += 1.0;
    state[1] += 1.0;
  }
}
__global__ void rng_advance_kernel(unsigned long long* __restrict__ key) {
  uint64_t z = *key + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  *key = z ^ (z >> 31);
}
}  // namespace

ESP_API int esp_opt_hyper(const double* state, double base_lr, double warmup, double b1, double b2, float* hyper,
                          void* stream) {
  hipLaunchKernelGGL(opt_hyper_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, state, base_lr, warmup, b1, b2, hyper);
  ESP_CHECK_LAUNCH("esp_opt_hyper");
  return 0;
}

ESP_API int esp_adam_dev(float* p, const float* g, float* m, float* v, long n, const float* clip, const float* hyper,
                         double b1, double b2, float eps, float wd, void* stream) {
  hipLaunchKernelGGL(adam_kernel<false>, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, nullptr,
                     n, clip, 0.f, (float)(1.0 - b1), (float)b2, (float)(1.0 - b2), eps, wd, 1.f, 1.f, hyper);
  ESP_CHECK_LAUNCH("esp_adam_dev");
  return 0;
}

ESP_API int esp_adam_dev_amsgrad(float* p, const float* g, float* m, float* v, float* vmax, long n, const float* clip,
                                 const float* hyper, double b1, double b2, float eps, float wd, void* stream) {
  ESP_ARG_CHECK(vmax != nullptr, "esp_adam_dev_amsgrad: vmax is NULL");
  hipLaunchKernelGGL(adam_kernel<true>, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, vmax, n,
                     clip, 0.f, (float)(1.0 - b1), (float)b2, (float)(1.0 - b2), eps, wd, 1.f, 1.f, hyper);
  ESP_CHECK_LAUNCH("esp_adam_dev_amsgrad");
  return 0;
}

ESP_API int esp_opt_advance(double* state, const float* clip, void* stream) {
  hipLaunchKernelGGL(opt_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, state, clip);
  ESP_CHECK_LAUNCH("esp_opt_advance");
  return 0;
}

ESP_API int esp_rng_advance(unsigned long long* key, void* stream) {
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, key);
  ESP_CHECK_LAUNCH("esp_rng_advance");
  return 0;
}

// ------------------------------------------------------------------------- bf16 operand casts
// Operands of the bf16-operand GEMM (esp_gemm_bf16), round-to-nearest-even.  Plain: y[r, c] =
// bf16(x[r, c]) with 4 columns per thread; transposed: y[c, r] through a 64 x 64 LDS tile
// (coalesced on both sides), for the weight-gradient operands dY^T and X^T and for W^T.
namespace {
__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));  // inf/nan
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__global__ void f32_to_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, long rows, int cols, long ldx,
                                   long ldy) {
  const int cq = (cols + 3) / 4;
  const long n = rows * cq;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cq;
    const int c = (int)(i - r * cq) * 4;
    const float* src = x + r * ldx + c;
    uint16_t* dst = y + r * ldy + c;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (c + e < cols) dst[e] = bf16_rne(src[e]);
  }
}
// the wide form: 8 columns per thread (two float4 loads, one 16-B store); cols % 8 == 0, ldx and
// ldy % 8 == 0, 16-B aligned x and y
__global__ void f32_to_bf16_8_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, long rows, int cols,
                                     long ldx, long ldy) {
  const int c8 = cols >> 3;
  const long n = rows * c8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / c8;
    const int c = (int)(i - r * c8) * 8;
    const float4 a = *reinterpret_cast<const float4*>(x + r * ldx + c);
    const float4 b = *reinterpret_cast<const float4*>(x + r * ldx + c + 4);
    uint4 o;
    o.x = bf16_rne(a.x) | ((uint32_t)bf16_rne(a.y) << 16);
    o.y = bf16_rne(a.z) | ((uint32_t)bf16_rne(a.w) << 16);
    o.z = bf16_rne(b.x) | ((uint32_t)bf16_rne(b.y) << 16);
    o.w = bf16_rne(b.z) | ((uint32_t)bf16_rne(b.w) << 16);
    *reinterpret_cast<uint4*>(y + r * ldy + c) = o;
  }
}
__global__ __launch_bounds__(256) void f32_to_bf16_t_kernel(const float* __restrict__ x, uint16_t* __restrict__ y,
                                                            long rows, int cols, long ldx, long ldy) {
  __shared__ uint16_t tile[64][66];
  const long r0 = (long)blockIdx.y * 64;
  const int c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int k = ty; k < 64; k += 4) {
    const long r = r0 + k;
    const int c = c0 + tx;
    tile[k][tx] = (r < rows && c < cols) ? bf16_rne(x[r * ldx + c]) : (uint16_t)0;
  }
  __syncthreads();
  for (int k = ty; k < 64; k += 4) {
    const int c = c0 + k;
    const long r = r0 + tx;
    if (c < cols && r < rows) y[(long)c * ldy + r] = tile[tx][k];
  }
}
}  // namespace

ESP_API int esp_f32_to_bf16(const float* x, void* y, long rows, int cols, long ldx, long ldy, int transpose,
                            void* stream) {
  ESP_ARG_CHECK(rows >= 0 && cols >= 0, "esp_f32_to_bf16: bad sizes");
  if (rows == 0 || cols == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (transpose) {
    ESP_ARG_CHECK((rows + 63) / 64 <= 65535, "esp_f32_to_bf16: too many rows for the transposed cast");
    hipLaunchKernelGGL(f32_to_bf16_t_kernel, dim3((cols + 63) / 64, (unsigned)((rows + 63) / 64)), dim3(256), 0, st,
                       x, (uint16_t*)y, rows, cols, ldx, ldy);
  } else if (cols % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    hipLaunchKernelGGL(f32_to_bf16_8_kernel, dim3(grid_for(rows * (cols / 8))), dim3(256), 0, st, x, (uint16_t*)y,
                       rows, cols, ldx, ldy);
  } else {
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for(rows * ((cols + 3) / 4))), dim3(256), 0, st, x,
                       (uint16_t*)y, rows, cols, ldx, ldy);
  }
  ESP_CHECK_LAUNCH("esp_f32_to_bf16");
  return 0;
}
