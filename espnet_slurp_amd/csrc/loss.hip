// Loss kernels of the hybrid CTC/attention objective (espnet_model.py:169-297):
//   * row log-softmax (CTC input, ctc.py:53)
//   * CTC alpha/beta (one block per utterance and direction, the two recursions run
//     concurrently) and the per-frame gradient w.r.t. the logits, following PyTorch's
//     CPU ctc_loss (max-shifted 3-way log-sum-exp, zero_infinity, grad
//     exp(lp) - exp(lcab + nll - lp), then log_softmax's adjoint)   [ctc.py:39-60]
//   * label-smoothed KL (t*log t included) + gradient + th_accuracy counts
//     [label_smoothing_loss.py:41-63, nets_utils.py:299-320]
//   * deterministic final reduction to the reported scalars
//   * CTC.argmax (ctc.py:119-127) and espnet1 CTC.forced_align Viterbi
//     (espnet/nets/pytorch_backend/ctc.py:185-249) with its fp32-add and s=0 wrap quirks.
#include "common.h"

namespace {

// log(e^a + e^b + e^c) with the max shift; the recursion values stay fp64 (alpha/beta reach
// -O(10^3): an fp32 running value would round by ~1e-4 per frame), the O(1) shifted
// exponentials are evaluated in fp32 (relative 1e-7, i.e. 1e-7 absolute after the log)
__device__ __forceinline__ double lse3(double a, double b, double c) {
  const double m = fmax(a, fmax(b, c));
  if (m == -INFINITY) return -INFINITY;
  return (double)logf(expf((float)(a - m)) + expf((float)(b - m)) + expf((float)(c - m))) + m;
}

// block-per-row log-softmax, any V
__global__ void log_softmax_kernel(const float* __restrict__ x, float* __restrict__ y, int V) {
  __shared__ float sh[16];
  const long row = blockIdx.x;
  const float* xr = x + row * V;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < V; c += blockDim.x) m = fmaxf(m, xr[c]);
  m = esp::block_max(m, sh);
  __shared__ double shd[16];
  double s = 0.0;
  for (int c = threadIdx.x; c < V; c += blockDim.x) s += (double)expf(xr[c] - m);
  s = esp::block_sum<double>(s, shd);
  const double lse = (double)m + log(s);
  float* yr = y + row * V;
  for (int c = threadIdx.x; c < V; c += blockDim.x) yr[c] = (float)((double)xr[c] - lse);
}

// blockIdx.x = utterance, blockIdx.y = 0 alpha / 1 beta.  lp: (B, T, V) log-probs.
// labels (B, Umax) int64 (row b valid for tlen[b]); la/lb: (B, T, Smax) outputs.
constexpr int CTC_NT = 256, CTC_SPT = 4;  // states per thread -> S <= 1024
__global__ __launch_bounds__(CTC_NT) void ctc_alpha_beta_kernel(const float* __restrict__ lp, const int64_t* __restrict__ labels,
                                                                int Umax, const int* __restrict__ ilen,
                                                                const int* __restrict__ tlen, int T, int V, int Smax,
                                                                int blank, double* __restrict__ la, double* __restrict__ lb,
                                                                double* __restrict__ nll) {
  const int b = blockIdx.x;
  const int dir = blockIdx.y;
  const int Tb = ilen[b], U = tlen[b], S = 2 * U + 1;
  __shared__ double buf[2][CTC_NT * CTC_SPT + 2];
  __shared__ int lab[CTC_NT * CTC_SPT + 2];
  const float* lpb = lp + (long)b * T * V;
  for (int s = threadIdx.x; s < S + 2; s += CTC_NT) {
    int l = blank;
    if (s < S && (s & 1)) l = (int)labels[(long)b * Umax + (s >> 1)];
    lab[s] = l;
  }
  __syncthreads();
  double* out = (dir == 0 ? la : lb) + (long)b * T * Smax;
  if (Tb <= 0) {
    if (dir == 0 && threadIdx.x == 0) nll[b] = INFINITY;
    return;
  }
  int cur = 0;
  if (dir == 0) {
    for (int s = threadIdx.x; s < S; s += CTC_NT) {
      double v = -INFINITY;
      if (s == 0) v = lpb[blank];
      else if (s == 1) v = lpb[lab[1]];
      buf[0][s] = v;
      out[s] = v;
    }
    __syncthreads();
    for (int t = 1; t < Tb; ++t) {
      const float* lpt = lpb + (long)t * V;
      for (int s = threadIdx.x; s < S; s += CTC_NT) {
        const double v = lse3(buf[cur][s], s > 0 ? buf[cur][s - 1] : -INFINITY,
                              (s > 1 && lab[s] != lab[s - 2]) ? buf[cur][s - 2] : -INFINITY) +
                         (double)lpt[lab[s]];
        buf[cur ^ 1][s] = v;
        out[(long)t * Smax + s] = v;
      }
      cur ^= 1;
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      nll[b] = -lse3(buf[cur][S - 1], S > 1 ? buf[cur][S - 2] : -INFINITY, -INFINITY);
    }
  } else {
    const float* lpt0 = lpb + (long)(Tb - 1) * V;
    for (int s = threadIdx.x; s < S; s += CTC_NT) {
      double v = -INFINITY;
      if (s == S - 1) v = lpt0[blank];
      else if (s == S - 2) v = lpt0[lab[S - 2]];
      buf[0][s] = v;
      out[(long)(Tb - 1) * Smax + s] = v;
    }
    __syncthreads();
    for (int t = Tb - 2; t >= 0; --t) {
      const float* lpt = lpb + (long)t * V;
      for (int s = threadIdx.x; s < S; s += CTC_NT) {
        const double v = lse3(buf[cur][s], s < S - 1 ? buf[cur][s + 1] : -INFINITY,
                              (s < S - 2 && lab[s] != lab[s + 2]) ? buf[cur][s + 2] : -INFINITY) +
                         (double)lpt[lab[s]];
        buf[cur ^ 1][s] = v;
        out[(long)t * Smax + s] = v;
      }
      cur ^= 1;
      __syncthreads();
    }
  }
}

// grid (T, B): gradient of gscale * nll_b w.r.t. the logits for frame t of utterance b
constexpr int MAXV_LDS = 8192;
__global__ __launch_bounds__(256) void ctc_grad_kernel(const float* __restrict__ lp, const int64_t* __restrict__ labels,
                                                       int Umax, const int* __restrict__ ilen,
                                                       const int* __restrict__ tlen, int T, int V, int Smax, int blank,
                                                       const double* __restrict__ la, const double* __restrict__ lb,
                                                       const double* __restrict__ nll, float gscale, int zero_infinity,
                                                       float* __restrict__ grad) {
  __shared__ float occ[MAXV_LDS];
  __shared__ float sh[16];
  __shared__ double shd[16];
  const int t = blockIdx.x, b = blockIdx.y;
  const int Tb = ilen[b], U = tlen[b], S = 2 * U + 1;
  float* gr = grad + ((long)b * T + t) * V;
  const double nl = nll[b];
  if (t >= Tb || (zero_infinity && isinf(nl))) {
    for (int c = threadIdx.x; c < V; c += blockDim.x) gr[c] = 0.f;
    return;
  }
  for (int c = threadIdx.x; c < V; c += blockDim.x) occ[c] = 0.f;
  const double* lat = la + ((long)b * T + t) * Smax;
  const double* lbt = lb + ((long)b * T + t) * Smax;
  double m = -INFINITY;
  for (int s = threadIdx.x; s < S; s += blockDim.x) m = fmax(m, lat[s] + lbt[s]);
  m = esp::block_max<double>(m, shd);  // includes a barrier: occ is zeroed before the adds below
  if (m != -INFINITY) {
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
      const int l = (s & 1) ? (int)labels[(long)b * Umax + (s >> 1)] : blank;
      const double v = lat[s] + lbt[s];
      if (v != -INFINITY) atomicAdd(&occ[l], expf((float)(v - m)));
    }
  }
  __syncthreads();
  const float* lpt = lp + ((long)b * T + t) * V;
  const double mn = m + nl;  // log occupancy offset: exp(lcab + nll - lp) = occ * exp(m + nll - lp)
  float gs = 0.f;
  for (int c = threadIdx.x; c < V; c += blockDim.x) {
    const float l = lpt[c];
    const float o = occ[c];
    const float q = o > 0.f ? o * expf((float)(mn - (double)l)) : 0.f;
    gs += expf(l) - q;
  }
  gs = esp::block_sum<float>(gs, sh);
  for (int c = threadIdx.x; c < V; c += blockDim.x) {
    const float l = lpt[c];
    const float o = occ[c];
    const float q = o > 0.f ? o * expf((float)(mn - (double)l)) : 0.f;
    const float e = expf(l);
    gr[c] = (e - q) * gscale - e * (gs * gscale);
  }
}

// label smoothing: block per row.  rows with target == ignore get zero loss/grad.
__global__ __launch_bounds__(256) void ls_kernel(const float* __restrict__ x, const int64_t* __restrict__ target,
                                                 int V, int ignore, float smoothing, float gscale,
                                                 float* __restrict__ grad, double* __restrict__ row_loss,
                                                 int* __restrict__ row_stat) {
  __shared__ float sh[16];
  __shared__ int shi[16];
  const long row = blockIdx.x;
  const float* xr = x + row * V;
  float* gr = grad ? grad + row * V : nullptr;
  const int64_t tg = target[row];
  if (tg == ignore) {
    if (gr)
      for (int c = threadIdx.x; c < V; c += blockDim.x) gr[c] = 0.f;
    if (threadIdx.x == 0) {
      row_loss[row] = 0.0;
      row_stat[2 * row] = 0;
      row_stat[2 * row + 1] = 0;
    }
    return;
  }
  // max + first argmax
  float m = -INFINITY;
  int am = 0x7fffffff;
  for (int c = threadIdx.x; c < V; c += blockDim.x) {
    const float v = xr[c];
    if (v > m) { m = v; am = c; }
  }
  // wave/block argmax with first-index tie-break
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > m || (om == m && oa < am)) { m = om; am = oa; }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) { sh[w] = m; shi[w] = am; }
  __syncthreads();
  m = sh[0];
  am = shi[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i)
    if (sh[i] > m || (sh[i] == m && shi[i] < am)) { m = sh[i]; am = shi[i]; }
  __syncthreads();
  __shared__ double shd[16];
  double s = 0.0, slp = 0.0;
  for (int c = threadIdx.x; c < V; c += blockDim.x) {
    s += (double)expf(xr[c] - m);
    slp += (double)xr[c];
  }
  s = esp::block_sum<double>(s, shd);
  slp = esp::block_sum<double>(slp, shd);
  const double lse_d = (double)m + log(s);
  const float lse = (float)lse_d;
  const float conf = 1.0f - smoothing;
  const float sv = smoothing / (float)(V - 1);
  if (threadIdx.x == 0) {  // KL(true_dist || p) in fp64 from the fp32 logits
    const double lpt = (double)xr[tg] - lse_d;
    const double sum_lp = slp - (double)V * lse_d;
    const double cd = 1.0 - (double)smoothing, svd = (double)smoothing / (double)(V - 1);
    double l = 0.0;
    if (conf > 0.f) l += cd * (log(cd) - lpt);
    if (sv > 0.f) l += svd * ((double)(V - 1) * log(svd) - (sum_lp - lpt));
    row_loss[row] = l;
    row_stat[2 * row] = (am == (int)tg) ? 1 : 0;
    row_stat[2 * row + 1] = 1;
  }
  if (gr) {
    const float tot = conf + sv * (float)(V - 1);
    for (int c = threadIdx.x; c < V; c += blockDim.x) {
      const float p = expf(xr[c] - lse);
      const float td = (c == (int)tg) ? conf : sv;
      gr[c] = (p * tot - td) * gscale;
    }
  }
}

// out[0] = ctc loss = sum_b nll_b' / B ;  out[1] = att loss = sum rows / denom ;
// out[2] = acc ; out[3] = w*out[0] + (1-w)*out[1].  One block, fixed order.
__global__ void reduce_losses_kernel(const double* __restrict__ nll, int B, int zero_inf, const double* __restrict__ row_loss,
                                     const int* __restrict__ row_stat, int R, float denom, float ctc_w,
                                     float* __restrict__ out) {
  __shared__ double shd[16];
  double a = 0.0;
  for (int i = threadIdx.x; i < B && nll; i += blockDim.x) {
    double v = nll[i];
    if (zero_inf && isinf(v)) v = 0.0;
    a += v;
  }
  a = esp::block_sum<double>(a, shd);
  double l = 0.0, c = 0.0, n = 0.0;
  for (int i = threadIdx.x; i < R && row_loss; i += blockDim.x) {
    l += row_loss[i];
    c += row_stat[2 * i];
    n += row_stat[2 * i + 1];
  }
  l = esp::block_sum<double>(l, shd);
  c = esp::block_sum<double>(c, shd);
  n = esp::block_sum<double>(n, shd);
  if (threadIdx.x == 0) {
    const double lc = nll ? a / B : 0.0;
    // denom <= 0: length-normalised loss (label_smoothing_loss.py:56-60 normalize_length):
    // the count of non-ignored targets of THIS batch, taken on device (a captured graph
    // must not bake a host value); its reciprocal goes to out[4] for the gradient scale
    const double dn = denom > 0.f ? (double)denom : n;
    const double lat = row_loss ? l / dn : 0.0;
    if (denom <= 0.f) out[4] = (float)(1.0 / dn);
    out[0] = (float)lc;
    out[1] = (float)lat;
    out[2] = (n > 0) ? (float)(c / n) : 0.f;
    if (!nll) out[3] = (float)lat;
    else if (!row_loss) out[3] = (float)lc;
    else out[3] = (float)((double)ctc_w * lc + (1.0 - (double)ctc_w) * lat);
  }
}

__global__ void argmax_kernel(const float* __restrict__ x, int64_t* __restrict__ out, long rows, int V) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * V;
  float m = -INFINITY;
  int am = 0x7fffffff;
  for (int c = lane; c < V; c += 64) {
    const float v = xr[c];
    if (v > m || (v != v && m == m)) { m = v; am = c; }  // NaN propagates like torch.argmax
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > m || (om == m && oa < am)) { m = om; am = oa; }
  }
  if (lane == 0) out[row] = am == 0x7fffffff ? 0 : am;
}

// espnet1 forced_align (ctc.py:185-249), one block per sequence. lpz (T,V) fp32; y (U); out (T) labels;
// path: (T, S) int32 workspace.  The reference's quirks are kept: candidate s-1 of state 0 is Python's
// index -1 (the last state; a back-pointer -1 decodes to the last label, the blank), every step's sum is
// an fp32 add stored in a float64 table (log-zero -1e11 included), and ties keep the first candidate
// (np.argmax: stay, then s-1, then s-2; the final pair prefers S-1).
__device__ __forceinline__ void forced_align_body(const float* __restrict__ lpz, int T, int V,
                                                  const int64_t* __restrict__ y, int U, int blank,
                                                  int* __restrict__ path, int64_t* __restrict__ out, double (*dl)[1025],
                                                  int* lab) {
  const int S = 2 * U + 1;
  for (int s = threadIdx.x; s < S; s += blockDim.x) lab[s] = (s & 1) ? (int)y[s >> 1] : blank;
  __syncthreads();
  for (int s = threadIdx.x; s < S; s += blockDim.x) {
    double v = -100000000000.0;
    if (s == 0) v = (double)lpz[lab[0]];
    else if (s == 1) v = (double)lpz[lab[1]];
    dl[0][s] = v;
  }
  __syncthreads();
  int cur = 0;
  for (int t = 1; t < T; ++t) {
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
      const int sm1 = s - 1 < 0 ? S - 1 : s - 1;  // python index -1 -> last state
      const double c0 = dl[cur][s], c1 = dl[cur][sm1];
      double best = c0;
      int prev = s;
      if (c1 > best) { best = c1; prev = s - 1; }
      if (!(lab[s] == blank || s < 2 || lab[s] == lab[s - 2])) {
        const double c2 = dl[cur][s - 2];
        if (c2 > best) { best = c2; prev = s - 2; }
      }
      const float add = (float)best + lpz[(long)t * V + lab[s]];  // fp32, as the reference
      dl[cur ^ 1][s] = (double)add;
      path[(long)t * S + s] = prev;
    }
    cur ^= 1;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int st = dl[cur][S - 2] > dl[cur][S - 1] ? S - 2 : S - 1;
    out[T - 1] = lab[st];
    for (int t = T - 2; t >= 0; --t) {
      int idx = st < 0 ? st + S : st;
      st = path[(long)(t + 1) * S + idx];
      out[t] = lab[st < 0 ? st + S : st];
    }
  }
}

__global__ __launch_bounds__(1024) void forced_align_kernel(const float* __restrict__ lpz, int T, int V,
                                                            const int64_t* __restrict__ y, int U, int blank,
                                                            int* __restrict__ path, int64_t* __restrict__ out) {
  __shared__ double dl[2][1025];
  __shared__ int lab[1025];
  forced_align_body(lpz, T, V, y, U, blank, path, out, dl, lab);
}

// a batch: block b aligns utterance b (its own T_b = tlen[b] frames of lpz[b], its own U_b = ulen[b] labels
// of row b of y) exactly as one forced_align call on that utterance would; frames t >= T_b of out row b
// are -1.  path: B x T x (2 Umax + 1) int32.
__global__ __launch_bounds__(1024) void forced_align_batch_kernel(const float* __restrict__ lpz, int T, int V,
                                                                  const int* __restrict__ tlen,
                                                                  const int64_t* __restrict__ y, int Umax,
                                                                  const int* __restrict__ ulen, int blank,
                                                                  int* __restrict__ path, int64_t* __restrict__ out) {
  __shared__ double dl[2][1025];
  __shared__ int lab[1025];
  const int b = blockIdx.x;
  const int Tb = min(max(tlen[b], 0), T), Ub = min(max(ulen[b], 0), Umax);
  int64_t* ob = out + (long)b * T;
  for (int t = Tb + threadIdx.x; t < T; t += blockDim.x) ob[t] = -1;
  if (Tb < 1 || Ub < 1) {  // nothing to align (the reference needs T >= 1 and a non-empty y)
    for (int t = threadIdx.x; t < Tb; t += blockDim.x) ob[t] = -1;
    return;
  }
  forced_align_body(lpz + (long)b * T * V, Tb, V, y + (long)b * Umax, Ub, blank,
                    path + (long)b * T * (2 * Umax + 1), ob, dl, lab);
}

}  // namespace

ESP_API int esp_log_softmax(const float* x, float* y, long rows, int V, void* stream) {
  hipLaunchKernelGGL(log_softmax_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, x, y, V);
  ESP_CHECK_LAUNCH("esp_log_softmax");
  return 0;
}

// lp (B,T,V) log-probs; labels (B,Umax) int64; ilen/tlen int32 device arrays.
// Outputs: nll (B); grad (B,T,V) = gscale * d nll_b / d logits (zeroed where infinite
// when zero_infinity).  work: 2*B*T*Smax doubles, Smax = 2*Umax+1 <= 1024
// (esp_ctc_loss_workspace_bytes).
ESP_API long esp_ctc_loss_workspace_bytes(int B, int T, int Umax) {
  return B <= 0 || T <= 0 || Umax < 0 ? 0 : 8L * 2 * B * T * (2L * Umax + 1);
}
ESP_API int esp_ctc_loss(const float* lp, const long long* labels, int Umax, const int* ilen, const int* tlen, int B,
                         int T, int V, int blank, float gscale, int zero_infinity, double* nll, float* grad,
                         double* work, long work_bytes, void* stream) {
  const long need__ = esp_ctc_loss_workspace_bytes(B, T, Umax);
  ESP_ARG_CHECK(work_bytes >= need__, "esp_ctc_loss: workspace %ld B < %ld B required (esp_ctc_loss_workspace_bytes)", work_bytes, need__);
  const int Smax = 2 * Umax + 1;
  ESP_ARG_CHECK(Smax <= CTC_NT * CTC_SPT, "esp_ctc_loss: 2*Umax+1=%d > %d", Smax, CTC_NT * CTC_SPT);
  ESP_ARG_CHECK(V <= MAXV_LDS, "esp_ctc_loss: V=%d > %d", V, MAXV_LDS);
  double* la = work;
  double* lb = work + (long)B * T * Smax;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ctc_alpha_beta_kernel, dim3(B, 2), dim3(CTC_NT), 0, st, lp, (const int64_t*)labels, Umax, ilen, tlen,
                     T, V, Smax, blank, la, lb, nll);
  if (grad)
    hipLaunchKernelGGL(ctc_grad_kernel, dim3(T, B), dim3(256), 0, st, lp, (const int64_t*)labels, Umax, ilen, tlen, T, V,
                       Smax, blank, la, lb, nll, gscale, zero_infinity, grad);
  ESP_CHECK_LAUNCH("esp_ctc_loss");
  return 0;
}

ESP_API int esp_label_smoothing(const float* x, const long long* target, long rows, int V, int ignore, float smoothing,
                                float gscale, float* grad, double* row_loss, int* row_stat, void* stream) {
  hipLaunchKernelGGL(ls_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, x, (const int64_t*)target, V,
                     ignore, smoothing, gscale, grad, row_loss, row_stat);
  ESP_CHECK_LAUNCH("esp_label_smoothing");
  return 0;
}

ESP_API int esp_reduce_losses(const double* nll, int B, int zero_inf, const double* row_loss, const int* row_stat, int R,
                              float denom, float ctc_w, float* out, void* stream) {
  hipLaunchKernelGGL(reduce_losses_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, nll, B, zero_inf, row_loss,
                     row_stat, R, denom, ctc_w, out);
  ESP_CHECK_LAUNCH("esp_reduce_losses");
  return 0;
}

ESP_API int esp_argmax(const float* x, long long* out, long rows, int V, void* stream) {
  hipLaunchKernelGGL(argmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x,
                     (int64_t*)out, rows, V);
  ESP_CHECK_LAUNCH("esp_argmax");
  return 0;
}

ESP_API int esp_ctc_forced_align(const float* lpz, int T, int V, const long long* y, int U, int blank, int* path,
                                 long long* out, void* stream) {
  ESP_ARG_CHECK(2 * U + 1 <= 1024 && U >= 1 && T >= 1, "esp_ctc_forced_align: bad sizes T=%d U=%d", T, U);
  hipLaunchKernelGGL(forced_align_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, lpz, T, V, (const int64_t*)y, U,
                     blank, path, (int64_t*)out);
  ESP_CHECK_LAUNCH("esp_ctc_forced_align");
  return 0;
}

ESP_API int esp_ctc_forced_align_batch(const float* lpz, int B, int T, int V, const int* tlen, const long long* y,
                                       int Umax, const int* ulen, int blank, int* path, long long* out, void* stream) {
  ESP_ARG_CHECK(2 * Umax + 1 <= 1024 && Umax >= 1 && T >= 1 && B >= 0 && V >= 1,
                "esp_ctc_forced_align_batch: bad sizes B=%d T=%d V=%d Umax=%d", B, T, V, Umax);
  if (B == 0) return 0;
  hipLaunchKernelGGL(forced_align_batch_kernel, dim3(B), dim3(1024), 0, (hipStream_t)stream, lpz, T, V, tlen,
                     (const int64_t*)y, Umax, ulen, blank, path, (int64_t*)out);
  ESP_CHECK_LAUNCH("esp_ctc_forced_align_batch");
  return 0;
}

// ============================================================================ CTC prefix scoring
// Beam-search CTC prefix scorer (espnet/nets/ctc_prefix_score.py:279-359, CTCPrefixScore,
// used through espnet/nets/scorers/ctc.py CTCPrefixScorer): for every running hypothesis g
// (states r_prev = log r_t^n(g), log r_t^b(g), t < T) and each candidate label c, the forward
// variables of h = g + c and the prefix probability log psi(h).  fp32 like the reference's
// numpy path; logaddexp in numpy's form; logzero = -1e10.
// One thread per (hypothesis, candidate): the recursion over t is serial, the (hyp, cand)
// pairs are independent.  lp is one utterance's (T, V) log-softmax.
namespace {
constexpr float kLogZero = -10000000000.0f;
__device__ __forceinline__ float logaddexpf_np(float x, float y) {
  if (x == y) return x + 0.693147180559945309f;
  const float d = x - y;
  return d > 0.f ? x + log1pf(expf(-d)) : y + log1pf(expf(d));
}
__global__ void ctc_prefix_init_kernel(const float* __restrict__ lp, int T, int V, int blank, float* __restrict__ r) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  float acc = lp[blank];
  r[0] = kLogZero;
  r[1] = acc;
  for (int t = 1; t < T; ++t) {
    acc = acc + lp[(long)t * V + blank];
    r[2 * t] = kLogZero;
    r[2 * t + 1] = acc;
  }
}
__global__ void ctc_prefix_score_kernel(const float* __restrict__ lp, int T, int V, const float* __restrict__ r_prev,
                                        const long long* __restrict__ last, int out_len, const long long* __restrict__ cands,
                                        int NH, int C, int blank, int eos, float* __restrict__ r_new,
                                        float* __restrict__ log_psi) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NH * C) return;
  const int hy = idx / C;
  const int c = (int)cands[idx];
  const float* rp = r_prev + (long)hy * T * 2;
  float* rn = r_new + (long)idx * T * 2;
  const bool same_as_last = out_len > 0 && c == (int)last[hy];
  for (int t = 0; t < T; ++t) {  // rows before the recursion start are never read downstream
    rn[2 * t] = kLogZero;
    rn[2 * t + 1] = kLogZero;
  }
  if (out_len == 0) rn[0] = lp[c];
  const int start = out_len > 1 ? out_len : 1;
  float rn0 = rn[2 * (start - 1)], rb0 = rn[2 * (start - 1) + 1];
  float psi = rn0;
  for (int t = start; t < T; ++t) {
    const float phi = same_as_last ? rp[2 * (t - 1) + 1] : logaddexpf_np(rp[2 * (t - 1)], rp[2 * (t - 1) + 1]);
    const float xc = lp[(long)t * V + c];
    const float n1 = logaddexpf_np(rn0, phi) + xc;
    const float b1 = logaddexpf_np(rn0, rb0) + lp[(long)t * V + blank];
    psi = logaddexpf_np(psi, phi + xc);
    rn[2 * t] = n1;
    rn[2 * t + 1] = b1;
    rn0 = n1;
    rb0 = b1;
  }
  if (c == eos) psi = logaddexpf_np(rp[2 * (T - 1)], rp[2 * (T - 1) + 1]);
  if (c == blank) psi = kLogZero;
  log_psi[idx] = psi;
}
}  // namespace

ESP_API int esp_ctc_prefix_init(const float* lp, int T, int V, int blank, float* r0, void* stream) {
  ESP_ARG_CHECK(T >= 1 && V >= 1 && blank >= 0 && blank < V, "esp_ctc_prefix_init: bad sizes T=%d V=%d", T, V);
  hipLaunchKernelGGL(ctc_prefix_init_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, lp, T, V, blank, r0);
  ESP_CHECK_LAUNCH("esp_ctc_prefix_init");
  return 0;
}

ESP_API int esp_ctc_prefix_score(const float* lp, int T, int V, const float* r_prev, const long long* last,
                                 int out_len, const long long* cands, int NH, int C, int blank, int eos,
                                 float* r_new, float* log_psi, void* stream) {
  ESP_ARG_CHECK(T >= 1 && V >= 1 && NH >= 1 && C >= 1 && out_len >= 0 && out_len <= T,
                "esp_ctc_prefix_score: bad sizes T=%d V=%d NH=%d C=%d out_len=%d", T, V, NH, C, out_len);
  const int n = NH * C;
  hipLaunchKernelGGL(ctc_prefix_score_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, lp, T, V, r_prev,
                     last, out_len, cands, NH, C, blank, eos, r_new, log_psi);
  ESP_CHECK_LAUNCH("esp_ctc_prefix_score");
  return 0;
}
