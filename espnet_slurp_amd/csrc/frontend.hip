// Feature front end: DefaultFrontend = STFT -> power -> LogMel
// (espnet2/asr/frontend/default.py:82-131, layers/stft.py:63-160, layers/log_mel.py:57-81) and
// GlobalMVN (layers/global_mvn.py:67-90).
//
// esp_fbank_fwd: one wave per frame, the whole chain in LDS/registers — HBM sees the raw
// samples once and the log-mel features once (memory-bound: ~(hop + n_mels) * 4 B per frame).
//   1. frame t of utterance b: samples t*hop - n_fft/2 + k (torch.stft center=True: reflect
//      padding at the edges of the (B, N) tensor, N = max length in the batch), x window.
//      A length-bucketed batch (the HIP-graph trainer) pads the samples past N; the reflection
//      point stays the reference batch's N, read from the device (nvalid)
//   2. n_fft-point complex FFT (radix-2, decimation in time, bit-reversed load), fp32; for an
//      n_fft that is not a power of two (e.g. 400) a direct DFT per bin over the same twiddle
//      table (exp(-2 pi i j / n_fft), j < n_fft) instead
//   3. power of the onesided bins; mel band sums over each filter's nonzero bin range (the
//      reference's dense matmul adds exact zeros elsewhere); clamp 1e-10; log
//   4. frames t >= olen[b] = len_b // hop + 1 are written as 0 (stft.py:150-158, log_mel.py:73)
#include "common.h"

namespace {

constexpr int FB_WAVES = 4;  // frames per block

__global__ __launch_bounds__(64 * FB_WAVES) void fbank_kernel(
    const float* __restrict__ wave, long ldw, const int* __restrict__ lens, int N, int T, int n_fft, int log2n,
    int hop, const float* __restrict__ window, const float2* __restrict__ twiddle, const float* __restrict__ melw,
    const int* __restrict__ mlo, const int* __restrict__ mhi, int n_mels, float* __restrict__ out,
    const int* __restrict__ nvalid) {
  extern __shared__ __attribute__((aligned(16))) float2 fbuf[];  // [FB_WAVES][n_fft] complex + power
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int t = blockIdx.x * FB_WAVES + w;
  float2* a = fbuf + (long)w * (n_fft + n_fft / 2 + 1);
  float* pw = reinterpret_cast<float*>(a + n_fft);
  const int olen = lens[b] / hop + 1;
  const bool live = t < T && t < olen;
  if (nvalid) N = min(max(*nvalid, n_fft / 2 + 1), N);

  // 1. windowed frame, stored at bit-reversed positions
  const float* xb = wave + (long)b * ldw;
  for (int k = lane; k < n_fft; k += 64) {
    float v = 0.f;
    if (live) {
      int p = t * hop + k - n_fft / 2;
      if (p < 0) p = -p;                       // reflect (torch pad_mode="reflect")
      if (p >= N) p = 2 * N - 2 - p;
      v = xb[p] * window[k];
    }
    const int r = log2n ? (int)(__brev((unsigned)k) >> (32 - log2n)) : k;
    a[r] = make_float2(v, 0.f);
  }
  __syncthreads();
  const int nb = n_fft / 2 + 1;
  if (!log2n) {  // direct DFT (n_fft not a power of two): bins f = lane, lane + 64, ...
    for (int f = lane; f < nb; f += 64) {
      float re = 0.f, im = 0.f;
      int idx = 0;
      for (int k = 0; k < n_fft; ++k) {
        const float2 wv = twiddle[idx];
        const float xv = a[k].x;
        re += xv * wv.x;
        im += xv * wv.y;
        idx += f;
        if (idx >= n_fft) idx -= n_fft;
      }
      pw[f] = re * re + im * im;
    }
    __syncthreads();
  }
  // 2. radix-2 DIT butterflies; twiddle[j] = exp(-2 pi i j / n_fft)
  for (int s = 1; s <= log2n; ++s) {
    const int half = 1 << (s - 1);
    const int tstep = n_fft >> s;
    for (int j = lane; j < n_fft / 2; j += 64) {
      const int pos = j & (half - 1);
      const int i1 = ((j >> (s - 1)) << s) + pos;
      const int i2 = i1 + half;
      const float2 wv = twiddle[pos * tstep];
      const float2 u = a[i1], v = a[i2];
      const float2 tv = make_float2(wv.x * v.x - wv.y * v.y, wv.x * v.y + wv.y * v.x);
      a[i1] = make_float2(u.x + tv.x, u.y + tv.y);
      a[i2] = make_float2(u.x - tv.x, u.y - tv.y);
    }
    __syncthreads();
  }
  // 3. power spectrum of the onesided bins
  if (log2n) {
    for (int f = lane; f < nb; f += 64) {
      const float2 c = a[f];
      pw[f] = c.x * c.x + c.y * c.y;
    }
    __syncthreads();
  }
  if (t >= T) return;
  float* o = out + ((long)b * T + t) * n_mels;
  for (int m = lane; m < n_mels; m += 64) {
    float acc = 0.f;
    if (live) {
      for (int f = mlo[m]; f < mhi[m]; ++f) acc += pw[f] * melw[(long)f * n_mels + m];
      acc = logf(fmaxf(acc, 1e-10f));
    }
    o[m] = acc;
  }
}

// GlobalMVN: y = ((x - mean) masked) / std, frames t >= lens[b] -> 0 (global_mvn.py:67-90)
__global__ void global_mvn_kernel(float* __restrict__ x, const int* __restrict__ lens, int B, int T, int F,
                                  const float* __restrict__ mean, const float* __restrict__ stdv, int norm_means,
                                  int norm_vars) {
  const long n = (long)B * T * F;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int f = (int)(i % F);
    const long r = i / F;
    const int t = (int)(r % T);
    const int b = (int)(r / T);
    float v = x[i];
    if (norm_means) v = v - mean[f];
    if (t >= lens[b]) v = 0.f;
    if (norm_vars) v = v / stdv[f];
    x[i] = v;
  }
}

}  // namespace

ESP_API int esp_fbank_fwd(const float* wave, long ldw, const int* lens, int B, int N, int n_fft, int hop,
                          const float* window, const float* twiddle, const float* melw, const int* mel_lo,
                          const int* mel_hi, int n_mels, float* out, int T, const int* nvalid, void* stream) {
  int log2n = 0;
  while ((1 << log2n) < n_fft) ++log2n;
  if ((1 << log2n) != n_fft) log2n = 0;  // direct-DFT path
  ESP_ARG_CHECK(n_fft >= 16 && n_fft <= 2048 && n_fft % 2 == 0, "esp_fbank_fwd: n_fft=%d must be even, in [16, 2048]",
                n_fft);
  ESP_ARG_CHECK(B >= 1 && N >= n_fft / 2 + 1 && hop >= 1 && n_mels >= 1 && n_mels <= 1024 && T >= 1 && ldw >= N,
                "esp_fbank_fwd: bad sizes B=%d N=%d hop=%d T=%d (reflect padding needs N > n_fft/2)", B, N, hop, T);
  const size_t shm = (size_t)FB_WAVES * (n_fft + n_fft / 2 + 1) * sizeof(float2);
  dim3 grid((unsigned)((T + FB_WAVES - 1) / FB_WAVES), (unsigned)B);
  hipLaunchKernelGGL(fbank_kernel, grid, dim3(64 * FB_WAVES), shm, (hipStream_t)stream, wave, ldw, lens, N, T, n_fft,
                     log2n, hop, window, reinterpret_cast<const float2*>(twiddle), melw, mel_lo, mel_hi, n_mels, out,
                     nvalid);
  ESP_CHECK_LAUNCH("esp_fbank_fwd");
  return 0;
}

ESP_API int esp_global_mvn(float* x, const int* lens, int B, int T, int F, const float* mean, const float* stdv,
                           int norm_means, int norm_vars, void* stream) {
  const long n = (long)B * T * F;
  long nb = (n + 255) / 256;
  if (nb > 65536) nb = 65536;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(global_mvn_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, x, lens, B, T, F, mean,
                     stdv, norm_means, norm_vars);
  ESP_CHECK_LAUNCH("esp_global_mvn");
  return 0;
}
