// Conv2dSubsampling pieces (subsampling.py:42-87) in NHWC layout:
//   conv1  Conv2d(1, D, 3, stride 2) + ReLU : direct kernel (K = 9, not GEMM-shaped)
//   conv2  Conv2d(D, D, 3, stride 2) + ReLU : implicit-im2col MFMA GEMM (gemm.hip)
//   adjoints: col2im gather (+ conv1 ReLU mask), conv1 weight gradient, and the weight
//   re-layouts between the reference (o, c, kt, kf) / (n, c*F2+f) order and the NHWC
//   order the GEMMs consume (forward copy; gradient scattered back, accumulated).
#include "common.h"

namespace {

inline int gridn(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 65536 ? 65536 : (b < 1 ? 1 : b));
}

// x (B,T,F) -> z (B,T1,F1,D).  A thread owns 4 output channels (weights + bias in registers,
// loaded once) and strides over pixels; a wave covers 64 channel quads of one pixel, so the
// 9-tap patch load is a broadcast and the store is 1 KB contiguous per wave.
// z16 != nullptr (the bf16 mode): the output's bf16 copy too (RNE), the A operand of the bf16 conv2
// forward (esp_conv2_fwd_bf16); z stays fp32 for the weight gradient's gather and the ReLU mask
#ifndef ESP_CONV1_NT
#define ESP_CONV1_NT 1
#endif
// zbits != nullptr: the ReLU mask as a packed bit map too, bit c % 32 of word p * D/32 + c / 32 = (z[p][c] > 0)
// (D % 32 == 0): the conv2 input gradient's mask read (esp_conv2_dgrad_bits), 1/32 of the fp32 map's bytes
template <bool B16>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                        const float* __restrict__ bias, float* __restrict__ z,
                                                        uint2* __restrict__ z16, uint32_t* __restrict__ zbits, int B,
                                                        int T, int F, int T1, int F1, int D, unsigned chunk) {
  // block b owns output pixels [b * chunk, (b + 1) * chunk); per step its 256 threads cover PS = 256 / (D/4)
  // consecutive pixels x all D channels (PS KB of contiguous float4 stores).  The pixel's (b, t1, f1) is
  // decomposed once and then advanced by PS (one row wrap per step at most when PS < F1) -- the per-pixel
  // integer divisions of a grid-stride loop were ~half of the kernel's VALU
  const int D4 = D / 4, PS = 256 / D4;
  const int o4 = threadIdx.x % D4, tp = threadIdx.x / D4;
  float w[4][9], bb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bb[q] = bias[o4 * 4 + q];
#pragma unroll
    for (int k = 0; k < 9; ++k) w[q][k] = W[(o4 * 4 + q) * 9 + k];
  }
  const unsigned npix = (unsigned)B * T1 * F1;  // < 2^32 (host check): 32-bit index math
  // c1 in 64 bits: c0 + chunk can pass 2^32 in the last block when npix is near it
  const unsigned c0 = blockIdx.x * chunk, c1 = (unsigned)min((unsigned long)npix, (unsigned long)c0 + chunk);
  unsigned p = c0 + tp;
  if (p >= c1) return;
  const unsigned r0 = p / (unsigned)F1;
  int f1 = (int)(p - r0 * (unsigned)F1);
  int bi = (int)(r0 / (unsigned)T1);
  int t1 = (int)(r0 - (unsigned)bi * T1);
  for (; p < c1; p += PS) {
    const float* xp = x + ((long)bi * T + 2 * t1) * F + 2 * f1;
    float patch[9];
#pragma unroll
    for (int kt = 0; kt < 3; ++kt)
#pragma unroll
      for (int kf = 0; kf < 3; ++kf) patch[kt * 3 + kf] = xp[(long)kt * F + kf];
    float out[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float a = bb[q];
#pragma unroll
      for (int k = 0; k < 9; ++k) a += w[q][k] * patch[k];
      out[q] = fmaxf(a, 0.f);
    }
#if ESP_CONV1_NT  // non-temporal stores of the 7.7 GB map: 2109 -> 1453 us at C2 B=256 (profiles/r05ac_conv1_nt_ab.txt)
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v ov = {out[0], out[1], out[2], out[3]};
    __builtin_nontemporal_store(ov, reinterpret_cast<f4v*>(z + (long)p * D + o4 * 4));
#else
    *reinterpret_cast<float4*>(z + (long)p * D + o4 * 4) = make_float4(out[0], out[1], out[2], out[3]);
#endif
    if constexpr (B16) z16[((long)p * D + o4 * 4) >> 2] = make_uint2(esp::bf16_pair(out[0], out[1]), esp::bf16_pair(out[2], out[3]));
    if (zbits) {  // (uniform) 8 lanes (o4 & ~7 .. +7, one pixel: D4 % 8 == 0) OR their nibbles into one word
      uint32_t v = ((out[0] > 0.f ? 1u : 0u) | (out[1] > 0.f ? 2u : 0u) | (out[2] > 0.f ? 4u : 0u) |
                    (out[3] > 0.f ? 8u : 0u)) << (4 * (o4 & 7));
      // DPP, no LDS round trip: quad_perm [1,0,3,2], [2,3,0,1], then row_half_mirror (lane i <-> 7 - i)
      v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
      v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
      v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
      if ((o4 & 7) == 0) zbits[(long)p * (D >> 5) + (o4 >> 3)] = v;
    }
    f1 += PS;
    while (f1 >= F1) {  // (once at most when PS < F1, the C2 / C5 shapes)
      f1 -= F1;
      if (++t1 == T1) {
        t1 = 0;
        ++bi;
      }
    }
  }
}

// dz1pre[b,t1,f1,c] = (z1>0) * sum over valid taps of dcol[(b,t2,f2)][(kt*3+kf)*D + c]
__global__ void col2im_relu_kernel(const float* __restrict__ dcol, const float* __restrict__ z1, float* __restrict__ dz1,
                                   int B, int T1, int F1, int T2, int F2, int D) {
  const int D4 = D / 4;
  const long n = (long)B * T1 * F1 * D4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c4 = (int)(i % D4);
    long p = i / D4;
    const int f1 = (int)(p % F1);
    p /= F1;
    const int t1 = (int)(p % T1);
    const int b = (int)(p / T1);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int kt = 0; kt < 3; ++kt) {
      const int tt = t1 - kt;
      if (tt < 0 || (tt & 1)) continue;
      const int t2 = tt >> 1;
      if (t2 >= T2) continue;
#pragma unroll
      for (int kf = 0; kf < 3; ++kf) {
        const int ff = f1 - kf;
        if (ff < 0 || (ff & 1)) continue;
        const int f2 = ff >> 1;
        if (f2 >= F2) continue;
        const float4 v = *reinterpret_cast<const float4*>(
            dcol + (((long)b * T2 + t2) * F2 + f2) * (9L * D) + (kt * 3 + kf) * D + c4 * 4);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
    const long o = (((long)b * T1 + t1) * F1 + f1) * D + c4 * 4;
    const float4 zz = *reinterpret_cast<const float4*>(z1 + o);
    acc.x = zz.x > 0.f ? acc.x : 0.f;
    acc.y = zz.y > 0.f ? acc.y : 0.f;
    acc.z = zz.z > 0.f ? acc.z : 0.f;
    acc.w = zz.w > 0.f ? acc.w : 0.f;
    *reinterpret_cast<float4*>(dz1 + o) = acc;
  }
}

// Conv2dSubsampling6's second convolution (Conv2d(D, D, 5, 3), subsampling.py:101-146) on explicit columns:
// generic (k, s) NHWC im2col and its ReLU-masked col2im gather.  Column layout (kt, kf, c): row p =
// (b, t2, f2) holds x[b, s t2 + kt, s f2 + kf, c] at (kt k + kf) C + c -- the (o, kt, kf, c) weight image
// (esp_permute3) makes the convolution one KC x KC GEMM.  float4 over C, one thread per (pixel, tap, c4).
__global__ void im2col_nhwc_kernel(const float* __restrict__ x, float* __restrict__ col, int B, int T1, int F1,
                                   int C, int T2, int F2, int k, int s) {
  const int C4 = C / 4, KK = k * k;
  const long n = (long)B * T2 * F2 * KK * C4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    long q = i / C4;
    const int tap = (int)(q % KK);
    const long p = q / KK;
    const int f2 = (int)(p % F2);
    const long r = p / F2;
    const int t2 = (int)(r % T2);
    const int b = (int)(r / T2);
    const int kt = tap / k, kf = tap - kt * k;
    const float4 v = *reinterpret_cast<const float4*>(
        x + (((long)b * T1 + s * t2 + kt) * F1 + s * f2 + kf) * C + c4 * 4);
    *reinterpret_cast<float4*>(col + p * ((long)KK * C) + (long)tap * C + c4 * 4) = v;
  }
}

// dx[b,t1,f1,c] = (z>0) * sum over the taps (kt, kf) that reach (t1, f1) -- (t1 - kt) % s == 0 and
// (t1 - kt) / s < T2, likewise f -- of dcol[(b,t2,f2)][(kt k + kf) C + c], kt and kf ascending
__global__ void col2im_relu_nhwc_kernel(const float* __restrict__ dcol, const float* __restrict__ z,
                                        float* __restrict__ dx, int B, int T1, int F1, int C, int T2, int F2, int k,
                                        int s) {
  const int C4 = C / 4;
  const long n = (long)B * T1 * F1 * C4;
  const long rowc = (long)k * k * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    long p = i / C4;
    const int f1 = (int)(p % F1);
    p /= F1;
    const int t1 = (int)(p % T1);
    const int b = (int)(p / T1);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int kt = 0; kt < k; ++kt) {
      const int tt = t1 - kt;
      if (tt < 0 || tt % s) continue;
      const int t2 = tt / s;
      if (t2 >= T2) continue;
      for (int kf = 0; kf < k; ++kf) {
        const int ff = f1 - kf;
        if (ff < 0 || ff % s) continue;
        const int f2 = ff / s;
        if (f2 >= F2) continue;
        const float4 v = *reinterpret_cast<const float4*>(
            dcol + (((long)b * T2 + t2) * F2 + f2) * rowc + (long)(kt * k + kf) * C + c4 * 4);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
    const long o = (((long)b * T1 + t1) * F1 + f1) * C + c4 * 4;
    const float4 zz = *reinterpret_cast<const float4*>(z + o);
    acc.x = zz.x > 0.f ? acc.x : 0.f;
    acc.y = zz.y > 0.f ? acc.y : 0.f;
    acc.z = zz.z > 0.f ? acc.z : 0.f;
    acc.w = zz.w > 0.f ? acc.w : 0.f;
    *reinterpret_cast<float4*>(dx + o) = acc;
  }
}

// conv1 weight/bias gradient partials: block = chunk of pixels, thread = channel; the 9-tap
// patches of a sub-chunk are staged in LDS (3 x float4 per pixel, broadcast reads), the dz rows
// are read 4 pixels ahead.  Partials are stored output-major part[(o*10+k)*nb + block] so the
// finalize pass reads each output's partials contiguously.
constexpr int C1_CHUNK = 2048, C1_SUB = 256;
__global__ __launch_bounds__(1024) void conv1_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dz,
                                                          float* __restrict__ part, int B, int T, int F, int T1, int F1,
                                                          int D, int nb) {
  __shared__ float4 patch[C1_SUB][3];
  const long npix = (long)B * T1 * F1;
  const long p0 = (long)blockIdx.x * C1_CHUNK;
  const int o = threadIdx.x;  // blockDim == D rounded up to a wave
  const bool own = o < D;
  float acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = 0.f;
  for (long s0 = p0; s0 < p0 + C1_CHUNK && s0 < npix; s0 += C1_SUB) {
    __syncthreads();
    for (int e = threadIdx.x; e < C1_SUB * 12; e += blockDim.x) {
      const int q = e / 12, k = e - q * 12;
      const long p = s0 + q;
      float v = 0.f;
      if (p < npix && k < 9) {
        const int f1 = (int)(p % F1);
        const long r = p / F1;
        const int t1 = (int)(r % T1);
        const int b = (int)(r / T1);
        v = x[((long)b * T + 2 * t1 + k / 3) * F + 2 * f1 + k % 3];
      }
      reinterpret_cast<float*>(&patch[q][0])[k] = v;
    }
    __syncthreads();
    const int lim = own ? (int)min((long)C1_SUB, npix - s0) : 0;
    const float* dzp = dz + s0 * D + o;
    int q = 0;
    for (; q + 4 <= lim; q += 4) {
      float g[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) g[u] = dzp[(long)(q + u) * D];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 a = patch[q + u][0], bq = patch[q + u][1], c = patch[q + u][2];
        acc[0] += g[u] * a.x; acc[1] += g[u] * a.y; acc[2] += g[u] * a.z; acc[3] += g[u] * a.w;
        acc[4] += g[u] * bq.x; acc[5] += g[u] * bq.y; acc[6] += g[u] * bq.z; acc[7] += g[u] * bq.w;
        acc[8] += g[u] * c.x; acc[9] += g[u];
      }
    }
    for (; q < lim; ++q) {
      const float gg = dzp[(long)q * D];
      const float4 a = patch[q][0], bq = patch[q][1], c = patch[q][2];
      acc[0] += gg * a.x; acc[1] += gg * a.y; acc[2] += gg * a.z; acc[3] += gg * a.w;
      acc[4] += gg * bq.x; acc[5] += gg * bq.y; acc[6] += gg * bq.z; acc[7] += gg * bq.w;
      acc[8] += gg * c.x; acc[9] += gg;
    }
  }
  if (own)
#pragma unroll
    for (int k = 0; k < 10; ++k) part[((long)o * 10 + k) * nb + blockIdx.x] = acc[k];
}

// one block per (o, k) output: fixed-order strided sum + LDS tree (deterministic)
__global__ __launch_bounds__(256) void conv1_wgrad_finalize(const float* __restrict__ part, int nb, int D,
                                                            float* __restrict__ dW, float* __restrict__ db) {
  __shared__ float sh[16];
  const int e = blockIdx.x;
  float s = 0.f;
  for (int p = threadIdx.x; p < nb; p += blockDim.x) s += part[(long)e * nb + p];
  s = esp::block_sum(s, sh);
  if (threadIdx.x == 0) {
    const int o = e / 10, k = e - o * 10;
    if (k < 9) dW[o * 9 + k] += s;
    else db[o] += s;
  }
}

// out[o][a][b] (+)= in[o][b][a], in = (O, Bd, Ad)
__global__ void permute3_kernel(const float* __restrict__ in, float* __restrict__ out, int O, int Bd, int Ad,
                                int accumulate) {
  const long n = (long)O * Bd * Ad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int bb = (int)(i % Bd);
    long r = i / Bd;
    const int a = (int)(r % Ad);
    const int o = (int)(r / Ad);
    const float v = in[((long)o * Bd + bb) * Ad + a];
    out[i] = accumulate ? out[i] + v : v;
  }
}

}  // namespace

static int conv1_fwd_impl(const float* x, const float* W, const float* bias, float* z, void* z16, unsigned* zbits, int B,
                          int T, int F, int D, void* stream);
ESP_API int esp_conv1_fwd(const float* x, const float* W, const float* bias, float* z, int B, int T, int F, int D,
                          void* stream) {
  return conv1_fwd_impl(x, W, bias, z, nullptr, nullptr, B, T, F, D, stream);
}
ESP_API int esp_conv1_fwd_bf16(const float* x, const float* W, const float* bias, float* z, void* z16, int B, int T,
                               int F, int D, void* stream) {
  ESP_ARG_CHECK(z16 && ((uintptr_t)z16 & 7) == 0, "esp_conv1_fwd_bf16: z16 must be 8-B aligned");
  return conv1_fwd_impl(x, W, bias, z, z16, nullptr, B, T, F, D, stream);
}
ESP_API int esp_conv1_fwd_bits(const float* x, const float* W, const float* bias, float* z, void* z16, unsigned* zbits,
                               int B, int T, int F, int D, void* stream) {
  ESP_ARG_CHECK(!z16 || ((uintptr_t)z16 & 7) == 0, "esp_conv1_fwd_bits: z16 must be 8-B aligned");
  ESP_ARG_CHECK(zbits && ((uintptr_t)zbits & 3) == 0 && D % 32 == 0,
                "esp_conv1_fwd_bits: zbits (4-B aligned) and D %% 32 == 0 needed");
  return conv1_fwd_impl(x, W, bias, z, z16, zbits, B, T, F, D, stream);
}
static int conv1_fwd_impl(const float* x, const float* W, const float* bias, float* z, void* z16, unsigned* zbits, int B,
                          int T, int F, int D, void* stream) {
  ESP_ARG_CHECK(D % 4 == 0, "esp_conv1_fwd: D %% 4 != 0");
  const int T1 = (T - 3) / 2 + 1, F1 = (F - 3) / 2 + 1;
  ESP_ARG_CHECK(256 % (D / 4) == 0, "esp_conv1_fwd: D/4 must divide 256");
  const long npix = (long)B * T1 * F1;
  ESP_ARG_CHECK(npix < (1L << 32), "esp_conv1_fwd: %ld output pixels (32-bit index math)", npix);
  const long ps = 256 / (D / 4);
  long nblk = (npix + ps - 1) / ps;
  if (nblk > 8192) nblk = 8192;  // ~16 pixels per thread at the C2 sizes: weights amortised
  const unsigned chunk = (unsigned)((npix + nblk - 1) / nblk);
  if (z16)
    hipLaunchKernelGGL(conv1_fwd_kernel<true>, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, x, W, bias, z,
                       (uint2*)z16, (uint32_t*)zbits, B, T, F, T1, F1, D, chunk);
  else
    hipLaunchKernelGGL(conv1_fwd_kernel<false>, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, x, W, bias, z,
                       nullptr, (uint32_t*)zbits, B, T, F, T1, F1, D, chunk);
  ESP_CHECK_LAUNCH("esp_conv1_fwd");
  return 0;
}

ESP_API int esp_im2col_nhwc(const float* x, float* col, int B, int T1, int F1, int C, int k, int s, void* stream) {
  ESP_ARG_CHECK(C % 4 == 0 && k >= 1 && s >= 1 && T1 >= k && F1 >= k && B >= 0,
                "esp_im2col_nhwc: bad shape B=%d T1=%d F1=%d C=%d k=%d s=%d", B, T1, F1, C, k, s);
  const int T2 = (T1 - k) / s + 1, F2 = (F1 - k) / s + 1;
  const long n = (long)B * T2 * F2 * k * k * (C / 4);
  if (n == 0) return 0;
  hipLaunchKernelGGL(im2col_nhwc_kernel, dim3(gridn(n)), dim3(256), 0, (hipStream_t)stream, x, col, B, T1, F1, C, T2,
                     F2, k, s);
  ESP_CHECK_LAUNCH("esp_im2col_nhwc");
  return 0;
}

ESP_API int esp_col2im_relu_nhwc(const float* dcol, const float* z, float* dx, int B, int T1, int F1, int C, int k,
                                 int s, void* stream) {
  ESP_ARG_CHECK(C % 4 == 0 && k >= 1 && s >= 1 && T1 >= k && F1 >= k && B >= 0,
                "esp_col2im_relu_nhwc: bad shape B=%d T1=%d F1=%d C=%d k=%d s=%d", B, T1, F1, C, k, s);
  const int T2 = (T1 - k) / s + 1, F2 = (F1 - k) / s + 1;
  const long n = (long)B * T1 * F1 * (C / 4);
  if (n == 0) return 0;
  hipLaunchKernelGGL(col2im_relu_nhwc_kernel, dim3(gridn(n)), dim3(256), 0, (hipStream_t)stream, dcol, z, dx, B, T1,
                     F1, C, T2, F2, k, s);
  ESP_CHECK_LAUNCH("esp_col2im_relu_nhwc");
  return 0;
}

ESP_API int esp_col2im_relu(const float* dcol, const float* z1, float* dz1, int B, int T1, int F1, int D, void* stream) {
  ESP_ARG_CHECK(D % 4 == 0, "esp_col2im_relu: D %% 4 != 0");
  const int T2 = (T1 - 3) / 2 + 1, F2 = (F1 - 3) / 2 + 1;
  hipLaunchKernelGGL(col2im_relu_kernel, dim3(gridn((long)B * T1 * F1 * (D / 4))), dim3(256), 0, (hipStream_t)stream,
                     dcol, z1, dz1, B, T1, F1, T2, F2, D);
  ESP_CHECK_LAUNCH("esp_col2im_relu");
  return 0;
}

// workspace: ceil(B*T1*F1/2048) * D * 10 floats (esp_conv1_wgrad_workspace_bytes).  dW (D,9) and
// db (D) accumulated.
ESP_API long esp_conv1_wgrad_workspace_bytes(int B, int T, int F, int D) {
  const int T1 = (T - 3) / 2 + 1, F1 = (F - 3) / 2 + 1;
  if (B <= 0 || T1 <= 0 || F1 <= 0 || D <= 0) return 0;
  return 4L * (((long)B * T1 * F1 + C1_CHUNK - 1) / C1_CHUNK) * D * 10;
}
ESP_API int esp_conv1_wgrad(const float* x, const float* dz1, float* dW, float* db, int B, int T, int F, int D,
                            float* work, long work_bytes, void* stream) {
  const long need__ = esp_conv1_wgrad_workspace_bytes(B, T, F, D);
  ESP_ARG_CHECK(work_bytes >= need__, "esp_conv1_wgrad: workspace %ld B < %ld B required (esp_conv1_wgrad_workspace_bytes)", work_bytes, need__);
  const int T1 = (T - 3) / 2 + 1, F1 = (F - 3) / 2 + 1;
  const long npix = (long)B * T1 * F1;
  const int nb = (int)((npix + C1_CHUNK - 1) / C1_CHUNK);
  hipStream_t st = (hipStream_t)stream;
  ESP_ARG_CHECK(D <= 1024, "esp_conv1_wgrad: D > 1024");
  hipLaunchKernelGGL(conv1_wgrad_kernel, dim3(nb), dim3((D + 63) / 64 * 64), 0, st, x, dz1, work, B, T, F, T1, F1, D, nb);
  hipLaunchKernelGGL(conv1_wgrad_finalize, dim3(D * 10), dim3(256), 0, st, work, nb, D, dW, db);
  ESP_CHECK_LAUNCH("esp_conv1_wgrad");
  return 0;
}

ESP_API int esp_permute3(const float* in, float* out, int O, int Bd, int Ad, int accumulate, void* stream) {
  hipLaunchKernelGGL(permute3_kernel, dim3(gridn((long)O * Bd * Ad)), dim3(256), 0, (hipStream_t)stream, in, out, O, Bd,
                     Ad, accumulate);
  ESP_CHECK_LAUNCH("esp_permute3");
  return 0;
}
