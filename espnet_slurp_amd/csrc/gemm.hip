// FP32 / bf16 MFMA GEMM: host side (launch selection, split-K, tile choice, C-ABI) and the
// register-staged fallback / split-K reduction kernels.  Device code: gemm_kernels.h.
#include <stdlib.h>

#include <algorithm>

#include "gemm_kernels.h"

using namespace espg;

namespace {

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Split-K reduction + the fused epilogue.  Block = 64 float4 slots x 4 split groups: thread
// (slot, grp) sums splits grp, grp+4, ... of its float4 (independent 16-B loads, fixed order),
// the 4 group partials are combined in fixed order through LDS, and each of the 4 threads of a
// slot then finishes one element (deterministic).  The fused row sums (bias gradient) are
// reduced by the first blocks.  Requires N % 4 == 0 (else the scalar kernel below).
constexpr int RED_SLOTS = 64, RED_GROUPS = 4;
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(GemmArgs g) {
  __shared__ float4 part[RED_GROUPS][RED_SLOTS];
  const long MN = (long)g.M * g.N;
  const long split_stride = MN * g.batch;
  if (g.rowsum && g.rs_work) {
    const long m = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (m < g.M) {
      float acc = 0.f;
      int s = 0;
      for (; s + 8 <= g.splits; s += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = g.rs_work[(long)(s + u) * g.M + m];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
      }
      for (; s < g.splits; ++s) acc += g.rs_work[(long)s * g.M + m];
      g.rowsum[m] += acc;
    }
  }
  const int slot = threadIdx.x & (RED_SLOTS - 1), grp = threadIdx.x / RED_SLOTS;
  const long total4 = split_stride >> 2;
  const long e4 = blockIdx.x * (long)RED_SLOTS + slot;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e4 < total4) {
    const float4* w = reinterpret_cast<const float4*>(g.work) + e4;
    const long st4 = split_stride >> 2;
    int s = grp;
    for (; s + 3 * RED_GROUPS < g.splits; s += 4 * RED_GROUPS) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = w[(long)(s + u * RED_GROUPS) * st4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
    for (; s < g.splits; s += RED_GROUPS) {
      const float4 v = w[(long)s * st4];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  part[grp][slot] = acc;
  __syncthreads();
  if (e4 >= total4) return;
  float r = 0.f;
#pragma unroll
  for (int q = 0; q < RED_GROUPS; ++q) {
    const float4 v = part[q][slot];
    r += grp == 0 ? v.x : grp == 1 ? v.y : grp == 2 ? v.z : v.w;
  }
  const long e = (e4 << 2) + grp;
  const int z = (int)(e / MN);
  const long rr = e - (long)z * MN;
  const int m = (int)(rr / g.N), n = (int)(rr - (long)m * g.N);
  reduce_store(g, z, m, n, r);
}

// scalar fallback (N % 4 != 0)
__global__ void splitk_reduce_kernel(GemmArgs g) {
  if (g.rowsum && g.rs_work) {
    for (long m = blockIdx.x * (long)blockDim.x + threadIdx.x; m < g.M; m += (long)gridDim.x * blockDim.x) {
      float acc = 0.f;
      for (int s = 0; s < g.splits; ++s) acc += g.rs_work[(long)s * g.M + m];
      g.rowsum[m] += acc;
    }
  }
  const long MN = (long)g.M * g.N;
  const long split_stride = MN * g.batch;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < split_stride; e += (long)gridDim.x * blockDim.x) {
    const int z = (int)(e / MN);
    const long r = e - (long)z * MN;
    const int m = (int)(r / g.N), n = (int)(r - (long)m * g.N);
    float acc = 0.f;
    for (int s = 0; s < g.splits; ++s) acc += g.work[s * split_stride + e];
    reduce_store(g, z, m, n, acc);
  }
}

// rowsum[r] += sum_k A(r,k) for an RC-mode A (element (r,k) at p[k*ld + r]) — used only when
// the LDS-DMA kernel (which fuses it) is not eligible; fixed k order per row
__global__ void rowsum_rc_kernel(const float* __restrict__ p, long ld, int M, int K, float* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= M) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += p[(long)k * ld + r];
  out[r] += s;
}

// resident blocks of the persistent LDS-DMA kernel: per_cu per CU (64 KB LDS each)
long g_cus = -1;
long persist_blocks(int per_cu) {
  if (g_cus < 0) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    g_cus = cus;
  }
  return (long)per_cu * g_cus;
}

int g_compute = 0;  // 0: fp32 MFMA (exact f32 fma chain), 1: bf16-input MFMA with fp32 accumulate
int g_last_grid = 0;  // the grid of the last LDS-DMA launch (EPI_C1FOLD: its per-block records)

// split-K combine: 0 the reduction launch (default), 1 in-kernel (last-arriving unit per tile;
// measured slower, kept for esp_set_splitk_mode and its parity test)
int g_splitk = 0;
int splitk_mode() { return g_splitk; }

// smallest K a split-K split keeps on grids of >= 64 tiles (128 before round 4's end)
constexpr long kSplitkMinK = 256;
long splitk_mink() { return kSplitkMinK; }

// work units split-K aims for: two resident blocks on each of 256 CUs (256 / 384 / 768 measured within
// +-0.5 %, profiles/r03i_abc_splitk_target.txt)
constexpr long kSplitkTarget = 2 * 256;
// most splits of one GEMM: 128, so the 4-tile d x d weight gradients (256 x 256 over K = B*T') reach
// the two resident blocks per CU (64 left them at one: 99 TF/s, profiles/r04l_gemm_shapes_trace_b128.txt)
constexpr long kMaxSplits = 128;
#ifndef ESP_GEMM_TILE_TIE
#define ESP_GEMM_TILE_TIE 0.95
#endif

// Launch the LDS-DMA kernel with the epilogue kind compiled in (each kind is its own kernel,
// so the plain GEMMs carry none of the fused epilogues' registers; the instantiations live in
// the gemm_glds_*.hip units).  Returns false when the mode pair has no instantiation of the
// needed kind (the caller falls back to the register-staged kernel).
bool launch_glds(int MA, int MB, const GemmArgs& g, int batch, hipStream_t st, const GldsArgs* tconv = nullptr) {
  const int BNT = g.bnt;
  const bool can_rs = MA == RC;
  const bool can_fwd = (MA == KC && (MB == KC || MB == RC)) || (MA == I2C_KC && MB == KC);
  const bool can_bwd = (MA == KC || MA == I2CT_KC) && MB == RC;
  const bool can_spec_fwd = MA == KC && MB == KC, can_spec_bwd = MA == KC && MB == RC;
  const bool can_brelu = (MA == KC || MA == I2C_KC) && MB == KC;
  const bool can_pspec = (MA == KC || MA == RC) && (MB == KC || MB == RC);
  // implicit-im2col A: every slab lies inside one tap (kt, kf), so the LDS-DMA source offset is
  // one scalar per slab; other channel counts take the register-staged kernel
  if (MA == I2C_KC && (g.a.ic.C % GL_BK || g.K % GL_BK)) return false;
  // StageS: the pixel offsets of a 128-pixel run (<= 2 maps) as 32-bit byte offsets
  if (MA == I2C_KC && 8L * g.a.ic.H * g.a.ic.W * g.a.ic.C >= (1L << 32)) return false;
  // implicit-im2col B: pixel offsets on 24-bit multiplies (i2c_pix_off24)
  if (MB == I2C_RC) {
    const long kpix = g.bf16 == 2 ? 2L * g.K : (long)g.K;  // (bf16: K counts pixel pairs)
    const long rows = kpix / ((long)g.b.ic.Ho * g.b.ic.Wo) * g.b.ic.H * g.b.ic.W;  // Bn * H * W
    if (rows >= (1L << 24) || rows * g.b.ic.C >= (1L << 32)) return false;
  }
  int kind = g.splits > 1 ? EPI_PLAIN : epi_kind_spec(g);
  if (g.cpn) {  // planes output: only its specialised kinds, no fallback kind
    if (kind < 0 || !g.wide) return false;
    if (kind == EPI_P0_PL && !(MA == KC && MB == RC)) return false;
    if ((kind == EPI_FFN_SWISH_PL || kind == EPI_FFN_RELU_PL) && !(MA == KC && MB == KC)) return false;
    if ((kind == EPI_BMUL_PL || kind == EPI_RMASK_PL) && !(MA == KC && MB == RC)) return false;
  }
  if (kind == EPI_SMB && !(MA == KC && MB == KC && g.bf16 == 0)) return false;
  if (!g.cpn && (((kind == EPI_BMUL || kind == EPI_RMASK) && !can_spec_bwd) || ((kind == EPI_P0 || kind == EPI_PR) && !can_pspec) ||
      (kind == EPI_RMASKMAP && !(MA == I2CT_KC && MB == RC)) ||
      (kind == EPI_BRELU && !can_brelu) ||
      (kind >= EPI_BIAS && kind <= EPI_FFN_RELU && !can_spec_fwd)))
    kind = epi_kind(g);
  if ((kind == EPI_FWD && !can_fwd) || (kind == EPI_BWD && !can_bwd)) return false;
  GldsArgs x{};
  if (MA == I2CT_KC) x = *tconv;  // the transposed-conv gather parameters
  x.ntx = (g.N + BNT - 1) / BNT;
  const int bm = g.bm == 64 || g.bm == 256 ? g.bm : BM;
  x.nty = (g.M + bm - 1) / bm;
  if (MA == I2C_KC) {
    x.c_a = make_fastdiv(g.a.ic.C);
    x.hw_a = make_fastdiv(g.a.ic.Ho * g.a.ic.Wo);
    x.wo_a = make_fastdiv(g.a.ic.Wo);
  }
  if (MB == I2C_RC) {
    x.c_b = make_fastdiv(g.b.ic.C);
    x.hw_b = make_fastdiv(g.b.ic.Ho * g.b.ic.Wo);
    x.wo_b = make_fastdiv(g.b.ic.Wo);
  }
  x.ntiles = (int)((long)x.ntx * x.nty * batch * g.splits);
  const bool rs = can_rs && g.rowsum;
  if (rs) kind = EPI_PLAIN;
  if (kind == EPI_C1FOLD && !(MA == I2CT_KC && MB == RC && BNT == 128 && bm == 128 && x.ntx <= C1NT)) return false;
  const dim3 grid((unsigned)std::min<long>(x.ntiles, persist_blocks(glds_occupancy_rt(BNT, kind, bm, g.bf16))));
  g_last_grid = (int)grid.x;
  x.fd_grid = make_fastdiv(grid.x);
  x.fd_ntx = make_fastdiv((uint32_t)x.ntx);
  x.fd_nty = make_fastdiv((uint32_t)x.nty);
  x.fd_splits = make_fastdiv((uint32_t)g.splits);
  x.fd_nb2 = make_fastdiv((uint32_t)g.nb2);
  const int prec = g.bf16;
  if (kind == EPI_PLAIN) return glds_launch_plain(MA, MB, BNT, prec, rs, grid, st, g, x);
  if (kind == EPI_FWD || kind == EPI_BWD) return glds_launch_epi(MA, MB, BNT, prec, kind, grid, st, g, x);
  if (kind == EPI_P0 || kind == EPI_PR || kind == EPI_SMB || kind == EPI_P0_PL)
    return glds_launch_pspec(MA, MB, BNT, prec, kind, grid, st, g, x);
  return glds_launch_spec(MA, MB, BNT, prec, kind, grid, st, g, x);
}

template <int MA, int MB>
int launch(const GemmArgs& g0, int batch, hipStream_t st, const Operand* b_fp32 = nullptr,
           const Operand* a_fp32 = nullptr) {
  bool done = false;
  if (g0.bnt == 64 || g0.bnt == 128) done = launch_glds(MA, MB, g0, batch, st);
  GemmArgs g = g0;
  if (!done && g.bf16 == 5) {  // no planes x planes kernel for this epilogue kind: the fp32 A operand
    if (!a_fp32 || !a_fp32->p) {
      esp::set_error("esp_gemm_f32_pl: no planes kernel for this launch and no fp32 A to fall back to");
      return -1;
    }
    g.a = *a_fp32;
    g.bf16 = 3;
    if (g.bnt == 64 || g.bnt == 128) done = launch_glds(MA, MB, g, batch, st);
  }
  if (!done && g.bf16 == 3) {  // no B-planes kernel for this epilogue kind: the fp32 B operand
    if (!b_fp32 || !b_fp32->p) {
      esp::set_error("esp_gemm_f32_bp: no B-planes kernel for this launch and no fp32 B to fall back to");
      return -1;
    }
    g.b = *b_fp32;
    g.bf16 = 0;
    if (g.bnt == 64 || g.bnt == 128) done = launch_glds(MA, MB, g, batch, st);
  }
  if (!done && g.cpn) {
    esp::set_error("esp_gemm_f32_pl: no kernel writes this epilogue as planes (planes output: plain, the ReLU mask, or the FFN "
                   "bias + activation + dropout + derivative; N %% 4 == 0, 16-B aligned, LDS-DMA operands)");
    return -1;
  }
  if (!done && g.smb_rel) {
    esp::set_error("esp_attn_dscores: operands not eligible for the LDS-DMA kernel (16-B alignment, ld %% 4)");
    return -1;
  }
  if (!done && g.bf16 == 2) {
    esp::set_error("esp_gemm_bf16: operands not eligible for the LDS-DMA kernel (16-B alignment, ld %% 8)");
    return -1;
  }
  if (!done) {
    g.rs_work = nullptr;
    g.tickets = nullptr;  // the register-staged kernel: [split][z][M][N] partials + the reduction launch
    if (g.rowsum && MA == RC)  // the register-staged kernel does not fuse the row sums
      hipLaunchKernelGGL(rowsum_rc_kernel, dim3((g.M + 255) / 256), dim3(256), 0, st, g.a.p, g.a.ld, g.M, g.K,
                         g.rowsum);
    dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, batch * g.splits);
    if (g.bf16) hipLaunchKernelGGL((gemm_bf16_kernel<MA, MB>), grid, dim3(NT), 0, st, g);
    else hipLaunchKernelGGL((gemm_f32_kernel<MA, MB, 1>), grid, dim3(NT), 0, st, g);
  }
  if (g.splits > 1 && !g.tickets) {
    const long total = (long)g.M * g.N * batch;
    if ((g.N & 3) == 0 && aligned16(g.work)) {
      long nb = (total / 4 + RED_SLOTS - 1) / RED_SLOTS;
      if (g.rowsum && g.rs_work && nb < (g.M + 255) / 256) nb = (g.M + 255) / 256;
      hipLaunchKernelGGL(splitk_reduce4_kernel, dim3((unsigned)nb), dim3(256), 0, st, g);
    } else {
      const long nb = (total + 255) / 256;
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)(nb > 16384 ? 16384 : nb)), dim3(256), 0, st, g);
    }
  }
  ESP_CHECK_LAUNCH("gemm_f32");
  return 0;
}


// LDS-DMA staging reads whole 16-B quads along the contiguous dim `cont` (K for KC, the row
// count for RC) at clamped indices: legal when quads are aligned and the row pitch covers the
// rounded-up run (or there is a single line whose run is a multiple of 4).
bool glds_ok(int mode, const void* p, long ld, long s1, long s2, int rows, int K) {
  if (!aligned16(p) || s1 % 4 || s2 % 4) return false;
  if (mode >= 2) return true;  // im2col: C % 4 == 0 checked by the caller
  const long cont = mode == 0 ? K : rows, lines = mode == 0 ? rows : K;
  if (lines == 1) return cont % 4 == 0;
  // StageS per-lane byte offsets are 32-bit: 128 rows (KC) / 32 k-rows (RC) of pitch ld
  if (ld > (mode == 0 ? 8000000L : 32000000L)) return false;
  return ld % 4 == 0 && ld >= cont;
}

}  // namespace

// C-ABI: see include/espnet_mi355.h for the contract.
ESP_API int esp_set_gemm_compute(int dtype) {
  ESP_ARG_CHECK(dtype == 0 || dtype == 1, "esp_set_gemm_compute: dtype must be 0 (fp32) or 1 (bf16), got %d", dtype);
  const int prev = g_compute;
  g_compute = dtype;
  return prev;
}
ESP_API int esp_get_gemm_compute(void) { return g_compute; }
ESP_API int esp_f32_gemm_products(void) { return ESP_F32_SPLIT ? 6 : 1; }
ESP_API int esp_set_splitk_mode(int mode) {
  ESP_ARG_CHECK(mode == 0 || mode == 1, "esp_set_splitk_mode: mode must be 0 or 1, got %d", mode);
  const int prev = splitk_mode();
  g_splitk = mode;
  return prev;
}

static int gemm_run(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2, const float* A, long lda,
                    long sa1, long sa2, const float* B, long ldb, long sb1, long sb2, float* C, long ldc, long sc1,
                    long sc2, const float* bias, float alpha, float beta, const float* R, int act, float* aux,
                    float drop_p, unsigned long long seed, int bwd_act, const float* pre, float* rowsum,
                    const int* im2col_a, const int* im2col_b, float* work, long work_bytes, void* stream,
                    int prec_in, const GemmArgs* smb = nullptr, const void* b_planes = nullptr, long ldbp = 0,
                    long sbp1 = 0, long sbp2 = 0, long bps = 0, const void* a_planes = nullptr, long ldap = 0,
                    long sap1 = 0, long sap2 = 0, long aps = 0, int cpn = 0, long cps = 0, const int* band = nullptr);

ESP_API int esp_gemm_f32(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2,
                         const float* A, long lda, long sa1, long sa2,
                         const float* B, long ldb, long sb1, long sb2,
                         float* C, long ldc, long sc1, long sc2,
                         const float* bias, float alpha, float beta, const float* R,
                         int act, float* aux, float drop_p, unsigned long long seed,
                         int bwd_act, const float* pre, float* rowsum,
                         const int* im2col_a, const int* im2col_b, float* work, long work_bytes,
                         void* stream) {
  return gemm_run(mode_a, mode_b, M, N, K, batch, nb2, A, lda, sa1, sa2, B, ldb, sb1, sb2, C, ldc, sc1, sc2, bias,
                  alpha, beta, R, act, aux, drop_p, seed, bwd_act, pre, rowsum, im2col_a, im2col_b, work, work_bytes,
                  stream, -1);
}

ESP_API int esp_gemm_f32_bp(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2, const float* A, long lda,
                            long sa1, long sa2, const float* B, long ldb, long sb1, long sb2, float* C, long ldc,
                            long sc1, long sc2, const float* bias, float alpha, float beta, const float* R, int act,
                            float* aux, float drop_p, unsigned long long seed, int bwd_act, const float* pre,
                            float* rowsum, const int* im2col_a, float* work, long work_bytes, const void* b_planes,
                            long ldbp, long sbp1, long sbp2, long b_pstride, void* stream) {
  ESP_ARG_CHECK(mode_b == KC || mode_b == RC, "esp_gemm_f32_bp: mode_b must be 0 (KC) or 1 (RC)");
  ESP_ARG_CHECK(b_planes || B, "esp_gemm_f32_bp: B planes and B both NULL");
  return gemm_run(mode_a, mode_b, M, N, K, batch, nb2, A, lda, sa1, sa2, B, ldb, sb1, sb2, C, ldc, sc1, sc2, bias,
                  alpha, beta, R, act, aux, drop_p, seed, bwd_act, pre, rowsum, im2col_a, nullptr, work, work_bytes,
                  stream, -1, nullptr, b_planes, ldbp, sbp1, sbp2, b_pstride);
}

// esp_gemm_f32 with either operand (or both) also given as its three bf16 split planes
ESP_API int esp_gemm_f32_pl(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2, const float* A, long lda,
                            long sa1, long sa2, const void* a_planes, long ldap, long sap1, long sap2, long a_pstride,
                            const float* B, long ldb, long sb1, long sb2, const void* b_planes, long ldbp, long sbp1,
                            long sbp2, long b_pstride, float* C, long ldc, long sc1, long sc2, const float* bias,
                            float alpha, float beta, const float* R, int act, float* aux, float drop_p,
                            unsigned long long seed, int bwd_act, const float* pre, float* rowsum, int c_nplanes,
                            long c_pstride, float* work, long work_bytes, void* stream) {
  ESP_ARG_CHECK(mode_a == KC || mode_a == RC, "esp_gemm_f32_pl: mode_a must be 0 (KC) or 1 (RC)");
  ESP_ARG_CHECK(mode_b == KC || mode_b == RC, "esp_gemm_f32_pl: mode_b must be 0 (KC) or 1 (RC)");
  ESP_ARG_CHECK((A || a_planes) && (B || b_planes), "esp_gemm_f32_pl: an operand has neither fp32 values nor planes");
  return gemm_run(mode_a, mode_b, M, N, K, batch, nb2, A, lda, sa1, sa2, B, ldb, sb1, sb2, C, ldc, sc1, sc2, bias,
                  alpha, beta, R, act, aux, drop_p, seed, bwd_act, pre, rowsum, nullptr, nullptr, work, work_bytes,
                  stream, -1, nullptr, b_planes, ldbp, sbp1, sbp2, b_pstride, a_planes, ldap, sap1, sap2, a_pstride,
                  c_nplanes, c_pstride);
}

namespace {
// the three bf16 planes of an fp32 matrix, split3_bf16's split (so a B-planes GEMM multiplies the
// values the in-register split would): 8 columns per thread, one 16-B store per plane; columns
// cols..ldy-1 written 0
__global__ void f32_to_planes_kernel(const float* __restrict__ x, uint4* __restrict__ y, long rows, int cols, long ldx,
                                     long ldy, long ps, int vec) {
  const long c8 = ldy >> 3;
  const long n = rows * c8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / c8;
    const int c = (int)(i - r * c8) * 8;
    const float* src = x + r * ldx + c;
    float v[8];
    if (vec && c + 8 <= cols) {
      const float4 a = *reinterpret_cast<const float4*>(src);
      const float4 b = *reinterpret_cast<const float4*>(src + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = c + e < cols ? src[e] : 0.f;
    }
    bf16x8 hi, mid, lo;
    split3_bf16(v, hi, mid, lo);
    const long o = (r * ldy + c) >> 3, po = ps >> 3;
    y[o] = __builtin_bit_cast(uint4, hi);
    y[o + po] = __builtin_bit_cast(uint4, mid);
    y[o + 2 * po] = __builtin_bit_cast(uint4, lo);
  }
}
}  // namespace

ESP_API int esp_f32_to_planes(const float* x, void* y, long rows, int cols, long ldx, long ldy, long pstride,
                              void* stream) {
  ESP_ARG_CHECK(rows >= 0 && cols >= 0 && ldx >= cols && ldy >= cols && ldy % 8 == 0 && pstride % 8 == 0 &&
                    pstride >= rows * ldy && aligned16(y),
                "esp_f32_to_planes: bad sizes rows=%ld cols=%d ldx=%ld ldy=%ld pstride=%ld (ldy, pstride %% 8, y 16-B aligned)",
                rows, cols, ldx, ldy, pstride);
  if (rows == 0 || ldy == 0) return 0;
  const long n = rows * (ldy >> 3);
  const int vec = aligned16(x) && ldx % 4 == 0;
  hipLaunchKernelGGL(f32_to_planes_kernel, dim3((unsigned)std::min<long>((n + 255) / 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, x, (uint4*)y, rows, cols, ldx, ldy, pstride, vec);
  ESP_CHECK_LAUNCH("esp_f32_to_planes");
  return 0;
}

ESP_API int esp_gemm_bf16(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2, const void* A, long lda,
                          long sa1, long sa2, const void* B, long ldb, long sb1, long sb2, float* C, long ldc,
                          long sc1, long sc2, const float* bias, float alpha, float beta, const float* R, int act,
                          float* aux, float drop_p, unsigned long long seed, int bwd_act, const float* pre,
                          float* rowsum, float* work, long work_bytes, void* stream) {
  ESP_ARG_CHECK((mode_a == KC || mode_a == RC) && (mode_b == KC || mode_b == RC),
                "esp_gemm_bf16: modes must be 0 (KC) or 1 (RC)");
  ESP_ARG_CHECK(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && sa1 % 8 == 0 && sa2 % 8 == 0 && sb1 % 8 == 0 &&
                    sb2 % 8 == 0 && aligned16(A) && aligned16(B),
                "esp_gemm_bf16: K, ld and strides must be multiples of 8 bf16 and A, B 16-B aligned");
  ESP_ARG_CHECK((mode_a == KC || M % 8 == 0) && (mode_b == KC || N % 8 == 0),
                "esp_gemm_bf16: an RC operand's row count must be a multiple of 8 (M=%d N=%d)", M, N);
  // bf16 pairs viewed as fp32 elements by the staging code (PREC 2): K, ld and strides in pairs
  return gemm_run(mode_a, mode_b, M, N, K / 2, batch, nb2, (const float*)A, lda / 2, sa1 / 2, sa2 / 2,
                  (const float*)B, ldb / 2, sb1 / 2, sb2 / 2, C, ldc, sc1, sc2, bias, alpha, beta, R, act, aux, drop_p,
                  seed, bwd_act, pre, rowsum, nullptr, nullptr, work, work_bytes, stream, 2);
}

// The conv2 forward of the bf16 mode (subsampling.py:53-87 in NHWC): z2 = ReLU(im2col(z1) W^T + b)
// with z1 and the (o, kt, kf, c)-laid weights in bf16 (z1_16 from esp_conv1_fwd_bf16, w16 row pitch
// 9D), fp32 accumulate and output: the implicit-im2col GEMM on bf16 operands (PREC 2, the gather in
// bf16-pair units).  D % 64 == 0.
ESP_API int esp_conv2_fwd_bf16(const void* z1_16, const void* w16, const float* bias, float* z2, int B, int T1, int F1,
                               int D, float* work, long work_bytes, void* stream) {
  ESP_ARG_CHECK(B >= 1 && T1 >= 3 && F1 >= 3 && D % 64 == 0 && aligned16(z1_16) && aligned16(w16) && aligned16(z2),
                "esp_conv2_fwd_bf16: bad sizes / alignment (D %% 64 == 0, 16-B aligned operands)");
  const int T2 = (T1 - 3) / 2 + 1, F2 = (F1 - 3) / 2 + 1;
  const int ic[5] = {T1, F1, D / 2, T2, F2};  // channel pairs
  return gemm_run(I2C_KC, KC, B * T2 * F2, D, 9 * D / 2, 1, 1, (const float*)z1_16, 0, 0, 0, (const float*)w16,
                  9 * D / 2, 0, 0, z2, D, 0, 0, bias, 1.f, 0.f, nullptr, ACT_RELU, nullptr, 0.f, 0, 0, nullptr, nullptr,
                  ic, nullptr, work, work_bytes, stream, 2);
}

// The bf16 mode's conv2 weight gradient: dW2r (D x 9D, (o, kt, kf, c)) = dz2^T im2col(z1) and the bias
// gradient db += sum over pixels of dz2, on bf16 operands (dz2_16 [pixels][D], z1_16 from
// esp_conv1_fwd_bf16): RC x gathered-RC GEMM on bf16 pairs (PREC 2), K = pixels / 2 pairs (an even pixel
// count), split K with the fixed-order reduction.  D % 64 == 0.
ESP_API int esp_conv2_wgrad_bf16(const void* dz2_16, const void* z1_16, float* dw, float* db, int B, int T1, int F1,
                                 int D, float* work, long work_bytes, void* stream) {
  const int T2 = (T1 - 3) / 2 + 1, F2 = (F1 - 3) / 2 + 1;
  const long npix = (long)B * T2 * F2;
  ESP_ARG_CHECK(B >= 1 && T1 >= 3 && F1 >= 3 && D % 64 == 0 && npix % 2 == 0 && aligned16(dz2_16) &&
                    aligned16(z1_16) && aligned16(dw),
                "esp_conv2_wgrad_bf16: bad sizes / alignment (D %% 64 == 0, an even pixel count, 16-B aligned)");
  const int ic[5] = {T1, F1, D, T2, F2};  // bf16 channels (the gather's offsets are halved in the kernel)
  return gemm_run(RC, I2C_RC, D, 9 * D, (int)(npix / 2), 1, 1, (const float*)dz2_16, D / 2, 0, 0,
                  (const float*)z1_16, 0, 0, 0, dw, 9 * D, 0, 0, nullptr, 1.f, 0.f, nullptr, 0, nullptr, 0.f, 0, 0,
                  nullptr, db, nullptr, ic, work, work_bytes, stream, 2);
}

ESP_API int esp_gemm_bf16_pl(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2, const void* A, long lda,
                             long sa1, long sa2, const void* B, long ldb, long sb1, long sb2, void* C, long ldc,
                             long sc1, long sc2, const float* bias, float alpha, float beta, int act, float* aux,
                             float drop_p, unsigned long long seed, int bwd_act, const float* pre, int c_nplanes,
                             long c_pstride, float* work, long work_bytes, void* stream) {
  ESP_ARG_CHECK((mode_a == KC || mode_a == RC) && (mode_b == KC || mode_b == RC),
                "esp_gemm_bf16_pl: modes must be 0 (KC) or 1 (RC)");
  ESP_ARG_CHECK(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && sa1 % 8 == 0 && sa2 % 8 == 0 && sb1 % 8 == 0 &&
                    sb2 % 8 == 0 && aligned16(A) && aligned16(B),
                "esp_gemm_bf16_pl: K, ld and strides must be multiples of 8 bf16 and A, B 16-B aligned");
  ESP_ARG_CHECK((mode_a == KC || M % 8 == 0) && (mode_b == KC || N % 8 == 0),
                "esp_gemm_bf16_pl: an RC operand's row count must be a multiple of 8 (M=%d N=%d)", M, N);
  ESP_ARG_CHECK(c_nplanes == 1, "esp_gemm_bf16_pl: c_nplanes must be 1 (bf16 operands: a bf16 result)");
  return gemm_run(mode_a, mode_b, M, N, K / 2, batch, nb2, (const float*)A, lda / 2, sa1 / 2, sa2 / 2,
                  (const float*)B, ldb / 2, sb1 / 2, sb2 / 2, (float*)C, ldc, sc1, sc2, bias, alpha, beta, nullptr, act,
                  aux, drop_p, seed, bwd_act, pre, nullptr, nullptr, nullptr, work, work_bytes, stream, 2, nullptr,
                  nullptr, 0, 0, 0, 0, nullptr, 0, 0, 0, 0, c_nplanes, c_pstride);
}

// Rel-pos attention score gradient in one GEMM: dP = dctx V^T per (head, utterance) with the
// softmax + attention-dropout + rel_shift adjoints in the epilogue (EPI_SMB):
//   dS[i][j] = P[i][j] * (drop'(dP[i][j]) - dot[i]) / sqrt(d_k),  dot[i] = dctx_i . ctx_i
// (= sum_j P_drop[i][j] dP[i][j]: FlashAttention-2's row term, esp_attn_bwd_prep), and dS scattered
// into the bd gradient rows (latest / legacy rel_shift adjoint; esp_attn_bwd_prep zeroes the
// elements without a source).  Replaces the dP GEMM + the row-wise softmax / rel_shift pass
// (attention.py:64-96, 145-165 backward): no dP tensor round trip through HBM.
ESP_API int esp_attn_dscores(const float* dctx, long ldd, const float* vmat, long ldv, const float* attn,
                             const float* dot, float* dS, float* dbd, long ldp, int relpos, int nb, int H, int dk,
                             float sqrt_dk, float drop_p, unsigned long long seed, int T, long lds, void* stream) {
  ESP_ARG_CHECK(relpos == 1 || relpos == 2, "esp_attn_dscores: relpos must be 1 or 2");
  ESP_ARG_CHECK(T >= 1 && nb >= 1 && H >= 1 && dk >= 1 && lds >= T && lds % 4 == 0 &&
                    ldp >= (relpos == 1 ? 2 * T - 1 : T) && sqrt_dk > 0.f,
                "esp_attn_dscores: bad sizes T=%d lds=%ld ldp=%ld", T, lds, ldp);
  ESP_ARG_CHECK(((uintptr_t)attn & 15) == 0 && ((uintptr_t)dS & 15) == 0, "esp_attn_dscores: attn / dS not 16-B aligned");
  GemmArgs smb{};
  smb.smb_rel = relpos;
  smb.smb_dot = dot;
  smb.smb_dbd = dbd;
  smb.smb_ldp = ldp;
  const int Z = nb * H;
  return gemm_run(KC, KC, T, T, dk, Z, nb, dctx, ldd, dk, (long)T * ldd, vmat, ldv, dk, (long)T * ldv, dS, lds,
                  (long)nb * T * lds, (long)T * lds, nullptr, 1.0f / sqrt_dk, 0.f, nullptr, 0, nullptr, drop_p, seed, 0,
                  attn, nullptr, nullptr, nullptr, nullptr, 0, stream, 0, &smb);
}

static int gemm_run(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2, const float* A, long lda,
                    long sa1, long sa2, const float* B, long ldb, long sb1, long sb2, float* C, long ldc, long sc1,
                    long sc2, const float* bias, float alpha, float beta, const float* R, int act, float* aux,
                    float drop_p, unsigned long long seed, int bwd_act, const float* pre, float* rowsum,
                    const int* im2col_a, const int* im2col_b, float* work, long work_bytes, void* stream,
                    int prec_in, const GemmArgs* smb, const void* b_planes, long ldbp, long sbp1, long sbp2,
                    long bps, const void* a_planes, long ldap, long sap1, long sap2, long aps, int cpn, long cps,
                    const int* band) {
  ESP_ARG_CHECK(M >= 0 && N >= 0 && K >= 0 && batch >= 1 && nb2 >= 1 && batch % nb2 == 0,
                "esp_gemm_f32: bad sizes M=%d N=%d K=%d batch=%d nb2=%d", M, N, K, batch, nb2);
  ESP_ARG_CHECK(mode_a >= 0 && mode_a <= 3 && mode_b >= 0 && mode_b <= 3, "esp_gemm_f32: bad mode");
  ESP_ARG_CHECK(drop_p >= 0.f && drop_p < 1.f, "esp_gemm_f32: bad dropout p");
  ESP_ARG_CHECK(!bwd_act || (pre && !aux && act == 0), "esp_gemm_f32: bwd_act needs pre and no forward activation");
  ESP_ARG_CHECK(bwd_act >= 0 && bwd_act <= ACT_MUL && (act & ~(3 | ACT_AUX_DERIV)) == 0 && (act & 3) <= ACT_SWISH,
                "esp_gemm_f32: bad act / bwd_act code");
  ESP_ARG_CHECK(!(act & ACT_AUX_DERIV) || aux, "esp_gemm_f32: ACT_AUX_DERIV needs aux");
  ESP_ARG_CHECK(!rowsum || (mode_a == 1 && batch == 1), "esp_gemm_f32: rowsum needs an RC-mode A and batch 1");
  if (M == 0 || N == 0) return 0;
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K; g.nb2 = nb2;
  g.a = Operand{A, lda, sa1, sa2, 0, {}};
  g.b = Operand{B, ldb, sb1, sb2, 0, {}};
  g.a.vec = aligned16(A) && lda % 4 == 0 && sa1 % 4 == 0 && sa2 % 4 == 0;
  g.b.vec = aligned16(B) && ldb % 4 == 0 && sb1 % 4 == 0 && sb2 % 4 == 0;
  // (PREC 2: an RC operand's contiguous run is rows / 2 pairs)
  g.a.glds = glds_ok(mode_a, A, lda, sa1, sa2, prec_in == 2 && mode_a == RC ? M / 2 : M, K);
  g.b.glds = glds_ok(mode_b, B, ldb, sb1, sb2, prec_in == 2 && mode_b == RC ? N / 2 : N, K);
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
  g.bwd_act = bwd_act; g.pre = pre; g.rowsum = rowsum;
  g.seed = seed;
  g.key = esp::rng_key_ptr();
  if (smb) {  // esp_attn_dscores: the softmax / rel_shift adjoint epilogue
    g.smb_rel = smb->smb_rel;
    g.smb_dot = smb->smb_dot;
    g.smb_dbd = smb->smb_dbd;
    g.smb_ldp = smb->smb_ldp;
  }
  g.cpn = cpn;
  g.cps = cps;
  if (band) {
    g.band_c0 = band[0];
    g.band_w = band[1];
  }
  if (cpn) {  // planes output: 8-B quads per plane (C is plane 0, bf16)
    ESP_ARG_CHECK((cpn == 1 || cpn == 3) && N % 4 == 0 && ldc % 4 == 0 && cps % 4 == 0 && ((uintptr_t)C & 7) == 0 &&
                      !R && !rowsum && (cpn == 1 || cps >= (long)M * ldc || batch > 1),
                  "esp_gemm_f32_pl: planes output needs N %% 4 == 0, ldc / pstride %% 4 == 0, no residual / row sums");
    work = nullptr;  // never split-K: the epilogue writes the planes once
  }
  g.wide = N % 4 == 0 && ldc % 4 == 0 && ldc < (1L << 24) && sc1 % 4 == 0 && sc2 % 4 == 0 && (cpn ? true : aligned16(C)) && (!R || aligned16(R)) &&
           (!aux || aligned16(aux)) && (!pre || aligned16(pre)) && (!bias || aligned16(bias)) &&
           (!work || aligned16(work));
  g.ragged4 = !g.wide && N % 4 != 0 && ldc % 4 == 0 && sc1 % 4 == 0 && sc2 % 4 == 0 && aligned16(C) &&
              (!R || aligned16(R)) && !aux && !pre && !bias;
  g.drop_scale = 1.f;  // (the specialised dropout epilogues run unconditionally: p = 0 keeps every element at scale 1)
  if (drop_p > 0.f) {
    g.drop_thresh = esp::drop_threshold(drop_p);
    g.drop_scale = esp::drop_scale(g.drop_thresh);
  }
  // Tile choice: the LDS-DMA kernel when both operands allow it, 128x64 tiles when N <= 64
  // or when 128x128 tiles leave the grid under two blocks per CU but 128x64 tiles do not
  // (e.g. N = 256 over 23936 rows: 374 -> 748 tiles, no split-K reduction pass needed).
  // Then split-K when the grid still cannot fill the 256 CUs (weight gradients: small
  // M x N, huge K).
  g.batch = batch;
  g.splits = 1;
  g.kchunk = K;
  const long target = kSplitkTarget;
  auto ntiles = [&](int bn, int bm = BM) { return (long)((N + bn - 1) / bn) * ((M + bm - 1) / bm) * batch; };
  g.bnt = 0;
  g.bm = BM;
  g.bf16 = prec_in >= 0 ? prec_in : (g_compute == 1 ? 1 : 0);
  // B as three bf16 planes (esp_gemm_f32_bp): the fp32 split-product GEMM without B's split in the
  // k-loop, when the fp32 compute type runs on split products and the planes suit the LDS-DMA
  // kernel (else the fp32 B operand)
  // A as planes too (esp_gemm_f32_pl, PREC 5): no split in the k-loop at all (64-wide tiles: the
  // two operands' planes fill 72 KB of LDS per block)
  const Operand b_fp32 = g.b, a_fp32 = g.a;
  auto planes_ok = [&](const void* pl, long ld, long s1, long s2, long ps, int mode, int rows) {
    return pl && aligned16(pl) && ld % 8 == 0 && s1 % 8 == 0 && s2 % 8 == 0 && ps % 8 == 0 &&
           (mode == KC ? (K % 8 == 0 && ld >= K && 128L * ld * 2 < (1L << 32))
                       : (rows % 8 == 0 && ld >= rows && 32L * ld * 2 + 2L * rows < (1L << 32)));
  };
  const bool split_ok = prec_in < 0 && g.bf16 == 0 && ESP_F32_SPLIT && K > 0;
  if (split_ok && mode_b <= RC && planes_ok(b_planes, ldbp, sbp1, sbp2, bps, mode_b, N) &&
      (((mode_a == KC || mode_a == I2C_KC) && mode_b == KC) || ((mode_a == KC || mode_a == RC) && mode_b == RC) ||
       (a_planes && mode_a <= RC))) {
    if (mode_a <= RC && planes_ok(a_planes, ldap, sap1, sap2, aps, mode_a, M)) {
      g.a = Operand{(const float*)a_planes, ldap, sap1, sap2, 1, {}, 1};
      g.a.ps = aps;
      g.bf16 = 5;
    } else if (g.a.glds) {
      g.bf16 = 3;
    }
    if (g.bf16 >= 3) {
      g.b = Operand{(const float*)b_planes, ldbp, sbp1, sbp2, 1, {}, 1};
      g.b.ps = bps;
    }
  }
  if (!g.b.p || !g.a.p) {
    esp::set_error("esp_gemm_f32_pl: operand planes not eligible (alignment, ld / strides %% 8, K / M / N %% 8) "
                   "and the fp32 operand is NULL");
    return -1;
  }
  const bool bplanes = g.bf16 >= 3;
  if (g.a.glds && g.b.glds && K > 0) {
    // per-CU time model: ceil(tiles / CUs) tiles of bn/64 units each, x1.3 when the grid
    // leaves CUs with a single resident block (one wave per SIMD); ties keep 128 (intensity)
    // fp32 on split products (ESP_F32_SPLIT): a 64-wide tile costs ~3/4 of a 128-wide one (its
    // waves split 1.5x the operand values per MFMA), and a grid that split-K will refill is
    // priced by its total work (the K ~ 48k weight gradients: 3.8 vs 4.9 ms on 128-wide tiles)
    // (B planes, PREC 3, are the same split-product arithmetic: a weight gradient on X planes is priced
    // like its PREC 0 form -- priced per tile instead, its split-K grid took 64-wide tiles, 12.6 ms for what
    // 128-wide tiles do in ~11, profiles/r05j_*)
    const bool split_f32 = ESP_F32_SPLIT && (g.bf16 == 0 || g.bf16 == 3);
    auto cost = [&](int bn) {
      const long t = ntiles(bn);
      // (B planes: only A is split, 3.7 split VALU per MFMA at either width)
      const double per = split_f32 && !bplanes && bn == 64 ? 1.5 : bn / 64;
      // (bf16 operands, PREC 2: a weight gradient's split-K grid is priced by its total work too -- the
      // 128-wide tiles halve its B re-reads, which bound the bf16 k-loop: C5 (1,1,2048,512,23936)
      // 2.50 -> 2.03 ms, (1,1,512,2048,23936) 2.34 -> 1.79, r04 ESP_GEMM_BNT=128 A/B)
      if ((split_f32 || (g.bf16 == 2 && mode_a == RC && mode_b == RC)) && work && t < target && K >= 2 * (t >= 64 ? splitk_mink() : 128))
        return (double)t * per / 256.0;
      double c = (double)((t + 255) / 256) * per;
      if (t < 2 * 256) c *= 1.3;
      return c;
    };
    // a 64-wide tile must win by 5 %: near-ties go to 128-wide tiles (half the A re-reads, half the tile
    // count): the FFN w_1 forward 441 -> 420 us, its input gradient 9.4 -> 8.0 ms per C2 B=256 step, bench
    // +0.8 % (profiles/r05g_gemm_tile_tie_ab.txt); ESP_GEMM_TILE_TIE=1.0 builds the strict comparison
    g.bnt = (N <= 64 || g.bf16 == 5 || cost(64) < ESP_GEMM_TILE_TIE * cost(128)) ? 64 : 128;
    // the conv2 forward (implicit-im2col A gathered from the conv1 map, K = 9 D): 128-wide tiles halve the
    // gathered-A re-reads -- 13.79 -> 11.97 ms per C2 B=256 step (the cost model's near-tie picked 64;
    // profiles/r05f_conv2_fwd_width_ab.txt)
    if (mode_a == I2C_KC && N % 128 == 0) g.bnt = 128;
    // 64 x 64 tiles for grids that 128-row tiles leave under-filled (decoder M ~ 5k tokens, the
    // 41-query source attention): one work unit per tile, x1.15 for the halved operand reuse
    if (g.bnt == 64 && mode_a <= RC && mode_b <= RC && g.bf16 != 2 && !smb) {
      const long t = ntiles(64, 64);
      double c = (double)((t + 255) / 256) * 1.15;
      if (t < 2 * 256) c *= 1.3;
      if (c < cost(64)) g.bm = 64;
    }
    // the conv2 weight gradient (im2col-gathered B, K = B*T2*F2 ~ 1M): 128-wide tiles halve the
    // gathered-B re-reads and split-K refills the chip (8.39 vs 9.22 ms at C2 B=128,
    // tools/gemm_bench.py with ESP_GEMM_BNT; the K ~ 48k linear weight gradients keep 128x64)
    if (mode_b == I2C_RC && work && K >= 65536) g.bnt = 128;

    // (256 x 128 bf16 tiles -- one block, one wave per SIMD, per CU -- measured slower, C5 B=64 860.3 vs
    // 889.3 utt/s, and were removed in round 5)
#if ESP_GEMM_WIDE_KCRC
    // the KC x RC GEMMs on B planes (linear input gradients, P0 / FFN w_2 shapes): 256 x 128 tiles of 8 waves
    // on a 2-slab ring, 3-7 % faster per kernel at C2 B=256 (the other pairs measured slower, r05am)
    if (g.bnt == 128 && g.bm == BM && g.bf16 == 3 && mode_a == KC && mode_b == RC && !smb && M >= 256 &&
        256L * g.a.ld * 4 < (1L << 32))
      g.bm = 256;
#endif
  }
  {
    const long tiles = ntiles(g.bnt ? g.bnt : BN, g.bm);
    // each split keeps >= splitk_mink() of K on grids of >= 64 tiles: the reduction launch (~8-10 us)
    // outweighs halving a K = 256 k-loop (the decoder's M = 5248 shapes: 24.8 -> 17.5 and 12.6 us,
    // profiles/r04j_ vs r04l_gemm_shapes_trace_b128.txt); a grid of a few tiles (the d x d weight
    // gradients over K = 747 / 5248 rows: 8 tiles) needs the splits to fill the chip (19.7 -> 31 us
    // and 21 -> 26 us with 256), so it keeps 128
    const long mink = tiles >= 64 ? splitk_mink() : 128;
    if (work && tiles < target && K >= 2 * mink) {
      long sp = (target + tiles - 1) / tiles;
      const long by_k = K / mink;
      if (sp > by_k) sp = by_k;
      // in-kernel combine (LDS-DMA kernel): partials on whole tiles + tickets in the last 64 KB
      const int bmt = g.bm == 64 || g.bm == 256 ? g.bm : BM;
      const long mp = (long)(M + bmt - 1) / bmt * bmt, np = g.bnt ? (long)(N + g.bnt - 1) / g.bnt * g.bnt : N;
      // opt-in (ESP_SPLITK_INKERNEL=1): measured slower at C2 B=128 -- the last-arriving unit of a
      // tile sums all of its splits alone (64 splits x 32 KB behind 8 tiles for the d x d weight
      // gradients: 222 vs 68 us), where the separate reduction spreads them over the chip
      const bool inkernel = splitk_mode() == 1 && g.bnt && !bplanes && g.bm != 256 && tiles <= ESP_GEMM_TICKETS &&
                            work_bytes > ESP_GEMM_TICKET_BYTES;
      const long part = inkernel ? mp * np : (long)M * N;
      const long cap = (work_bytes - (inkernel ? ESP_GEMM_TICKET_BYTES : 0)) / (4L * (part * batch + (rowsum ? M : 0)));
      if (sp > cap) sp = cap;
      if (sp > kMaxSplits) sp = kMaxSplits;
      // CU balance: with ceil(tiles*sp / 256) tile-rounds on the busiest CU, 72 tiles x 8 splits
      // (conv2 weight gradient) leave a third of the chip idle in the last round; take the
      // smallest sp up to 4x the target-derived one whose last round is >= 95 % full.
      if (sp >= 2) {
        // score the split count that is actually launched: the chunk is rounded up to BK, so
        // ceil(K / chunk) can be smaller than the candidate
        auto launched = [&](long s) {
          const long chunk = ((K + s - 1) / s + BK - 1) / BK * BK;
          return (K + chunk - 1) / chunk;
        };
        auto imb = [&](long s) { const long t = tiles * s; return (double)((t + 255) / 256 * 256) / (double)t; };
        const long hi = std::min(std::min(by_k, cap), std::min<long>(kMaxSplits, 4 * sp));
        long best = launched(sp);
        for (long s = sp; s <= hi; ++s) {
          const long e = launched(s);
          if (imb(e) < imb(best) - 1e-9) best = e;
          if (imb(best) <= 1.05) break;
        }
        sp = best;
      }
      if (sp >= 2) {
        int chunk = (int)((K + sp - 1) / sp);
        chunk = (chunk + BK - 1) / BK * BK;
        g.splits = (int)((K + chunk - 1) / chunk);
        g.kchunk = chunk;
        g.work = work;
        if (rowsum && g.bnt) g.rs_work = work + (long)g.splits * batch * part;
        if (inkernel) {
          g.tickets = reinterpret_cast<int*>(reinterpret_cast<char*>(work) + work_bytes - ESP_GEMM_TICKET_BYTES);
          g.sk_mp = (int)mp;
          g.sk_np = (int)np;
        }
      }
    }
  }
  hipStream_t st = (hipStream_t)stream;
  const int key = mode_a * 4 + mode_b;
  switch (key) {
    case KC * 4 + KC: return launch<KC, KC>(g, batch, st, &b_fp32, &a_fp32);
    case KC * 4 + RC: return launch<KC, RC>(g, batch, st, &b_fp32, &a_fp32);
    case RC * 4 + KC: return launch<RC, KC>(g, batch, st, &b_fp32, &a_fp32);
    case RC * 4 + RC: return launch<RC, RC>(g, batch, st, &b_fp32, &a_fp32);
    case I2C_KC * 4 + KC: return launch<I2C_KC, KC>(g, batch, st, &b_fp32);
    case RC * 4 + I2C_RC: return launch<RC, I2C_RC>(g, batch, st);
    default:
      esp::set_error("esp_gemm_f32: unsupported mode pair %d,%d", mode_a, mode_b);
      return -1;
  }
}


// Rel-pos attention (latest rel_shift), the q_v gradient through the band scores:
//   dq_v[z](i, :) = sum_k dbd[z](i, k) p[k, 64 h : 64 h + 64],  z = h * nb + b
// (attention.py:240-263 backward; the dbd.p contraction of RelPositionMultiHeadedAttention.bwd).  Row i of
// dbd is zero outside its rel_shift band, columns T-1-i .. 2T-2-i (esp_attn_softmax_bwd_relpos_band / the
// full-row kernel), so each 128-row tile's k-loop runs over its rows' band union only: T + 127 of the
// 2T - 1 columns.  dbd (Z, T) rows of pitch ldp (>= 2T-1, % 4 == 0); p (2T-1, H*64) pitch ldpm; out rows
// (b*T + i) pitch ldo, head h at column 64 h.  d_k = 64.
ESP_API int esp_relpos_dqv(const float* dbd, long ldp, const float* p, long ldpm, float* out, long ldo, int nb, int H,
                           int T, float* work, long work_bytes, void* stream) {
  ESP_ARG_CHECK(T >= 1 && nb >= 1 && H >= 1 && ldp >= 2 * T - 1 && ldp % 4 == 0 && ldpm >= 64L * H && ldo >= 64L * H,
                "esp_relpos_dqv: bad sizes T=%d ldp=%ld ldpm=%ld ldo=%ld", T, ldp, ldpm, ldo);
  const int band[2] = {T - 1, T};
  const int P = 2 * T - 1;
  return gemm_run(KC, RC, T, 64, P, nb * H, nb, dbd, ldp, (long)nb * T * ldp, (long)T * ldp, p, ldpm, 64, 0, out, ldo,
                  64, (long)T * ldo, nullptr, 1.f, 0.f, nullptr, 0, nullptr, 0.f, 0, 0, nullptr, nullptr, nullptr,
                  nullptr, work, work_bytes, stream, -1, nullptr, nullptr, 0, 0, 0, 0, nullptr, 0, 0, 0, 0, 0, 0, band);
}

// ============================================================================ conv2 input gradient
// Conv2d(D, D, 3, stride 2) input gradient as 4 implicit GEMMs, one per parity class (ph, pw)
// of the conv1 output grid (the sub-pixel decomposition of a strided transposed convolution):
//   dz1[b, 2a+ph, 2e+pw, c] = relu'(z1) * sum_{taps (kt,kf) of the class, o} dz2[b, a-dt, e-df, o] W[o,c,kt,kf]
// with kt in {0,2} (ph = 0) or {1} (ph = 1), dt = (kt-ph)/2 (same for f).  A = the dz2 gather
// (I2CT_KC: LDS-DMA from dz2, lanes outside the T2 x F2 grid read a zero page), B = the class's
// taps of W re-laid [(t*D + o)][c], epilogue = the conv1 ReLU mask (EPI_BWD, act' from z1) with
// the output row map to the class's pixels.  Replaces the (B*T2*F2, 9D) column GEMM + col2im:
// no 9x column buffer.  (subsampling.py:53-87 backward)
namespace {
__global__ void conv2_class_weights_kernel(const float* __restrict__ W, float* __restrict__ Wc, int D) {
  // global tap slots: class (0,0) taps 0-3, (0,1) 4-5, (1,0) 6-7, (1,1) 8
  const long n = 9L * D * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % D);
    const long r = i / D;
    const int o = (int)(r % D);
    const int slot = (int)(r / D);
    int kt, kf;
    if (slot < 4) { kt = 2 * (slot >> 1); kf = 2 * (slot & 1); }
    else if (slot < 6) { kt = 2 * (slot - 4); kf = 1; }
    else if (slot < 8) { kt = 1; kf = 2 * (slot - 6); }
    else { kt = 1; kf = 1; }
    Wc[i] = W[(((long)o * D + c) * 3 + kt) * 3 + kf];
  }
}
// EPI_C1FOLD records -> conv1 weight / bias gradient, in fixed order (deterministic).  c1fold_reduce: block
// (combo = tn * 4 + wave, chunk) sums element e (0..639: lane * 10 + slot) of its chunk of the records (the
// class launches' blocks in order) -> red[combo][chunk][640]
constexpr int C1_NCH = 32;
struct C1Regions {
  long off[4];  // record region of class launch i (floats)
  int grid[4];  // its grid
  int ncls;
};
__global__ __launch_bounds__(640) void c1fold_reduce_kernel(const float* __restrict__ part, C1Regions r,
                                                            float* __restrict__ red) {
  const int combo = blockIdx.x, chunk = blockIdx.y, e = threadIdx.x;
  const int tn = combo >> 2, wave = combo & 3;
  int total = 0;
  for (int i = 0; i < r.ncls; ++i) total += r.grid[i];
  const int r0 = (int)((long)total * chunk / C1_NCH), r1 = (int)((long)total * (chunk + 1) / C1_NCH);
  float acc = 0.f;
  int cls = 0, base = 0;
  for (int rec = r0; rec < r1; ++rec) {
    while (rec - base >= r.grid[cls]) base += r.grid[cls++];
    const long b = rec - base;
    acc += part[r.off[cls] + ((b * C1NT + tn) * 4 + wave) * 640 + e];
  }
  red[((long)combo * C1_NCH + chunk) * 640 + e] = acc;
}
// c1fold_finalize: output (c, k): column c = 128 tn + 64 wn + 32 j + 4 grp + col, sum v = 10 col + k held by lane
// (h, l32) = (s >> 2, 4 grp + (s & 3)), s = v / 5, slot 5 j + v % 5 of waves wn and 2 + wn (store_c1fold)
__global__ void c1fold_finalize_kernel(const float* __restrict__ red, int D, float* __restrict__ dW,
                                       float* __restrict__ db) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= D * 10) return;
  const int c = o / 10, k = o - c * 10;
  const int tn = c >> 7, cc = c & 127, wn = cc >> 6, j = (cc >> 5) & 1, grp = (cc & 31) >> 2, col = cc & 3;
  const int v = col * 10 + k, sl = v / 5, u = v - 5 * sl;
  const int lane = (sl >> 2) * 32 + grp * 4 + (sl & 3), slot = 5 * j + u;
  float acc = 0.f;
  for (int wm = 0; wm < 2; ++wm) {
    const int combo = tn * 4 + wm * 2 + wn;
    for (int ch = 0; ch < C1_NCH; ++ch) acc += red[((long)combo * C1_NCH + ch) * 640 + lane * 10 + slot];
  }
  if (k < 9) dW[c * 9 + k] += acc;
  else db[c] += acc;
}
}  // namespace

// wc_work: the four parity classes' re-laid weights, 9 * D * D floats, then their three bf16 split
// planes (the B-planes class GEMMs of the fp32 split build), 3 * 9 * D * D bf16
// (esp_conv2_dgrad_workspace_bytes)
ESP_API long esp_conv2_dgrad_workspace_bytes(int D) { return D <= 0 ? 0 : 4L * 9 * D * D + 6L * 9 * D * D; }
struct C1FoldArgs {  // esp_conv2_dgrad_c1fold: the conv1 weight gradient folded into the class GEMMs
  const float* x;
  int T, F;
  float *dW, *db, *work;
  long work_bytes;
};
static int conv2_dgrad_impl(const float* dz2, const void* dz2_16, const float* W, const float* z1,
                            const unsigned* z1bits, float* dz1, int B, int T1, int F1, int D, const float* zeros16,
                            float* wc_work, long work_bytes, void* stream, const C1FoldArgs* c1 = nullptr);
ESP_API int esp_conv2_dgrad(const float* dz2, const float* W, const float* z1, float* dz1, int B, int T1, int F1,
                            int D, const float* zeros16, float* wc_work, long work_bytes, void* stream) {
  return conv2_dgrad_impl(dz2, nullptr, W, z1, nullptr, dz1, B, T1, F1, D, zeros16, wc_work, work_bytes, stream);
}
// the conv1 ReLU mask from esp_conv1_fwd_bits' packed bit map (D/32 words per pixel) instead of the fp32 map:
// the epilogue reads 1/32 of the bytes; dz2 fp32 (dz2) or bf16 (dz2_16, the bf16 mode, D % 64 == 0), one of them
ESP_API int esp_conv2_dgrad_bits(const float* dz2, const void* dz2_16, const float* W, const unsigned* z1bits,
                                 float* dz1, int B, int T1, int F1, int D, const float* zeros16, float* wc_work,
                                 long work_bytes, void* stream) {
  ESP_ARG_CHECK(z1bits && ((uintptr_t)z1bits & 3) == 0 && (dz2 == nullptr) != (dz2_16 == nullptr) &&
                    (!dz2_16 || D % 64 == 0),
                "esp_conv2_dgrad_bits: z1bits (4-B aligned) and exactly one of dz2 / dz2_16 (D %% 64 == 0) needed");
  return conv2_dgrad_impl(dz2, dz2_16, W, nullptr, z1bits, dz1, B, T1, F1, D, zeros16, wc_work, work_bytes, stream);
}
// the bf16 mode's form: dz2 as bf16 (dz2_16), the class weights cast to bf16 in the workspace, the class
// GEMMs on bf16 operands (PREC 2, the tap gather in bf16-pair units); D % 64 == 0
ESP_API int esp_conv2_dgrad_bf16(const void* dz2_16, const float* W, const float* z1, float* dz1, int B, int T1,
                                 int F1, int D, const float* zeros16, float* wc_work, long work_bytes, void* stream) {
  ESP_ARG_CHECK(D % 64 == 0, "esp_conv2_dgrad_bf16: D %% 64 == 0 needed");
  return conv2_dgrad_impl(nullptr, dz2_16, W, z1, nullptr, dz1, B, T1, F1, D, zeros16, wc_work, work_bytes, stream);
}
// the records of the four class launches (<= C1NT column tiles of 128, <= 4 resident blocks per CU) + the
// reduction's chunk sums (esp_conv2_dgrad_c1fold)
ESP_API long esp_conv2_c1fold_workspace_bytes(void) {
  return 4L * (4L * persist_blocks(4) * C1NT * 256 * 10 + (long)C1NT * 4 * C1_NCH * 640);
}
// esp_conv2_dgrad_bits with conv1's weight / bias gradient folded into the class GEMMs' epilogue (EPI_C1FOLD):
// dW (D x 9) += sum over the conv1 map of dz1 * x-patch, db (D) += sum dz1, and dz1 itself is never written
// (no 7.7 GB store at C2 B=256, no esp_conv1_wgrad pass over it).  x: the conv1 input (B, T, F), as esp_conv1_fwd
// took it.  D % 128 == 0, D <= 512.
ESP_API int esp_conv2_dgrad_c1fold(const float* dz2, const void* dz2_16, const float* W, const unsigned* z1bits,
                                   const float* x, int T, int F, float* dW, float* db, int B, int T1, int F1, int D,
                                   const float* zeros16, float* wc_work, long work_bytes, float* c1_work,
                                   long c1_work_bytes, void* stream) {
  ESP_ARG_CHECK(z1bits && ((uintptr_t)z1bits & 3) == 0 && (dz2 == nullptr) != (dz2_16 == nullptr) &&
                    (!dz2_16 || D % 64 == 0) && D % 128 == 0 && D <= 128 * C1NT && x && dW && db && c1_work,
                "esp_conv2_dgrad_c1fold: z1bits, x, dW, db, c1_work, exactly one of dz2 / dz2_16, D %% 128 == 0 and "
                "D <= 512 needed");
  ESP_ARG_CHECK(T1 == (T - 3) / 2 + 1 && F1 == (F - 3) / 2 + 1, "esp_conv2_dgrad_c1fold: T1 / F1 do not match T / F");
  const long need = esp_conv2_c1fold_workspace_bytes();
  ESP_ARG_CHECK(c1_work_bytes >= need, "esp_conv2_dgrad_c1fold: c1 workspace %ld B < %ld B", c1_work_bytes, need);
  const C1FoldArgs c1{x, T, F, dW, db, c1_work, c1_work_bytes};
  return conv2_dgrad_impl(dz2, dz2_16, W, nullptr, z1bits, nullptr, B, T1, F1, D, zeros16, wc_work, work_bytes, stream,
                          &c1);
}
static int conv2_dgrad_impl(const float* dz2, const void* dz2_16, const float* W, const float* z1,
                            const unsigned* z1bits, float* dz1, int B, int T1, int F1, int D, const float* zeros16,
                            float* wc_work, long work_bytes, void* stream, const C1FoldArgs* c1) {
  const bool b16 = dz2_16 != nullptr;
  if (b16) dz2 = (const float*)dz2_16;  // bf16 pairs viewed as fp32 elements
  const int T2 = (T1 - 3) / 2 + 1, F2 = (F1 - 3) / 2 + 1;
  const long need__ = esp_conv2_dgrad_workspace_bytes(D);
  ESP_ARG_CHECK(work_bytes >= need__, "esp_conv2_dgrad: workspace %ld B < %ld B required (esp_conv2_dgrad_workspace_bytes)", work_bytes, need__);
  ESP_ARG_CHECK(B >= 1 && T2 >= 1 && F2 >= 1 && D % 32 == 0, "esp_conv2_dgrad: bad sizes (D %% 32 == 0 needed)");
  ESP_ARG_CHECK(aligned16(dz2) && (z1bits || aligned16(z1)) && (c1 || aligned16(dz1)) && aligned16(zeros16) &&
                    aligned16(wc_work),
                "esp_conv2_dgrad: operands must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(conv2_class_weights_kernel, dim3(1024), dim3(256), 0, st, W, wc_work, D);
  ESP_CHECK_LAUNCH("esp_conv2_dgrad (weights)");
  // fp32 compute on split products: the class weights as B planes (PREC 3, no B split in the k-loop);
  // the bf16 form: their bf16 copy (plane 0 of the same conversion: hi = RNE)
  const bool bp = !b16 && g_compute == 0 && ESP_F32_SPLIT;
  const long ps = 9L * D * D;
  __bf16* planes = reinterpret_cast<__bf16*>(wc_work + ps);
  if (b16) {
    hipLaunchKernelGGL(f32_to_planes_kernel, dim3((unsigned)std::min<long>((ps / 8 + 255) / 256, 8192)), dim3(256), 0,
                       st, wc_work, (uint4*)planes, 9L * D, D, (long)D, (long)D, ps, 1);
    ESP_CHECK_LAUNCH("esp_conv2_dgrad (bf16 weights)");
  }
  if (bp) {
    hipLaunchKernelGGL(f32_to_planes_kernel, dim3((unsigned)std::min<long>((ps / 8 + 255) / 256, 8192)), dim3(256), 0,
                       st, wc_work, (uint4*)planes, 9L * D, D, (long)D, (long)D, ps, 1);
    ESP_CHECK_LAUNCH("esp_conv2_dgrad (planes)");
  }
  const int slot0[4] = {0, 4, 6, 8};
  C1Regions c1r{};
  long c1off = 0;
  for (int cls = 0; cls < 4; ++cls) {
    const int ph = cls >> 1, pw = cls & 1;
    const int Ha = (T1 - ph + 1) / 2, We = (F1 - pw + 1) / 2;
    const int nkt = ph ? 1 : 2, nkf = pw ? 1 : 2, ntap = nkt * nkf;
    GldsArgs t{};
    t.t_hw = make_fastdiv((uint32_t)(Ha * We));
    t.t_w = make_fastdiv((uint32_t)We);
    t.t_T2 = T2; t.t_F2 = F2; t.t_C = b16 ? D / 2 : D;  // (bf16: channel pairs)
    for (int ti = 0; ti < ntap; ++ti) {
      const int kt = ph ? 1 : 2 * (ti / nkf), kf = pw ? 1 : 2 * (ti % nkf);
      t.t_dt[ti] = (kt - ph) / 2;
      t.t_df[ti] = (kf - pw) / 2;
    }
    t.t_zeros = zeros16;
    GemmArgs g{};
    g.M = B * Ha * We; g.N = D; g.K = b16 ? ntap * D / 2 : ntap * D; g.nb2 = 1;
    g.a = Operand{dz2, 0, 0, 0, 1, {}, 1};
    g.b = Operand{wc_work + (long)slot0[cls] * D * D, D, 0, 0, 1, {}, 1};
    g.c = dz1; g.ldc = D; g.alpha = 1.f; g.beta = 0.f;
    g.bwd_act = ACT_RELU; g.pre = z1bits ? zeros16 : z1;  // (bits: pre is never read; any aligned pointer)
    g.cm_bits = reinterpret_cast<const uint32_t*>(z1bits); g.cm_bw = D / 32;
    if (c1) {  // no C: the conv1 gradient records of this class launch
      g.c = wc_work;  // (never written by EPI_C1FOLD)
      g.c1_x = c1->x; g.c1_T = c1->T; g.c1_F = c1->F;
      g.c1_part = c1->work + c1off;
    }
    g.bf16 = g_compute;  // bf16 MFMA in the reduced-precision mode, as every other GEMM of the step
    if (bp) {
      g.b = Operand{reinterpret_cast<const float*>(planes + (long)slot0[cls] * D * D), D, 0, 0, 1, {}, 1};
      g.b.ps = ps;
      g.bf16 = 3;
    }
    if (b16) {  // RC bf16: rows = D, ld in pairs
      g.b = Operand{reinterpret_cast<const float*>(planes + (long)slot0[cls] * D * D), D / 2, 0, 0, 1, {}, 1};
      g.bf16 = 2;
    }
    g.key = esp::rng_key_ptr();
    g.wide = 1;
    // 128-wide tiles (64-wide measured 6.95 -> 8.69 ms per step, profiles/r04g_gemm_shapes_b128_gs_dg64.txt)
    g.batch = 1; g.splits = 1; g.kchunk = g.K; g.bnt = D % 128 == 0 ? 128 : 64; g.bm = BM;
    g.cmap = 1;
    g.cm_hw = t.t_hw; g.cm_w = t.t_w;
    g.cm_T1 = T1; g.cm_F1 = F1; g.cm_ph = ph; g.cm_pw = pw;
    if (!launch_glds(I2CT_KC, RC, g, 1, st, &t)) {
      esp::set_error("esp_conv2_dgrad: no kernel for the class GEMM");
      return -1;
    }
    ESP_CHECK_LAUNCH("esp_conv2_dgrad");
    if (c1) {
      c1r.off[cls] = c1off;
      c1r.grid[cls] = g_last_grid;
      c1off += (long)g_last_grid * C1NT * 256 * 10;
    }
  }
  if (c1) {
    c1r.ncls = 4;
    float* red = c1->work + 4L * persist_blocks(4) * C1NT * 256 * 10;
    hipLaunchKernelGGL(c1fold_reduce_kernel, dim3((D / 128) * 4, C1_NCH), dim3(640), 0, st, c1->work, c1r, red);
    hipLaunchKernelGGL(c1fold_finalize_kernel, dim3((D * 10 + 255) / 256), dim3(256), 0, st, red, D, c1->dW, c1->db);
    ESP_CHECK_LAUNCH("esp_conv2_dgrad_c1fold (reduce)");
  }
  return 0;
}
