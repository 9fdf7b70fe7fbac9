// Microbenchmark: can f32-input MFMA (v_mfma_f32_32x32x2_f32) and ordinary fp32 VALU work overlap
// on one SIMD?  Four kernels, one block of 256 threads per CU x 4 (enough to fill every SIMD):
//   mfma    : every wave runs NI iterations of 4 independent 32x32x2 f32 MFMA chains
//   valu    : every wave runs the same number of iterations of 32 dependent-free v_fma_f32
//   mixed   : every wave runs both streams interleaved (same instruction counts as mfma + valu)
//   split   : even waves the MFMA stream, odd waves the VALU stream (2 waves per SIMD)
// If MFMA and VALU share the SIMD's issue/datapath, mixed ~= mfma + valu; if they overlap,
// mixed ~= max(mfma, valu).  Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_valu_overlap.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((ext_vector_type(16))) float f32x16;
constexpr int NI = 2048;

template <bool DO_MFMA, bool DO_VALU, bool SPLIT>
__global__ __launch_bounds__(256) void probe(float* out, float a0, float b0) {
  const int wave = threadIdx.x >> 6;
  bool mf = DO_MFMA, va = DO_VALU;
  if (SPLIT) {
    mf = (wave & 1) == 0;
    va = !mf;
  }
  f32x16 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  float v[32];
#pragma unroll
  for (int e = 0; e < 32; ++e) v[e] = a0 + e;
  float a = a0 + threadIdx.x, b = b0;
  for (int it = 0; it < NI; ++it) {
    if (mf) {
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
    }
    if (va) {
#pragma unroll
      for (int e = 0; e < 32; ++e) v[e] = fmaf(v[e], b, a);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[c][r];
#pragma unroll
  for (int e = 0; e < 32; ++e) s += v[e];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class K>
float timeit(K kern, int blocks, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1.0f, 0.999f);
  hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1.0f, 0.999f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  hipMalloc(&out, sizeof(float) * 256 * cus * 2);
  for (int per_cu = 1; per_cu <= 2; ++per_cu) {
    const int blocks = cus * per_cu;
    const float tm = timeit(probe<true, false, false>, blocks, out);
    const float tv = timeit(probe<false, true, false>, blocks, out);
    const float tx = timeit(probe<true, true, false>, blocks, out);
    const float ts = timeit(probe<false, false, true>, blocks, out);
    // cycles per iteration per wave at 2.4 GHz (the MFMA stream is 4 x 64 = 256 issue cycles)
    const double cyc = 2.4e6 / NI;
    printf("blocks/CU %d (waves/SIMD %d): mfma %.3f ms (%.0f cyc/it)  valu %.3f ms (%.0f)  mixed %.3f ms (%.0f)  "
           "split %.3f ms (%.0f)\n",
           per_cu, per_cu, tm, tm * cyc, tv, tv * cyc, tx, tx * cyc, ts, ts * cyc);
  }
  hipFree(out);
  return 0;
}
