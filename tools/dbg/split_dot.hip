// Probe: the bf16x3 split residuals as v_dot2c_f32_bf16 vs the exact CPU definition (round to nearest
// even parts of the exact residuals).  Prints mismatch counts for the SGPR-constant form.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
#include <random>
typedef __attribute__((ext_vector_type(2))) __bf16 b2;
typedef __attribute__((ext_vector_type(2))) float f2;
__global__ void k(const float* x, uint32_t* o, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a = x[2 * i], b = x[2 * i + 1];
  b2 hp = __builtin_convertvector((f2){a, b}, b2);
  uint32_t na, nb;
  asm("s_mov_b32 %0, 0xbf80" : "=s"(na));
  asm("s_mov_b32 %0, 0xbf800000" : "=s"(nb));
  const b2 NA = __builtin_bit_cast(b2, na), NB = __builtin_bit_cast(b2, nb);
  float ra = __builtin_amdgcn_fdot2_f32_bf16(hp, NA, a, false);
  float rb = __builtin_amdgcn_fdot2_f32_bf16(hp, NB, b, false);
  b2 mp = __builtin_convertvector((f2){ra, rb}, b2);
  float sa = __builtin_amdgcn_fdot2_f32_bf16(mp, NA, ra, false);
  float sb = __builtin_amdgcn_fdot2_f32_bf16(mp, NB, rb, false);
  b2 lp = __builtin_convertvector((f2){sa, sb}, b2);
  o[3 * i] = __builtin_bit_cast(uint32_t, hp);
  o[3 * i + 1] = __builtin_bit_cast(uint32_t, mp);
  o[3 * i + 2] = __builtin_bit_cast(uint32_t, lp);
}
static uint16_t rne(float v) {
  uint32_t u; memcpy(&u, &v, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float up(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); return f; }
int main() {
  const int n = 1 << 20;
  float* hx = new float[2 * n];
  std::mt19937 g(1);
  std::normal_distribution<float> nd;
  std::uniform_int_distribution<int> e(-120, 120);
  for (int i = 0; i < 2 * n; ++i) hx[i] = ldexpf(nd(g), e(g));
  hx[0] = 0.f; hx[1] = -0.f; hx[2] = 1.f + ldexpf(1.f, -23); hx[3] = 3.0e-39f; hx[4] = -1.5e-40f;
  float* dx; uint32_t* dout;
  hipMalloc(&dx, 8L * n); hipMalloc(&dout, 12L * n);
  hipMemcpy(dx, hx, 8L * n, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, dout, n);
  uint32_t* ho = new uint32_t[3 * n];
  hipMemcpy(ho, dout, 12L * n, hipMemcpyDeviceToHost);
  long bad[3] = {0, 0, 0}, badn = 0, denorm = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 2; ++j) {
      float v = hx[2 * i + j];
      uint16_t h = rne(v); float r = v - up(h);
      uint16_t m = rne(r); float s = r - up(m);
      uint16_t l = rne(s);
      uint16_t got[3] = {(uint16_t)(ho[3 * i] >> (16 * j)), (uint16_t)(ho[3 * i + 1] >> (16 * j)),
                         (uint16_t)(ho[3 * i + 2] >> (16 * j))};
      uint16_t want[3] = {h, m, l};
      bool any = false;
      for (int p = 0; p < 3; ++p) if (got[p] != want[p]) { bad[p]++; any = true; }
      if (any) {
        if (std::fpclassify(v) == FP_NORMAL) { if (badn++ < 5) printf("normal mismatch v=%a got %04x %04x %04x want %04x %04x %04x\n", v, got[0], got[1], got[2], h, m, l); }
        else denorm++;
      }
    }
  printf("pairs %d  mismatches hi %ld mid %ld lo %ld  (normal %ld, subnormal/zero %ld)\n", n, bad[0], bad[1], bad[2], badn, denorm);
  return badn != 0;
}
