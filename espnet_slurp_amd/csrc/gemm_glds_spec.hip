// Instantiations of gemm_glds_kernel with the specialised (compile-time feature set) epilogues
// of the production call sites: EPI_BIAS / EPI_BDR / EPI_FFN_SWISH / EPI_FFN_RELU for the linear
// forward (KC x KC), EPI_BRELU (bias + ReLU) for the conv2 forward (implicit-im2col I2C_KC x KC)
// and KC x KC, EPI_BMUL for the FFN input gradient and EPI_RMASK for the gradient through conv2's
// ReLU (KC x RC) and its row-mapped form for the implicit conv2 input gradient (I2CT_KC x RC); the
// FFN w_1 kinds with the hidden state written as bf16 planes (EPI_FFN_*_PL), the FFN and ReLU-mask input
// gradients as planes (EPI_BMUL_PL, EPI_RMASK_PL); EPI_C1FOLD (the implicit conv2 input gradient with the conv1
// weight gradient folded in, 128 x 128 tiles).
// See store_spec.
#include "gemm_kernels.h"

namespace espg {

bool glds_launch_spec(int ma, int mb, int bnt, int prec, int epi, dim3 grid, hipStream_t st, const GemmArgs& g,
                      const GldsArgs& x) {
  bool ok = false;
  const bool known = glds_switch(ma, mb, bnt, prec, g.bm, [&](auto A, auto B, auto N, auto F, auto R) {
    constexpr int MA = decltype(A)::value, MB = decltype(B)::value, BNT = decltype(N)::value;
    constexpr int BF = decltype(F)::value, BMT = decltype(R)::value;
#define ESP_SPEC(K)                                                                                   \
  if (epi == K) {                                                                                     \
    hipLaunchKernelGGL((gemm_glds_kernel<MA, MB, BNT, false, K, BF, BMT>), grid, dim3(glds_threads(BMT)), 0, st, g, x); \
    ok = true;                                                                                        \
  }
    if constexpr (MA == KC && MB == KC) {
      ESP_SPEC(EPI_BIAS)
      ESP_SPEC(EPI_BDR)
      ESP_SPEC(EPI_FFN_SWISH)
      ESP_SPEC(EPI_FFN_RELU)
      ESP_SPEC(EPI_BRELU)
      ESP_SPEC(EPI_FFN_SWISH_PL)
      ESP_SPEC(EPI_FFN_RELU_PL)
    } else if constexpr (MA == I2C_KC && MB == KC) {
      ESP_SPEC(EPI_BRELU)
    } else if constexpr (MA == KC && MB == RC) {
      ESP_SPEC(EPI_BMUL)
      ESP_SPEC(EPI_RMASK)
      ESP_SPEC(EPI_BMUL_PL)
      ESP_SPEC(EPI_RMASK_PL)
    } else if constexpr (MA == I2CT_KC && MB == RC) {
      ESP_SPEC(EPI_RMASKMAP)
      if constexpr (BNT == 128 && BMT == 128) ESP_SPEC(EPI_C1FOLD)
    }
#undef ESP_SPEC
  });
  return known && ok;
}

}  // namespace espg
