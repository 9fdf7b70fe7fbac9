// Instantiations of gemm_glds_kernel with the specialised plain epilogues (EPI_P0: alpha*acc,
// EPI_PR: alpha*acc + beta*R; unsplit, wide stores) for the linear / attention mode pairs, and the
// attention score-gradient epilogue (EPI_SMB, KC x KC fp32: esp_attn_dscores).
// See store_spec in gemm_kernels.h.
#include "gemm_kernels.h"

namespace espg {

bool glds_launch_pspec(int ma, int mb, int bnt, int prec, int epi, dim3 grid, hipStream_t st, const GemmArgs& g,
                       const GldsArgs& x) {
  bool ok = false;
  const bool known = glds_switch(ma, mb, bnt, prec, g.bm, [&](auto A, auto B, auto N, auto F, auto R) {
    constexpr int MA = decltype(A)::value, MB = decltype(B)::value, BNT = decltype(N)::value;
    constexpr int BF = decltype(F)::value, BMT = decltype(R)::value;
    if constexpr ((MA == KC || MA == RC) && (MB == KC || MB == RC)) {
      if (epi == EPI_P0) {
        hipLaunchKernelGGL((gemm_glds_kernel<MA, MB, BNT, false, EPI_P0, BF, BMT>), grid, dim3(glds_threads(BMT)), 0, st, g, x);
        ok = true;
      } else if (epi == EPI_PR) {
        hipLaunchKernelGGL((gemm_glds_kernel<MA, MB, BNT, false, EPI_PR, BF, BMT>), grid, dim3(glds_threads(BMT)), 0, st, g, x);
        ok = true;
      } else if constexpr (MA == KC && MB == RC && BF <= 1) {  // the attention context as planes (P.V)
        if (epi == EPI_P0_PL) {
          hipLaunchKernelGGL((gemm_glds_kernel<MA, MB, BNT, false, EPI_P0_PL, BF, BMT>), grid, dim3(glds_threads(BMT)), 0, st, g, x);
          ok = true;
        }
      } else if constexpr (MA == KC && MB == KC && BF == 0) {
        if (epi == EPI_SMB) {
          hipLaunchKernelGGL((gemm_glds_kernel<MA, MB, BNT, false, EPI_SMB, BF, BMT>), grid, dim3(glds_threads(BMT)), 0, st, g, x);
          ok = true;
        }
      }
    }
  });
  return known && ok;
}

}  // namespace espg
