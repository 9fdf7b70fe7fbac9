// Instantiations of gemm_glds_kernel with the generic (run-time feature flag) fused epilogues:
// EPI_FWD for the forward mode pairs, EPI_BWD for the input-gradient pairs.  Device code in
// gemm_kernels.h.
#include "gemm_kernels.h"

namespace espg {

bool glds_launch_epi(int ma, int mb, int bnt, int prec, int epi, dim3 grid, hipStream_t st, const GemmArgs& g,
                     const GldsArgs& x) {
  bool ok = false;
  const bool known = glds_switch(ma, mb, bnt, prec, g.bm, [&](auto A, auto B, auto N, auto F, auto R) {
    constexpr int MA = decltype(A)::value, MB = decltype(B)::value, BNT = decltype(N)::value;
    constexpr int BF = decltype(F)::value, BMT = decltype(R)::value;
    constexpr bool can_fwd = (MA == KC && (MB == KC || MB == RC)) || (MA == I2C_KC && MB == KC);
    constexpr bool can_bwd = (MA == KC || MA == I2CT_KC) && MB == RC;
    if constexpr (can_fwd) {
      if (epi == EPI_FWD) {
        hipLaunchKernelGGL((gemm_glds_kernel<MA, MB, BNT, false, EPI_FWD, BF, BMT>), grid, dim3(glds_threads(BMT)), 0, st, g, x);
        ok = true;
      }
    }
    if constexpr (can_bwd) {
      if (epi == EPI_BWD) {
        hipLaunchKernelGGL((gemm_glds_kernel<MA, MB, BNT, false, EPI_BWD, BF, BMT>), grid, dim3(glds_threads(BMT)), 0, st, g, x);
        ok = true;
      }
    }
  });
  return known && ok;
}

}  // namespace espg
