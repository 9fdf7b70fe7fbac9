// Instantiations of gemm_glds_kernel with the plain epilogue (alpha*acc + beta*R, split-K
// partials, fused row sums).  Compiled separately from gemm.hip so the GEMM family builds in
// parallel; device code in gemm_kernels.h.
#include "gemm_kernels.h"

namespace espg {

bool glds_launch_plain(int ma, int mb, int bnt, int prec, bool rs, dim3 grid, hipStream_t st, const GemmArgs& g,
                       const GldsArgs& x) {
  return glds_switch(ma, mb, bnt, prec, g.bm, [&](auto A, auto B, auto N, auto F, auto R) {
    constexpr int MA = decltype(A)::value, MB = decltype(B)::value, BNT = decltype(N)::value;
    constexpr int BF = decltype(F)::value, BMT = decltype(R)::value;
    if constexpr (MA == RC) {
      if (rs) {
        hipLaunchKernelGGL((gemm_glds_kernel<MA, MB, BNT, true, EPI_PLAIN, BF, BMT>), grid, dim3(glds_threads(BMT)), 0, st, g, x);
        return;
      }
    }
    hipLaunchKernelGGL((gemm_glds_kernel<MA, MB, BNT, false, EPI_PLAIN, BF, BMT>), grid, dim3(glds_threads(BMT)), 0, st, g, x);
  });
}

}  // namespace espg
