"""fp32 GEMM accuracy against fp64, for the library this process loads (ESP_LIB_VARIANT selects an
experiment build): max |C - C64| / (|A| |B|)(m, n) (the error bound's natural scale) and the
rms of the same ratio, over the step's shapes (K = 256 .. 47872) in every operand mode pair.
Usage: python tools/f32_gemm_accuracy.py   (prints one line per case)."""
import sys

import torch

sys.path.insert(0, ".")
from espnet_slurp_amd import kernels as K  # noqa: E402


def case(M, N, Kk, ma, mb, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(M, Kk, generator=g) * scale
    B = torch.randn(Kk, N, generator=g)
    Ad = (A if ma == K.KC else A.t().contiguous()).cuda()
    Bd = (B.t().contiguous() if mb == K.KC else B).cuda()
    C = torch.empty(M, N, device="cuda")
    K.gemm(M, N, Kk, Ad, Bd, C, mode_a=ma, lda=Ad.stride(0), mode_b=mb, ldb=Bd.stride(0), ldc=N)
    torch.cuda.synchronize()
    ref = A.double() @ B.double()
    den = A.double().abs() @ B.double().abs()
    r = (C.cpu().double() - ref).abs() / den
    # native fp32 reference on the CPU (sequential fp32 dot products) at the same scale
    c32 = (A @ B).double()
    r32 = (c32 - ref).abs() / den
    return r.max().item(), r.pow(2).mean().sqrt().item(), r32.max().item(), r32.pow(2).mean().sqrt().item()


def main():
    torch.cuda.init()
    for (M, N, Kk) in [(2048, 1024, 256), (2048, 256, 1024), (256, 1024, 47872), (1024, 256, 2304), (512, 512, 16384)]:
        for ma, mb in [(K.KC, K.KC), (K.KC, K.RC), (K.RC, K.RC)]:
            mx, rms, mx32, rms32 = case(M, N, Kk, ma, mb)
            print(f"M={M:5d} N={N:5d} K={Kk:6d} modes=({ma},{mb})  gpu max {mx:.3e} rms {rms:.3e}   "
                  f"cpu-fp32 max {mx32:.3e} rms {rms32:.3e}", flush=True)


if __name__ == "__main__":
    main()
