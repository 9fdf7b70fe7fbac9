"""One GEMM shape, repeated (for rocprofv3 --pmc passes and quick timings):
    python tools/gemm_one.py mode_a mode_b M N K [reps] [--rowsum] [--bw]
fp32 operands (the default fp32 split-product path; PREC 0, or with --bw B taken as a weight: its split
planes made per call, PREC 3; --pl: both operands given as split planes made once, PREC 5)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402


def main():
    a = [x for x in sys.argv[1:] if not x.startswith("--")]
    ma, mb, M, N, Kk = (int(v) for v in a[:5])
    reps = int(a[5]) if len(a) > 5 else 20
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn(M * Kk, device=dev, generator=g)
    B = torch.randn(N * Kk, device=dev, generator=g)
    C = torch.empty(M * N, device=dev)
    rs = torch.zeros(M, device=dev) if "--rowsum" in sys.argv else None
    lda = Kk if ma == K.KC else M
    ldb = Kk if mb == K.KC else N
    bw = "--bw" in sys.argv
    if "--pl" in sys.argv:
        A = K.Planes.of(A.view(M, Kk) if ma == K.KC else A.view(Kk, M))
        B = K.Planes.of(B.view(N, Kk) if mb == K.KC else B.view(Kk, N))
    fn = lambda: K.gemm(M, N, Kk, A, B, C, mode_a=ma, lda=lda, mode_b=mb, ldb=ldb, ldc=N, rowsum=rs,  # noqa: E731
                        b_weight=bw)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"({ma},{mb},{M},{N},{Kk}) {us:.1f} us  {2.0 * M * N * Kk / us / 1e6:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
