"""Conv2dSubsampling conv2 input gradient at C2 (B utterances, T=1500, D=256): the column GEMM +
col2im_relu path against the implicit parity-class GEMMs (esp_conv2_dgrad).

    python tools/conv2_dgrad_bench.py [B]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    D, T, F = 256, 1500, 80
    T1, F1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
    T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
    npix2 = B * T2 * F2
    g = torch.Generator(device=dev).manual_seed(0)
    dz2 = torch.randn(npix2, D, device=dev, generator=g)
    W = torch.randn(D, D, 3, 3, device=dev, generator=g) / 48.0
    w2r = W.permute(0, 2, 3, 1).reshape(D, 9 * D).contiguous()  # (o, kt, kf, c)
    z1 = torch.relu(torch.randn(B * T1 * F1 * D, device=dev, generator=g))
    dz1a = torch.empty(B * T1 * F1 * D, device=dev)
    dz1b = torch.empty(B * T1 * F1 * D, device=dev)
    flop = 2.0 * npix2 * 9 * D * D

    def column():
        dcol = torch.empty(npix2, 9 * D, device=dev)
        K.gemm(npix2, 9 * D, D, dz2, w2r, dcol, mode_a=K.KC, lda=D, mode_b=K.RC, ldb=9 * D, ldc=9 * D)
        K.col2im_relu(dcol, z1, dz1a, B, T1, F1, D)

    def implicit():
        K.conv2_dgrad(dz2, W, z1, dz1b, B, T1, F1, D)

    tc = timed(column)
    ti = timed(implicit)
    err = (dz1a - dz1b).abs().max().item() / max(1e-30, dz1a.abs().max().item())
    print(f"column GEMM + col2im  {tc:7.3f} ms  ({flop / tc / 1e9:6.1f} TF/s on the dgrad FLOPs)", flush=True)
    print(f"implicit classes      {ti:7.3f} ms  ({flop / ti / 1e9:6.1f} TF/s)   max rel diff {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
