"""The implicit conv2 input gradient with conv1's weight gradient folded in (esp_conv2_dgrad_c1fold) at C2
shapes, alone: B utterances, T=1500, D=256.  Run under rocprofv3 --kernel-trace --stats for the per-class times.

    python tools/c1fold_bench.py [B]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    D, T, F = 256, 1500, 80
    T1, F1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
    T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, T, F, device=dev, generator=g)
    w0 = torch.randn(D, 1, 3, 3, device=dev, generator=g) * 0.3
    b0 = torch.randn(D, device=dev, generator=g) * 0.1
    z1 = torch.empty(B * T1 * F1 * D, device=dev)
    bits = torch.empty(B * T1 * F1 * D // 32, dtype=torch.int32, device=dev)
    K.conv1_fwd(x, w0, b0, z1, B, T, F, D, zbits=bits)
    del z1
    dz2 = torch.randn(B * T2 * F2, D, device=dev, generator=g)
    W = torch.randn(D, D, 3, 3, device=dev, generator=g) / 48.0
    dW, db = torch.zeros(D, 9, device=dev), torch.zeros(D, device=dev)
    for _ in range(2):
        K.conv2_dgrad_c1fold(dz2, W, bits, x, T, F, dW, db, B, T1, F1, D)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        K.conv2_dgrad_c1fold(dz2, W, bits, x, T, F, dW, db, B, T1, F1, D)
    e1.record()
    torch.cuda.synchronize()
    print(f"c1fold {e0.elapsed_time(e1) / 5:.3f} ms per call", flush=True)


if __name__ == "__main__":
    main()
