"""Tile quantization probe: the ffn w1 input-gradient GEMM (KC x RC, N = 256, K = 1024, B as cached
planes) over M = 128-row tile counts around the 512 resident-block slots (2 per CU); time per tile
row shows whether a partly filled last round costs a full round."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N, Kd = 256, 1024
    B = torch.randn(Kd * N, device=dev)
    for rows in (256, 320, 374, 384, 448, 512, 640, 768):
        M = rows * 128
        A = torch.randn(M * Kd, device=dev)
        C = torch.empty(M * N, device=dev)
        kw = dict(mode_a=K.KC, lda=Kd, mode_b=K.RC, ldb=N, ldc=N, b_weight=True)
        with K.param_cast_scope():
            for _ in range(3):
                K.gemm(M, N, Kd, A, B, C, **kw)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                K.gemm(M, N, Kd, A, B, C, **kw)
            e1.record()
            torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"M={M:6d} tiles={rows * 2:5d} rounds={rows * 2 / 512:.2f}  {us:7.1f} us  {us / rows:6.3f} us per tile row "
              f"{2.0 * M * N * Kd / us / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
