"""Reference point: the vendor library's bf16 GEMM (torch.matmul -> hipBLASLt on ROCm) on the C5 B=64
shapes, against esp_gemm_bf16 (PREC 2) on the same bf16 operands.  Measurement only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402

SHAPES = [  # (M, N, K, label): C = A (M x K) B^T (N x K)
    (23936, 2048, 512, "ffn w1 fwd"), (23936, 512, 2048, "ffn w2 fwd"), (2048, 512, 23936, "ffn w1 dW"),
    (23936, 1536, 512, "qkv fwd"), (512, 512, 23936, "out dW"), (23936, 512, 512, "out fwd"),
    (454784, 512, 4608, "conv2 fwd shape")]


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
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    for m, n, k, label in SHAPES:
        a = torch.randn(m, k, device=dev).bfloat16()
        b = torch.randn(n, k, device=dev).bfloat16()
        c = torch.empty(m, n, device=dev)
        t_lib = timed(lambda: torch.matmul(a, b.t(), out=None))
        t_esp = timed(lambda: K.gemm_bf16(m, n, k, a, b, c, lda=k, ldb=k, ldc=n))
        fl = 2.0 * m * n * k
        print(f"{label:16s} ({m},{n},{k})  lib {t_lib:8.1f} us {fl / t_lib / 1e6:7.1f} TF/s   esp {t_esp:8.1f} us "
              f"{fl / t_esp / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
