"""bf16-operand GEMM (esp_gemm_bf16, PREC 2) vs the fp32-staged bf16 MFMA path (PREC 1) and the
fp32 path on C5-sized shapes; also the cost of the fp32 -> bf16 casts.  HIP events, 20 reps."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    shapes = [("ffn w1 fwd", 11968, 2048, 512), ("ffn w2 fwd", 11968, 512, 2048), ("qkv fwd", 11968, 1536, 512),
              ("ffn w1 dW", 2048, 512, 11968), ("ffn w2 dW", 512, 2048, 11968), ("big C2 w1", 47872, 1024, 256),
              ("square 8k", 8192, 8192, 8192)]
    for name, M, N, Kd in shapes:
        A = torch.randn(M, Kd, device=dev)
        B = torch.randn(N, Kd, device=dev)
        C = torch.empty(M, N, device=dev)
        A16, B16 = A.to(torch.bfloat16), B.to(torch.bfloat16)
        fl = 2.0 * M * N * Kd
        t2 = timeit(lambda: K.gemm_bf16(M, N, Kd, A16, B16, C, lda=Kd, ldb=Kd, ldc=N))
        ref = (A16.float() @ B16.float().t())
        err = ((C - ref).abs().max() / ref.abs().max()).item()
        with K.gemm_compute("bf16"):
            t1 = timeit(lambda: K.gemm(M, N, Kd, A, B, C, lda=Kd, ldb=Kd, ldc=N))
        t0 = timeit(lambda: K.gemm(M, N, Kd, A, B, C, lda=Kd, ldb=Kd, ldc=N))
        tc = timeit(lambda: K.to_bf16(A, M, Kd, Kd, out=A16))
        tt = timeit(lambda: K.to_bf16(A, M, Kd, Kd, transpose=True))
        print(f"{name:12s} M={M:6d} N={N:5d} K={Kd:6d}  bf16-operand {t2:8.1f} us {fl / t2 / 1e6:7.1f} TF/s | "
              f"bf16-staged {t1:8.1f} us {fl / t1 / 1e6:7.1f} | fp32 {t0:8.1f} us {fl / t0 / 1e6:6.1f} | "
              f"cast A {tc:6.1f} us, transposed {tt:6.1f} us | rel err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
