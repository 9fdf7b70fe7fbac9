"""Microbenchmark of the MFMA GEMM on the shapes of the C2 training step (B=64)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402

NB = int(os.environ.get("GEMM_BENCH_B", "64"))  # utterances per batch
M = NB * 374
SHAPES = [  # (mode_a, mode_b, M, N, K, batch, label)
    (0, 1, M, 1024, 256, 1, "ffn w1 fwd"),
    (0, 1, M, 256, 1024, 1, "ffn w2 fwd"),
    (0, 0, M, 256, 1024, 1, "ffn dX w2"),
    (0, 0, M, 1024, 256, 1, "ffn dX w1"),
    (1, 1, 256, 1024, M, 1, "ffn dW w2"),
    (1, 1, 1024, 256, M, 1, "ffn dW w1"),
    (1, 1, 256, 256, M, 1, "dW 256x256"),
    (0, 1, M, 768, 256, 1, "qkv fwd"),
    (0, 0, 374, 374, 64, 256, "scores ac"),
    (0, 1, 374, 64, 374, 256, "ctx = P V"),
    (1, 1, 374, 64, 374, 256, "dV / dk"),
    (0, 1, 374, 64, 374, 256, "ctx pad376", 376),
    (1, 1, 374, 64, 374, 256, "dV pad376", 376),
    (0, 0, 374, 374, 64, 256, "scores ldc376", 376),
    (1, 3, 256, 2304, NB * 374 * 19, 1, "conv2 dW"),
    (2, 0, NB * 374 * 19, 256, 2304, 1, "conv2 fwd"),
    (0, 1, NB * 374 * 19, 2304, 256, 1, "conv2 dcol"),
    (0, 1, NB * 41, 256, 256, 1, "decoder q"),
    (0, 1, NB * 41, 256, 2048, 1, "decoder ffn w2"),
]


def run(ma, mb, m, n, k, batch, pad=None, reps=20):
    dev = torch.device("cuda:0")
    lda = k if ma == 0 else m
    ldb = k if mb == 0 else n
    ldc = n
    if pad:  # padded pitch on the T-long dims (attention score layouts)
        if ma == 0 and k == 374:
            lda = pad
        if ma == 1 and m == 374:
            lda = pad
        if n == 374:
            ldc = pad
    ic_a = ic_b = None
    if ma == 2:  # conv2 forward: NHWC map (B, 749, 39, 256) -> pixels (B*374*19)
        ic_a = (749, 39, 256, 374, 19)
        A = torch.randn(NB * 749 * 39 * 256, device=dev)
    else:
        A = torch.randn(batch * max(m, lda) * max(k, lda), device=dev) if pad else torch.randn(batch * m * k, device=dev)
    if mb == 3:
        ic_b = (749, 39, 256, 374, 19)
        B = torch.randn(NB * 749 * 39 * 256, device=dev)
    else:
        B = torch.randn(batch * n * k, device=dev)
    C = torch.empty(batch * m * ldc, device=dev)
    sa = (m * k, 0) if not pad else (A.numel() // batch, 0)
    kw = dict(mode_a=ma, lda=lda, mode_b=mb, ldb=ldb, ldc=ldc, batch=batch, nb2=1, sa=sa, sb=(n * k, 0),
              sc=(m * ldc, 0), ic_a=ic_a, ic_b=ic_b)
    for _ in range(3):
        K.gemm(m, n, k, A, B, C, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        K.gemm(m, n, k, A, B, C, **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return ms, 2.0 * m * n * k * batch / (ms * 1e-3) / 1e12


def run_torch(ma, mb, m, n, k, batch, reps=20):
    """The same product through torch.matmul (rocBLAS / hipBLASLt fp32) for comparison."""
    dev = torch.device("cuda:0")
    A = torch.randn(batch, m, k, device=dev) if ma == 0 else torch.randn(batch, k, m, device=dev).transpose(1, 2)
    B = torch.randn(batch, n, k, device=dev).transpose(1, 2) if mb == 0 else torch.randn(batch, k, n, device=dev)
    if batch == 1:
        A, B = A[0], B[0]
    for _ in range(3):
        C = torch.matmul(A, B)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        C = torch.matmul(A, B)
    e1.record()
    torch.cuda.synchronize()
    del C
    ms = e0.elapsed_time(e1) / reps
    return ms, 2.0 * m * n * k * batch / (ms * 1e-3) / 1e12


if __name__ == "__main__":
    only = [int(a) for a in sys.argv[1:]]
    for i, sh in enumerate(SHAPES):
        ma, mb, m, n, k, b, lab = sh[:7]
        pad = sh[7] if len(sh) > 7 else None
        if only and i not in only:
            continue
        ms, tf = run(ma, mb, m, n, k, b, pad)
        line = f"{lab:16s} ({ma},{mb}) M={m:6d} N={n:5d} K={k:6d} b={b:3d}  {ms * 1e3:8.1f} us  {tf:6.1f} TF/s"
        if os.environ.get("GEMM_BENCH_TORCH") and ma < 2 and mb < 2 and not pad:
            tms, ttf = run_torch(ma, mb, m, n, k, b)
            line += f"   | torch.matmul {tms * 1e3:8.1f} us  {ttf:6.1f} TF/s"
        print(line, flush=True)
