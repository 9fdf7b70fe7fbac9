"""Planes GEMMs vs the in-register split (PREC 0) on the weight-B shapes of the C2 step at B=128:
forward (KC x KC) and input-gradient (KC x RC) linears and the conv2 forward; B planes (PREC 3) and
A + B planes (PREC 5, A as kernels.Planes).  Weight planes made once (param_cast_scope), as in the
Trainer step.  Prints per shape the kernel time of each and the max |difference| (0 when no split-K)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402

NB = int(os.environ.get("BP_BENCH_B", "128"))
M = NB * 374
SHAPES = [  # (mode_a, mode_b, M, N, K, label)
    (0, 0, M, 1024, 256, "ffn w1 fwd"),
    (0, 0, M, 256, 1024, "ffn w2 fwd"),
    (0, 1, M, 1024, 256, "ffn w2 dX"),
    (0, 1, M, 256, 1024, "ffn w1 dX"),
    (0, 0, M, 768, 256, "qkv fwd"),
    (0, 1, M, 256, 768, "qkv dX"),
    (0, 0, M, 256, 256, "out fwd"),
    (0, 1, M, 256, 256, "out dX"),
    (0, 0, M, 512, 256, "pw1 fwd"),
    (0, 1, M, 256, 512, "pw1 dX"),
    (2, 0, NB * 374 * 19, 256, 2304, "conv2 fwd"),
    (0, 0, NB * 41, 256, 256, "dec q fwd"),
    (0, 0, NB * 41, 2048, 256, "dec w1 fwd"),
]


def run(ma, mb, m, n, k, reps=10):
    """kernel ms of: the in-register split (fp32 A and B), B planes, A and B planes (A as kernels.Planes;
    KC / RC A only); max |difference| of the planes results to the split one"""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(m + n + k)
    ic_a = None
    if ma == 2:
        ic_a = (749, 39, 256, 374, 19)
        A = torch.randn(NB * 749 * 39 * 256, device=dev, generator=g)
        lda = 0
    else:
        A = torch.randn(m * k, device=dev, generator=g)
        lda = k
    B = torch.randn(n * k, device=dev, generator=g)
    ldb = k if mb == 0 else n
    out = {}
    modes = ("split", "bp", "pl") if ma in (0, 1) else ("split", "bp")
    for mode in modes:
        C = torch.empty(m * n, device=dev)
        Ax, la = A, lda
        if mode == "pl":
            Ax = K.Planes.of(A.view(m, k) if ma == 0 else A.view(k, m))
            la = Ax.ld
        kw = dict(mode_a=ma, lda=la, mode_b=mb, ldb=ldb, ldc=n, ic_a=ic_a, b_weight=mode != "split")
        with K.param_cast_scope():
            for _ in range(2):
                K.gemm(m, n, k, Ax, B, C, **kw)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                K.gemm(m, n, k, Ax, B, C, **kw)
            e1.record()
            torch.cuda.synchronize()
        out[mode] = (e0.elapsed_time(e1) / reps, C)
    d = max((out[x][1] - out["split"][1]).abs().max().item() for x in modes)
    return {x: out[x][0] for x in modes}, d


def one(i, bp, reps):
    """one shape, one mode, `reps` launches (for rocprofv3 --pmc passes)"""
    ma, mb, m, n, k, label = SHAPES[i]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(m + n + k)
    ic_a = (749, 39, 256, 374, 19) if ma == 2 else None
    A = torch.randn(NB * 749 * 39 * 256 if ma == 2 else m * k, device=dev, generator=g)
    B = torch.randn(n * k, device=dev, generator=g)
    C = torch.empty(m * n, device=dev)
    kw = dict(mode_a=ma, lda=0 if ma == 2 else k, mode_b=mb, ldb=k if mb == 0 else n, ldc=n, ic_a=ic_a, b_weight=bp)
    with K.param_cast_scope():
        for _ in range(reps):
            K.gemm(m, n, k, A, B, C, **kw)
    torch.cuda.synchronize()
    print(label, "bp" if bp else "split", "done")


def main():
    if len(sys.argv) > 1:
        return one(int(sys.argv[1]), sys.argv[2] == "1", int(sys.argv[3]) if len(sys.argv) > 3 else 5)
    tot = {}
    for ma, mb, m, n, k, label in SHAPES:
        t, d = run(ma, mb, m, n, k)
        fl = 2.0 * m * n * k
        line = f"{label:12s} ({ma},{mb},{m},{n},{k})"
        for x, ms in t.items():
            tot[x] = tot.get(x, 0.0) + ms
            line += f"  {x} {1e3 * ms:8.1f} us {fl / ms / 1e9:6.1f} TF/s"
        print(line + f"  maxdiff {d:.3g}", flush=True)
    print("total " + " ".join(f"{x} {v:.3f} ms" for x, v in tot.items()))


if __name__ == "__main__":
    main()
