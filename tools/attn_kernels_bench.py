"""Microbenchmark of the materialised rel-pos attention kernels of one C2 layer at B utterances
(default 128): the probabilities kernel, the P.V and dS.K batched GEMMs and the softmax /
rel_shift adjoint.  Used alone for timings and under rocprofv3 --pmc for per-kernel counters.

    python tools/attn_kernels_bench.py [B] [--only probs|pv|sbwd|dsk] [--legacy] [--nodrop]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
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
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B = int(args[0]) if args else 128
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    rel = 2 if "--legacy" in sys.argv else 1
    T, H, dk = 374, 4, 64
    D, Z = H * dk, H * B
    P = T if rel == 2 else 2 * T - 1
    Tp, Pp = K.pitch(T), K.pitch(P)
    g = torch.Generator(device=dev).manual_seed(0)
    qu = torch.randn(Z * T * dk, device=dev, generator=g)
    qv = torch.randn(Z * T * dk, device=dev, generator=g)
    qkv = torch.randn(B * T * 3 * D, device=dev, generator=g)
    p = torch.randn(P * D, device=dev, generator=g)
    klen = torch.full((B,), T, dtype=torch.int32, device=dev)
    attn = torch.empty(Z * T * Tp, device=dev)
    pdrop = torch.empty(Z * T * Tp, device=dev)
    ctx = torch.empty(B * T * D, device=dev)
    dctx = torch.randn(B * T * D, device=dev, generator=g)
    dS = torch.randn(Z * T * Tp, device=dev, generator=g)
    dbd = torch.empty(Z * T * Pp, device=dev)
    dqkv = torch.empty(B * T * 3 * D, device=dev)
    pa = 0.1
    K.relpos_attn_probs(qu, qv, qkv, 3 * D, p, D, rel, B, H, 8.0, klen, attn, pdrop, pa, 1, T, Tp, k_off=D)
    nt = (T + 15) // 16
    res = {}
    if "--nodrop" in sys.argv:  # the probabilities kernel without dropout and without the P_drop copy
        us = timed(lambda: K.relpos_attn_probs(qu, qv, qkv, 3 * D, p, D, rel, B, H, 8.0, klen, attn, None, 0.0, 1, T,
                                               Tp, k_off=D))
        res["probs0"] = (us, f"{2.0 * Z * T * T * dk * 2 / us / 1e6:.1f} TF/s algorithmic, no dropout / no P_drop")
    if only in (None, "probs"):
        us = timed(lambda: K.relpos_attn_probs(qu, qv, qkv, 3 * D, p, D, rel, B, H, 8.0, klen, attn, pdrop, pa, 1, T,
                                               Tp, k_off=D))
        alg = 2.0 * Z * T * T * dk * 2  # ac + bd over the T x T scores (algorithmic, no padded tiles)
        res["probs"] = (us, f"{alg / us / 1e6:.1f} TF/s algorithmic (ac + bd), "
                            f"{2.0 * 16 * 16 * 64 * (2 * nt + 1) * nt * Z / us / 1e6:.1f} TF/s on issued MFMAs")
    if only in (None, "pv"):
        us = timed(lambda: K.gemm(T, dk, T, pdrop, qkv, ctx, mode_a=K.KC, lda=Tp, mode_b=K.RC, ldb=3 * D, ldc=D,
                                  b_off=2 * D, batch=Z, nb2=B, sa=(B * T * Tp, T * Tp), sb=(dk, T * 3 * D),
                                  sc=(dk, T * D)))
        res["pv"] = (us, f"{2.0 * Z * T * T * dk / us / 1e6:.1f} TF/s")
    if only in (None, "dsk"):
        us = timed(lambda: K.gemm(T, dk, T, dS, qkv, dqkv, mode_a=K.KC, lda=Tp, mode_b=K.RC, ldb=3 * D, ldc=3 * D,
                                  b_off=D, batch=Z, nb2=B, sa=(B * T * Tp, T * Tp), sb=(dk, T * 3 * D),
                                  sc=(dk, T * 3 * D)))
        res["dsk"] = (us, f"{2.0 * Z * T * T * dk / us / 1e6:.1f} TF/s")
    if only in (None, "sbwd"):
        us = timed(lambda: K.attn_softmax_bwd_relpos(attn, dS, dS, dbd, Pp, pa, 1, 8.0, Z * T, T, Tp, relpos=rel))
        byt = 4.0 * Z * T * (3 * T + P)  # P, dP read; dS, dbd written
        res["sbwd"] = (us, f"{byt / us / 1e6:.2f} TB/s")
    for k, (us, info) in res.items():
        print(f"{k:6s} {us:8.1f} us  {info}", flush=True)


if __name__ == "__main__":
    main()
