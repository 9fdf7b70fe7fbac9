"""Microbenchmark of the fused rel-pos attention-probability kernel at the C2 shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, T, H, dk = 64, 374, 4, 64
    D, Z, P = H * dk, H * B, 2 * T - 1
    Tp = K.pitch(T)
    qu = torch.randn(Z * T * dk, device=dev)
    qv = torch.randn(Z * T * dk, device=dev)
    qkv = torch.randn(B * T * 3 * D, device=dev)
    p = torch.randn(P * D, device=dev)
    klen = torch.full((B,), T, dtype=torch.int32, device=dev)
    attn = torch.empty(Z * T * Tp, device=dev)
    pdrop = torch.empty(Z * T * Tp, device=dev)
    for pa in (0.0, 0.1):
        for _ in range(3):
            K.relpos_attn_fwd(qu, qv, qkv, 3 * D, p, D, B, H, 8.0, klen, attn, pdrop, pa, 1, T, Tp, k_off=D)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            K.relpos_attn_fwd(qu, qv, qkv, 3 * D, p, D, B, H, 8.0, klen, attn, pdrop, pa, 1, T, Tp, k_off=D)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        flop = 2.0 * Z * T * dk * (T + ((T + 31 + 31) // 32) * 32 * ((T + 31) // 32) / ((T + 31) // 32))
        print(f"fwd drop={pa}: {us:.1f} us  ({flop / us / 1e6:.1f} TF/s on ac + bd-window MFMAs)", flush=True)
    dctx = torch.randn(B * T * D, device=dev)
    dS = torch.empty(Z * T * Tp, device=dev)
    Pp = K.pitch(P)
    dbd = torch.empty(Z * T * Pp, device=dev)
    for pa in (0.0, 0.1):
        for _ in range(3):
            K.relpos_attn_bwd(dctx, D, qkv, 3 * D, attn, dS, dbd, Pp, B, H, 8.0, pa, 1, T, Tp, v_off=2 * D)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            K.relpos_attn_bwd(dctx, D, qkv, 3 * D, attn, dS, dbd, Pp, B, H, 8.0, pa, 1, T, Tp, v_off=2 * D)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"bwd drop={pa}: {us:.1f} us  ({Z * T * T * 4 * 4 / us / 1e6:.2f} TB/s on attn + dS + 2x dbd)", flush=True)


if __name__ == "__main__":
    main()
