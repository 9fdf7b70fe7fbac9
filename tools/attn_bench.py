"""Microbenchmark of the fused rel-pos attention-probability kernel at the C2 shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    fwd_only = '--fwd-only' in sys.argv
    T, H, dk = 374, 4, 64
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
    for name, rel in (("wave16 latest", 1), ("wave16 legacy", 2)):
        pt = p if rel == 1 else torch.randn(T * D, device=dev)
        for pa in (0.0, 0.1):
            for _ in range(3):
                K.relpos_attn_probs(qu, qv, qkv, 3 * D, pt, D, rel, B, H, 8.0, klen, attn, pdrop, pa, 1, T, Tp,
                                    k_off=D)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                K.relpos_attn_probs(qu, qv, qkv, 3 * D, pt, D, rel, B, H, 8.0, klen, attn, pdrop, pa, 1, T, Tp,
                                    k_off=D)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            flop = 2.0 * Z * T * dk * (T + 16 * ((T + 15) // 16 + 1))
            print(f"{name} drop={pa}: {us:.1f} us  ({flop / us / 1e6:.1f} TF/s on ac + band MFMAs)", flush=True)
    if fwd_only:
        return
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
