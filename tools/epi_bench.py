"""GEMM epilogue cost on the FFN w_1 shape (M=B*T'=23936, N=1024, K=256): plain / bias /
bias+Swish+aux / +dropout / backward-activation, HIP-event timed (20 reps each)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    M, N, Kk = 23936, 1024, 256
    x = torch.randn(M, Kk, device=dev)
    W = torch.randn(N, Kk, device=dev)
    b = torch.randn(N, device=dev)
    out = torch.empty(M, N, device=dev)
    aux = torch.empty(M, N, device=dev)
    dy = torch.randn(M, Kk, device=dev)
    W2 = torch.randn(Kk, N, device=dev)
    cases = {
        "plain": lambda: K.linear_fwd(x, W, None, out),
        "bias": lambda: K.linear_fwd(x, W, b, out),
        "bias+swish": lambda: K.linear_fwd(x, W, b, out, act=K.ACT_SWISH),
        "bias+swish+aux": lambda: K.linear_fwd(x, W, b, out, act=K.ACT_SWISH, aux=aux),
        "bias+swish+aux+drop": lambda: K.linear_fwd(x, W, b, out, act=K.ACT_SWISH, aux=aux, drop_p=0.1, seed=5),
        "dgrad plain": lambda: K.linear_bwd_data(dy, W2, out),
        "dgrad bwd_act": lambda: K.linear_bwd_data_act(dy, W2, out, aux, K.ACT_SWISH),
        "dgrad bwd_act+drop": lambda: K.linear_bwd_data_act(dy, W2, out, aux, K.ACT_SWISH, drop_p=0.1, seed=5),
        "act_bwd kernel+drop": lambda: K.act_bwd(out, aux, out, K.ACT_SWISH, drop_p=0.1, seed=5),
        "swish+deriv+drop": lambda: K.linear_fwd(x, W, b, out, act=K.ACT_SWISH | K.ACT_AUX_DERIV, aux=aux,
                                                 drop_p=0.1, seed=5),
        "dgrad mul": lambda: K.linear_bwd_data_act(dy, W2, out, aux, K.ACT_MUL),
        "dgrad plain +R": lambda: K.linear_bwd_data(dy, W2, out, accumulate=True),
        "fwd bias+drop+R": lambda: K.linear_fwd(x, W, b, out, drop_p=0.1, seed=5, alpha=0.5, R=aux, beta=1.0),
    }
    for name, fn in cases.items():
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name:24s} {us:8.1f} us  {2 * M * N * Kk / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
