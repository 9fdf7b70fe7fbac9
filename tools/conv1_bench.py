"""Microbenchmark of the conv1 forward (Conv2d(1, D, 3, 2) + ReLU, esp_conv1_fwd / esp_conv1_fwd_bits) at the C2
shape: B utterances of 1500 x 80 frames, D = 256 (7.7 GB map at B = 256).

    python tools/conv1_bench.py [B] [D]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402


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
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B = int(args[0]) if args else 256
    D = int(args[1]) if len(args) > 1 else 256
    T, F = 1500, 80
    T1, F1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, T, F, device=dev, generator=g)
    w = torch.randn(D, 1, 3, 3, device=dev, generator=g) * 0.3
    b = torch.randn(D, device=dev, generator=g) * 0.1
    z = torch.empty(B * T1 * F1 * D, device=dev)
    bits = torch.empty(B * T1 * F1 * D // 32, dtype=torch.int32, device=dev)
    gb = B * T1 * F1 * D * 4 / 1e9
    us = timed(lambda: K.conv1_fwd(x, w, b, z, B, T, F, D))
    print(f"conv1      {us:8.1f} us  {gb / us * 1e3:.2f} TB/s written", flush=True)
    us = timed(lambda: K.conv1_fwd(x, w, b, z, B, T, F, D, zbits=bits))
    print(f"conv1_bits {us:8.1f} us  {gb * 33 / 32 / us * 1e3:.2f} TB/s written", flush=True)


if __name__ == "__main__":
    main()
