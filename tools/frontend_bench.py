"""Front-end kernel throughput at the bench scale (64 utterances x 12 s of 16 kHz audio ->
1501 frames of 80 log-mel), against the HBM roofline of its algorithmic bytes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402
from espnet_slurp_amd.asr.frontend.default import DefaultFrontend  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, N = 64, 192000
    fe = DefaultFrontend()
    x = torch.randn(B, N, device=dev) * 0.3
    lens = K.h2d(torch.full((B,), N, dtype=torch.int32), dev)
    for _ in range(3):
        out = fe.apply_prepared(x, lens, N)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        out = fe.apply_prepared(x, lens, N)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    nbytes = x.numel() * 4 + out.numel() * 4
    print(f"fbank B={B} N={N} -> {tuple(out.shape)}: {us:.1f} us, {nbytes / us / 1e6:.2f} TB/s algorithmic "
          f"({nbytes / 1e6:.1f} MB), {B * N / 16000 / (us * 1e-6):.0f} s of audio per s", flush=True)


if __name__ == "__main__":
    main()
