"""Host enqueue cost of one training step (no sync inside) vs its GPU time: tells whether the
step is launch/host-bound.  Usage: python tools/host_overhead.py [--batch B]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from espnet_slurp_amd.optimizers.fused_adam import FusedAdam  # noqa: E402
from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR  # noqa: E402
from espnet_slurp_amd.train.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    args = argparse.Namespace(d=256, heads=4, ff=1024, layers=12, vocab=600, rel_pos="latest", batch=a.batch)
    dev = torch.device("cuda:0")
    model = bench.build(args, dev)
    opt = FusedAdam(model.parameters(), model.flat, lr=2e-4)
    tr = Trainer(model, opt, WarmupLR(opt, 25000))
    batch = bench.synthetic_batch(args.batch, 600, 0, dev)
    for _ in range(3):
        tr.train_one_step(batch)
    torch.cuda.synchronize()
    # GPU time of a step
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        tr.train_one_step(batch, check_finite=False)
    e1.record()
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / 5
    # host enqueue time with the GPU kept busy by a long sleep kernel first (queue never drains)
    torch.cuda._sleep(int(2e9))
    t0 = time.perf_counter()
    for _ in range(2):
        tr.train_one_step(batch, check_finite=False)
    host_ms = (time.perf_counter() - t0) * 1e3 / 2
    torch.cuda.synchronize()
    print(f"B={a.batch}: wall/step (no finite sync) {gpu_ms:.1f} ms, host enqueue/step {host_ms:.1f} ms")


if __name__ == "__main__":
    main()
