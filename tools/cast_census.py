"""Census of the bf16 operand casts (esp_f32_to_bf16 / esp_f32_to_planes launches) of one eager training
step in the reduced-precision mode: count and elements per call site (the first caller outside
kernels.py), so the casts a producer could absorb are named.  python tools/cast_census.py [--batch 64]"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from espnet_slurp_amd import kernels as K  # noqa: E402
from espnet_slurp_amd.optimizers.fused_adam import FusedAdam  # noqa: E402
from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR  # noqa: E402
from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--config", choices=sorted(bench.PRESETS), default="c5")
    a = ap.parse_args()
    d, heads, ff, layers, amp = bench.PRESETS[a.config]
    args = argparse.Namespace(d=d, heads=heads, ff=ff, layers=layers, vocab=600, rel_pos="latest", batch=a.batch)
    dev = torch.device("cuda:0")
    model = bench.build(args, dev)
    opt = FusedAdam(model.parameters(), model.flat, lr=2e-4)
    tr = Trainer(model, opt, WarmupLR(opt, 25000), TrainerOptions(use_amp=amp))
    batch = bench.synthetic_batch(args.batch, 600, 0, dev)
    tr.train_one_step(batch)
    torch.cuda.synchronize()
    census = collections.Counter()
    elems = collections.Counter()
    real = K._native.call
    here = os.path.abspath(K.__file__)

    def call(name, *xs):
        if name in ("esp_f32_to_bf16", "esp_f32_to_planes"):
            site = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if os.path.abspath(fr.filename) != here:
                    site = f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
                    break
            kernel_site = next((f"{fr.lineno} {fr.name}" for fr in reversed(traceback.extract_stack()[:-1])
                                if os.path.abspath(fr.filename) == here), "?")
            rows, cols = int(xs[2]), int(xs[3])
            key = (name, site, kernel_site, rows, cols)
            census[key] += 1
            elems[key] += rows * cols
        return real(name, *xs)

    K._native.call = call
    try:
        tr.train_one_step(batch)
        torch.cuda.synchronize()
    finally:
        K._native.call = real
    print(f"# {sum(census.values())} casts, {sum(elems.values()) / 1e6:.1f} M elements in one eager step "
          f"({a.config} B={a.batch})")
    for key, n in sorted(census.items(), key=lambda kv: -elems[kv[0]]):
        name, site, ks, rows, cols = key
        print(f"{n:4d} x {rows:7d} x {cols:5d}  {elems[key] / 1e6:8.1f} M  {name:17s} {site:45s} via kernels.py:{ks}")


if __name__ == "__main__":
    main()
