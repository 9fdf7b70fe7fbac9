"""Per-shape GEMM timing of one training step (HIP events around each launch)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from espnet_slurp_amd import kernels as K  # noqa: E402
from espnet_slurp_amd.optimizers.fused_adam import FusedAdam  # noqa: E402
from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR  # noqa: E402
from espnet_slurp_amd.train.trainer import Trainer  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--config", choices=sorted(bench.PRESETS), default="c2")
    ap.add_argument("--order", default=None,
                    help="write the profiled step's GEMM launches in launch order (flops + shape key per line) "
                         "for tools/gemm_shapes_trace.py")
    a = ap.parse_args()
    d, heads, ff, layers, amp = bench.PRESETS[a.config]
    args = argparse.Namespace(d=d, heads=heads, ff=ff, layers=layers, vocab=600, rel_pos="latest", batch=a.batch)
    dev = torch.device("cuda:0")
    model = bench.build(args, dev)
    opt = FusedAdam(model.parameters(), model.flat, lr=2e-4)
    from espnet_slurp_amd.train.trainer import TrainerOptions
    tr = Trainer(model, opt, WarmupLR(opt, 25000), TrainerOptions(use_amp=amp))
    batch = bench.synthetic_batch(args.batch, 600, 0, dev)
    tr.train_one_step(batch)
    torch.cuda.synchronize()
    K.profile_gemm_start()
    launches = K._PROF  # (the list profile_gemm_stop consumes; entries in launch order)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    tr.train_one_step(batch)
    t1.record()
    flops, ms, n, shapes = K.profile_gemm_stop(by_shape=True)
    step_ms = t0.elapsed_time(t1)
    if a.order:
        with open(a.order, "w") as f:
            for fl, ev0, ev1, key, _extra in launches:
                f.write(f"{fl:.0f}\t{ev0.elapsed_time(ev1):.6f}\t{key!r}\n")
    print(f"step {step_ms:.1f} ms, gemm {ms:.1f} ms in {n} launches, {flops / ms / 1e9:.1f} TFLOP/s")
    rows = sorted(shapes.items(), key=lambda kv: -kv[1][1])
    for key, (cnt, t, f, _extra) in rows[:40]:
        print(f"{str(key):48s} n={cnt:4d} {t:8.2f} ms  {f / t / 1e9:7.1f} TF/s")


if __name__ == "__main__":
    main()
