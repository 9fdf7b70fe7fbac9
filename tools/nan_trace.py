"""Find the first kernel wrapper (espnet_slurp_amd.kernels.*) whose call turns a finite float32
tensor argument non-finite, in one eager training step (diagnostic).
usage: python tools/nan_trace.py <d> <heads> <ff> <batch>"""
import functools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import argparse  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
from espnet_slurp_amd import kernels as K  # noqa: E402

FOUND = []


def wrap(name, fn):
    @functools.wraps(fn)
    def w(*args, **kw):
        ts = [a for a in list(args) + list(kw.values()) if isinstance(a, torch.Tensor) and a.is_cuda
              and a.dtype in (torch.float32, torch.float64)]
        torch.cuda.synchronize()
        before = [bool(torch.isfinite(t).all()) for t in ts]
        out = fn(*args, **kw)
        torch.cuda.synchronize()
        after = [bool(torch.isfinite(t).all()) for t in ts]
        for i, (b, a) in enumerate(zip(before, after)):
            if b and not a and len(FOUND) < 5:
                FOUND.append(name)
                shapes = [tuple(t.shape) for t in ts]
                print(f"NONFINITE after {name}: arg {i} shape {tuple(ts[i].shape)}; float args {shapes}; "
                      f"ints {[a for a in args if isinstance(a, int)]} kw { {k: v for k, v in kw.items() if not isinstance(v, torch.Tensor)} }",
                      flush=True)
        return out
    return w


def main():
    for n in dir(K):
        f = getattr(K, n)
        if callable(f) and not n.startswith("_") and getattr(f, "__module__", "") == K.__name__ and not isinstance(f, type):
            setattr(K, n, wrap(n, f))
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions
    a = argparse.Namespace(d=int(sys.argv[1]), heads=int(sys.argv[2]), ff=int(sys.argv[3]), layers=12, vocab=600,
                           rel_pos="latest", batch=int(sys.argv[4]), amp=False)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = bench.build(a, dev)
    model.train()
    opt = FusedAdam(model.parameters(), model.flat, lr=2e-4)
    tr = Trainer(model, opt, WarmupLR(opt, 25000), TrainerOptions(grad_clip=5.0), cuda_graph=False)
    batch = bench.synthetic_batch(a.batch, a.vocab, 0, dev)
    st = tr.train_one_step(batch)
    torch.cuda.synchronize()
    print("loss", st["loss"].item(), "found", FOUND, flush=True)


if __name__ == "__main__":
    main()
