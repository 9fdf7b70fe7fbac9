"""Per-parameter differences between the eager trainer (unpadded) and the bucketed graph
trainer over the steps of tests/test_gpu_buckets.py (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests.test_gpu_buckets import _batch, _copy, _trainer  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    te, me = _trainer(dev, False)
    tg, mg = _trainer(dev, True, buckets=(64, 8))
    batches = [
        _batch(dev, 112, [112, 90, 71], [6, 5, 4], 21),
        _batch(dev, 97, [97, 97, 97], [7, 3, 5], 22),
        _batch(dev, 80, [80, 66, 79], [2, 8, 1], 23),
        _batch(dev, 150, [150, 131, 140], [9, 4, 6], 24),
        _batch(dev, 120, [100, 120, 77], [3, 3, 3], 25),
    ]
    for i, b in enumerate(batches):
        torch.manual_seed(100 + i)
        le = te.train_one_step(_copy(b))["loss"].item()
        torch.manual_seed(100 + i)
        lg = tg.train_one_step(_copy(b))["loss"].item()
        te.resolve_pending()
        tg.sync_host_state()
        torch.cuda.synchronize()
        print(f"step {i} loss {le:.7f} {lg:.7f} lr {te.optimizer.param_groups[0]['lr']:.3e} "
              f"{tg.optimizer.param_groups[0]['lr']:.3e}", flush=True)
        for (n, p1), (_, p2) in zip(me.named_parameters(), mg.named_parameters()):
            d = (p1 - p2).abs().max().item()
            if d > 1e-6:
                print(f"  {n:60s} diff {d:.3e}")
        for (n, b1), (_, b2) in zip(me.named_buffers(), mg.named_buffers()):
            d = (b1.double() - b2.double()).abs().max().item()
            if d > 1e-6:
                print(f"  buffer {n:53s} diff {d:.3e}")


if __name__ == "__main__":
    main()
