"""Graph vs eager trainer losses / grad norms / parameter finiteness at a given model shape
(diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import argparse  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
from espnet_slurp_amd.optimizers.fused_adam import FusedAdam  # noqa: E402
from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR  # noqa: E402
from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions  # noqa: E402


def main():
    a = argparse.Namespace(d=int(sys.argv[1]), heads=int(sys.argv[2]), ff=int(sys.argv[3]), layers=12, vocab=600,
                           rel_pos="latest", batch=int(sys.argv[4]), amp=False)
    graph = sys.argv[5] == "graph"
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = bench.build(a, dev)
    model.train()
    opt = FusedAdam(model.parameters(), model.flat, lr=2e-4)
    tr = Trainer(model, opt, WarmupLR(opt, 25000), TrainerOptions(grad_clip=5.0), cuda_graph=graph)
    batch = bench.synthetic_batch(a.batch, a.vocab, 0, dev)
    for i in range(3):
        st = tr.train_one_step(batch)
        torch.cuda.synchronize()
        fin = bool(torch.isfinite(model.flat.flat).all())
        print(f"{'graph' if graph else 'eager'} step {i} loss {st['loss'].item():.5f} grad_norm "
              f"{st['grad_norm'].item():.4f} params finite {fin} "
              f"hs? stats {[(k, round(v.item(), 4)) for k, v in st.items() if k not in ('loss', 'grad_norm')]}",
              flush=True)


if __name__ == "__main__":
    main()
