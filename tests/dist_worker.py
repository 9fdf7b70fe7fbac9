"""One data-parallel rank of tests/test_gpu_distributed.py (run as a child process).

    python tests/dist_worker.py <out.pt> <eager|graph> <accum_grad> [c2]   (RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT from the environment; c2: the C2-shape DDP step of main_c2)

Every rank shares cuda:0 and talks over gloo (RCCL refuses two ranks on one GPU); the
trainer code path is the multi-GPU one (bucket hooks / prescale + SUM, fused stats)."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import espnet_cpu as O  # noqa: E402
from tests.helpers import build_model, load_seeded, small_cfg  # noqa: E402

# global batch per micro-step: utterance lengths / label lengths, split batch[rank::world]
# (abs_task.py:1542) -> unequal shard sizes 3 / 2, so the w_r / sum w weighting matters
# (each rank's padded label length stays 6 / 5 across steps, so graph mode replays)
GLOBAL = [([96, 90, 84, 80, 71], [6, 5, 5, 4, 3]), ([96, 93, 77, 70, 66], [6, 5, 2, 5, 3]),
          ([96, 95, 90, 85, 60], [5, 5, 6, 2, 4]), ([96, 81, 80, 79, 78], [6, 4, 5, 5, 6])]


def shard(step, rank, world):
    lens, ulens = GLOBAL[step]
    speech, slen, text, tlen = O.synthetic_batch(len(lens), 96, 80, 32, lens, ulens, 500 + step)
    idx = list(range(rank, len(lens), world))
    t = text[idx][:, : int(tlen[idx].max())]
    return speech[idx], slen[idx], t, tlen[idx]


def c2_shard(g, rank, world):
    """tests/golden/make_ddp_fixture.shard: batch[rank::world] of the fixture's global batch, padded
    to the shard's own longest utterance / label."""
    lens, ulens = [int(x) for x in g["lens"]], [int(x) for x in g["ulens"]]
    speech, slen, text, tlen = O.synthetic_batch(len(lens), max(lens), 80, 600, lens, ulens, int(g["seed"]) + 1)
    idx = list(range(rank, len(lens), world))
    T, U = int(slen[idx].max()), int(tlen[idx].max())
    return speech[idx][:, :T].contiguous(), slen[idx], text[idx][:, :U].contiguous(), tlen[idx]


def main_c2(out, mode, rank, world):
    """C3's model shape (the C2 Conformer: d=256, 12 blocks, T up to 1500) under DDP, 2 steps of the
    same shard with lr 0 (the HIP-graph path captures, then replays): the all-reduced gradient as
    the optimizer step sees it (before clipping), the recursive_average stats, and this rank's ReLU
    decisions at the fixture's flip sites (tests/golden/ddp_c2.npz, make_ddp_fixture.py)."""
    import numpy as np
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.train import trainer as TR
    from tests.helpers import FlipProbe, c2_cfg, golden
    g = golden("ddp_c2")
    dev = torch.device("cuda:0")
    cfg = c2_cfg("latest")
    model = build_model(cfg, dev)
    load_seeded(model, cfg, int(g["seed"]))
    model.train()
    opt = FusedAdam(model.parameters(), model.flat, lr=0.0)
    tr = TR.Trainer(model, opt, None, TR.TrainerOptions(grad_clip=5.0), distributed=True,
                    cuda_graph=(mode == "graph"))
    snap = torch.zeros_like(model.flat.grad)
    clip0 = TR.clip_grad_norm_

    def clip(flat, *a, **k):  # the reduced gradient, stream-ordered (captured in graph mode)
        snap.copy_(flat.grad)
        return clip0(flat, *a, **k)
    TR.clip_grad_norm_ = clip
    speech, slen, text, tlen = c2_shard(g, rank, world)
    stats = []
    with FlipProbe(model) as fp:
        for _ in range(2):
            st = tr.train_one_step(dict(speech=speech.to(dev), speech_lengths=slen, text=text.clone(),
                                        text_lengths=tlen))
            stats.append({k: float(v) for k, v in st.items() if k != "grad_norm"})
    tr.resolve_pending()
    torch.cuda.synchronize()
    TR.clip_grad_norm_ = clip0
    pre = f"r{rank}:"
    dec = {}
    for k in g:
        if k.startswith("flip/") and k.endswith("/idx"):
            site = k.split("/")[-2]
            if site.startswith(pre) and site not in dec:
                dec[site] = torch.from_numpy(fp.decisions(site[len(pre):], g[k]).astype(np.int8))
    grads = {n: snap[model.flat.slots[id(p)][0]:model.flat.slots[id(p)][0] + p.numel()].view(p.shape).cpu()
             for n, p in model.named_parameters()}
    torch.save({"grads": grads, "stats": stats, "dec": dec, "graphs": len(tr._graphs),
                "segments": max([len(e.segs) for e in tr._graphs.values()], default=0)}, out)
    dist.barrier()
    dist.destroy_process_group()


def main():
    import faulthandler
    faulthandler.dump_traceback_later(90, exit=True)  # a hung rank prints every thread's stack and exits
    out, mode, accum = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if len(sys.argv) > 4 and sys.argv[4] == "c2":
        return main_c2(out, mode, rank, world)
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions
    dev = torch.device("cuda:0")
    cfg = small_cfg("latest")
    model = build_model(cfg, dev)
    load_seeded(model, cfg, 11)
    model.train()
    opt = FusedAdam(model.parameters(), model.flat, lr=2e-3, weight_decay=1e-6)
    sch = WarmupLR(opt, warmup_steps=10)
    # small buckets (~20 KB): the model's gradient spans several, so the graph path's backward
    # is captured in several segments with bucket all-reduces between them
    tr = Trainer(model, opt, sch, TrainerOptions(grad_clip=5.0, accum_grad=accum), distributed=True,
                 cuda_graph=(mode == "graph"), bucket_mb=0.02)
    stats = []
    for step in range(len(GLOBAL)):
        speech, slen, text, tlen = shard(step, rank, world)
        st = tr.train_one_step(dict(speech=speech.to(dev), speech_lengths=slen, text=text, text_lengths=tlen))
        stats.append({k: float(v) for k, v in st.items() if k != "grad_norm"})
    tr.resolve_pending()
    tr.sync_host_state()
    torch.cuda.synchronize()
    torch.save({"params": {n: p.detach().cpu() for n, p in model.named_parameters()},
                "bufs": {n: b.detach().cpu() for n, b in model.named_buffers()},
                "stats": stats, "n_steps": opt.n_steps, "n_updates": tr.n_updates,
                "graphs": len(tr._graphs), "buckets": len(tr.reducer.buckets),
                "segments": max([len(e.segs) for e in tr._graphs.values()], default=0)}, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
