"""Data-parallel fixture at the C2 model shape (VERDICT r3 'next' 1b):

    python tests/golden/make_ddp_fixture.py        # writes tests/golden/ddp_c2.npz

The reference's DDP training step (espnet2/train/trainer.py:594-621 + DDP's gradient average,
abs_task.py:1542's batch[rank::world] sharding) on two replicas of the C2 Conformer (d=256, H=4,
FF 1024, 12 blocks, latest rel-pos; decoder 6 x FF 2048; V=600; dropout 0), restated with the
REFERENCE modules themselves (one ESPnetASRModel per rank, same parameters): a global batch of 5
utterances (T up to 1500) sharded 3 / 2, per-rank loss weighted by its batch size,
loss = sum_r w_r loss_r / sum_r w (what DDP's average of world * w_r / sum w * loss_r yields), one
backward over both replicas -> the averaged gradient.  fp32 AND fp64; stored in the format of
make_golden.fullsize_train_fixture (loss and stats as recursive_average's weighted means,
per-tensor gradient norms, slices and fingerprints) plus each rank's ReLU flip records ("r0:", "r1:" site
prefixes, flipfix.py).  Read by tests/test_gpu_distributed.py::test_two_rank_c2_shape_ddp_step.
Test infrastructure only.
"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as G  # noqa: E402  (sets up the reference import)
import fingerprint as FP  # noqa: E402
import flipfix  # noqa: E402
from oracle import espnet_cpu as O  # noqa: E402

LENS = [1500, 1480, 1410, 1350, 1290]
ULENS = [40, 33, 29, 25, 21]
SEED = 81
WORLD = 2


def shard(rank, world=WORLD):
    """The rank's utterances (batch[rank::world]), padded to the shard's own longest (the collate)."""
    speech, slen, text, tlen = O.synthetic_batch(len(LENS), max(LENS), 80, 600, LENS, ULENS, SEED + 1)
    idx = list(range(rank, len(LENS), world))
    T = int(slen[idx].max())
    U = int(tlen[idx].max())
    return speech[idx][:, :T].contiguous(), slen[idx], text[idx][:, :U].contiguous(), tlen[idx]


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    cfg = G.c2_cfg("latest")
    out = {}
    recs = {}
    rows = {}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        t0 = time.time()
        models, losses, ws, stats = [], [], [], {}
        for r in range(WORLD):
            m = G.build_reference(cfg).to(dt)
            G.load_params(m, cfg, SEED, dt)
            m.train()
            speech, slen, text, tlen = shard(r)
            with flipfix.ReferenceProbe(m) as probe:
                loss, st, w = m(speech.to(dt), slen, text, tlen)
            recs[(tag, r)] = probe
            models.append(m)
            losses.append(loss)
            ws.append(float(w))
            for k, v in st.items():
                if v is not None and k in ("loss", "loss_ctc", "loss_att", "acc"):
                    stats[k] = stats.get(k, 0.0) + float(v) * float(w)
        wsum = sum(ws)
        total = sum(l * w for l, w in zip(losses, ws)) / wsum
        total.backward()
        for r in range(WORLD):
            recs[(tag, r)] = recs[(tag, r)].rec.detach()
        # the averaged gradient: one replica's parameters receive their own rank's share; sum them
        for (n, p0), (_, p1) in zip(models[0].named_parameters(), models[1].named_parameters()):
            p0.grad = p0.grad + p1.grad
        G.grad_summary(models[0], tag, out, rows)
        shapes = {n: p.numel() for n, p in models[0].named_parameters()}
        out[f"loss_{tag}"] = np.float64(total.item())
        for k, v in stats.items():
            out[f"{k}_{tag}"] = np.float64(v / wsum)
        print(f"ddp {tag}: loss {total.item():.8f} ({time.time() - t0:.1f} s)", flush=True)
        del models, losses, total
    FP.finish_rows(out, rows)
    gs32 = {k[len("gs_f32/"):]: v for k, v in out.items() if k.startswith("gs_f32/")}
    corr, corr_fp = {}, {}
    for r in range(WORLD):
        flipfix.flip_records(recs[("f64", r)], recs[("f32", r)], lambda n: out["gidx/" + n], out, gs32,
                             log=lambda m: print(f"rank {r}: {m}", flush=True), prefix=f"r{r}:", corr=corr,
                             shapes=shapes, corr_fp=corr_fp)
    out.update(lens=np.array(LENS), ulens=np.array(ULENS), seed=np.int64(SEED), world=np.int64(WORLD))
    path = os.path.join(HERE, "ddp_c2.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, flush=True)


if __name__ == "__main__":
    main()
