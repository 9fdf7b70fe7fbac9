"""Multi-rank training step (VERDICT r1 'missing' 2; C3 readiness; A22): two data-parallel
ranks (child processes sharing cuda:0, gloo) run Trainer(distributed=True) in the eager
(module-done bucket hooks) and HIP-graph (prescale w_r / sum w + SUM all-reduce) paths, with
accum_grad 1 and 2.  The result must equal the reference's DDP semantics restated by the
fp64 oracle: per micro-batch loss = sum_r w_r loss_r / sum w (trainer.py:594-608, DDP's
average over ranks undoes the x world_size), BatchNorm statistics per replica, gradients
accumulated over accum_grad micro-batches, then clip_grad_norm_(5) + Adam + WarmupLR; the
reported stats are recursive_average's weighted means (recursive_op.py:8-47)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import espnet_cpu as O
from tests.helpers import golden, grad_gate, loss_gate, small_cfg

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dist_worker as W  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(tmp_path, mode, accum, world=2, extra=()):
    port = _free_port()
    procs, outs = [], []
    for r in range(world):
        out = str(tmp_path / f"{mode}_{accum}_r{r}.pt")
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PYTHONPATH=ROOT)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "dist_worker.py"), out, mode,
                                       str(accum), *extra], env=env, cwd=ROOT))
        outs.append(out)
    for p in procs:
        assert p.wait(timeout=240) == 0
    return [torch.load(o, weights_only=True) for o in outs]


def _oracle(accum, world=2):
    cfg = small_cfg("latest")
    P = {k: v.clone().double().requires_grad_(v.is_floating_point() and "running" not in k)
         for k, v in O.deterministic_params(cfg, 11).items()}
    names = [k for k in P if P[k].requires_grad]
    params = [P[k] for k in names]
    opt = torch.optim.Adam(params, lr=2e-3, weight_decay=1e-6)
    bn = [dict() for _ in range(world)]  # per-replica BatchNorm running statistics
    stats = []
    n_up = 0
    for step in range(len(W.GLOBAL)):
        tot, ws, st = 0.0, 0.0, {}
        for r in range(world):
            speech, slen, text, tlen = W.shard(step, r, world)
            loss, s, w = O.asr_forward(P, speech.double(), slen, text, tlen, cfg, bn_state=bn[r])
            w = float(w)
            tot = tot + loss * w
            ws += w
            for k, v in s.items():
                if v is not None:
                    st[k] = st.get(k, 0.0) + float(v) * w
        stats.append({k: v / ws for k, v in st.items()})
        (tot / ws / accum).backward()
        if (step + 1) % accum == 0:
            n_up += 1
            lr = 2e-3 * 10 ** 0.5 * min(n_up ** -0.5, n_up * 10 ** -1.5)
            for gr in opt.param_groups:
                gr["lr"] = lr
            torch.nn.utils.clip_grad_norm_(params, 5.0)
            opt.step()
            opt.zero_grad()
    return {k: P[k].detach() for k in names}, stats, bn[0]


@pytest.mark.parametrize("mode,accum", [("eager", 1), ("graph", 1), ("eager", 2), ("graph", 2)])
def test_two_rank_training_matches_ddp_oracle(dev, tmp_path, mode, accum):
    res = _run_ranks(tmp_path, mode, accum)
    ref, ref_stats, ref_bn = _oracle(accum)
    for r in res:
        assert r["n_updates"] == len(W.GLOBAL) // accum and r["n_steps"] == len(W.GLOBAL) // accum
    # replicas stay bit-identical (same averaged gradient, same update)
    for n in res[0]["params"]:
        assert torch.equal(res[0]["params"][n], res[1]["params"][n]), n
    # parameters vs the fp64 DDP oracle (Adam's sign-like first steps: see test_gpu_trainer)
    diffs = np.concatenate([np.abs(res[0]["params"][n].double().numpy() - ref[n].numpy()).ravel() for n in ref])
    assert (diffs < 5e-6).mean() > 0.995, (diffs < 5e-6).mean()
    # the elements that differ are Adam's sign-like updates of near-zero gradients: each
    # update moves an element by about lr (exactly lr at step 1), so two trajectories that
    # disagree on a sign differ by at most ~2 x the summed learning rates of the updates
    lrs = [2e-3 * 10 ** 0.5 * min(n ** -0.5, n * 10 ** -1.5) for n in range(1, len(W.GLOBAL) // accum + 1)]
    print(f"max |param - oracle| {diffs.max():.3g}, sign-flip bound {2 * sum(lrs):.3g}")
    assert diffs.max() <= 2 * sum(lrs), (diffs.max(), 2 * sum(lrs))
    # recursive_average: the same weighted stats on every rank
    for a, b, o in zip(res[0]["stats"], res[1]["stats"], ref_stats):
        for k in ("loss", "loss_ctc", "loss_att", "acc"):
            assert a[k] == b[k], k
            assert abs(a[k] - o[k]) <= 1e-4 * max(1.0, abs(o[k])), (k, a[k], o[k])
    # DDP broadcast_buffers: rank 0 is the source, so its BatchNorm running statistics are
    # exactly its own replica's chain (rank 1 starts every forward from rank 0's copy).  They are
    # statistics of activations under the updated parameters, which the gate above lets differ
    # from the oracle's in a few sign-like Adam updates: fp32 atol 1e-4 (north star) here.
    for n, b in res[0]["bufs"].items():
        if "running" in n:
            r = ref_bn[n].double().numpy()
            assert np.abs(b.double().numpy() - r).max() < 1e-4 * max(1.0, np.abs(r).max()), n
    if mode == "graph":
        assert res[0]["graphs"] == accum  # one step graph (accum 2: micro-batch + update)
        # the backward was captured in segments: bucket all-reduces overlap the later segments
        assert res[0]["buckets"] > 2 and res[0]["segments"] > 2, (res[0]["buckets"], res[0]["segments"])


class _Grads:
    """named_parameters() over saved gradients, for helpers.grad_gate."""

    def __init__(self, grads):
        self.g = grads

    def named_parameters(self):
        for n, v in self.g.items():
            yield n, type("P", (), {"grad": v})()


class _SavedFlips:
    def __init__(self, dec):
        self.dec = dec

    def decisions(self, site, idx):
        d = self.dec[site].numpy()
        assert len(d) == len(idx), site
        return d


@pytest.mark.parametrize("mode", ["eager", "graph"])
def test_two_rank_c2_shape_ddp_step(dev, tmp_path, mode):
    """C3's model shape under DDP (VERDICT r3 'next' 1b): the C2 Conformer (d=256, 12 blocks, T up to
    1500) on two data-parallel ranks (gloo, sharing cuda:0; the RCCL path is the same Trainer code at
    N>1), a 5-utterance global batch sharded 3 / 2.  Against the reference's own DDP step on two
    replicas (tests/golden/ddp_c2.npz, make_ddp_fixture.py): the all-reduced gradient the optimizer
    sees -- per-tensor norm and slice within max(1e-4, 2 e_ref) (the full-size gate, ReLU decisions
    near 0 set to the fp64 ones per rank) -- and the recursive_average stats (loss, loss_ctc, loss_att,
    acc) on both ranks, in the eager (bucket hooks) and HIP-graph (prescaled segments + SUM) paths;
    the second step (a graph replay) repeats the first (lr 0)."""
    g = golden("ddp_c2")
    res = _run_ranks(tmp_path, mode, 1, extra=("c2",))
    for n in res[0]["grads"]:
        assert torch.equal(res[0]["grads"][n], res[1]["grads"][n]), n
    dec = dict(res[0]["dec"])
    dec.update(res[1]["dec"])
    bad = grad_gate(_Grads(res[0]["grads"]), g, flips=_SavedFlips(dec))
    assert not bad, bad
    for r in res:
        for st in r["stats"]:
            for key, slack in (("loss", 0.0), ("loss_att", 0.0), ("loss_ctc", 0.0)):
                ok, info = loss_gate(st[key], g, key, slack)
                assert ok, info
            assert abs(st["acc"] - float(g["acc_f64"])) < 1e-6
        assert r["stats"][0] == r["stats"][1]
    if mode == "graph":
        assert res[0]["graphs"] == 1 and res[0]["segments"] >= 2
