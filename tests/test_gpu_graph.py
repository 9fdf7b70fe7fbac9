"""HIP-graph training step (Trainer(cuda_graph=True)): a captured + replayed step must do
exactly what the eager step does — same loss, same parameters after several optimizer steps —
and draw fresh dropout masks on every replay (device-resident dropout key)."""
import os

import pytest
import torch

from oracle import espnet_cpu as O
from tests.helpers import build_model, load_seeded, small_cfg

pytestmark = pytest.mark.gpu


def _trainer(dev, graph, dropout=0.0, seed=11, accum=1, lnorm=False, interctc=False, cond=False):
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions
    cfg = small_cfg("latest", blocks=3 if interctc else 2)
    cfg.length_normalized_loss = lnorm
    if interctc:
        cfg.enc.interctc_layer_idx = (1, 2)
        cfg.interctc_weight = 0.3
        cfg.enc.interctc_use_conditioning = cond
    model = build_model(cfg, dev, dropout=dropout)
    load_seeded(model, cfg, seed)
    model.train()
    opt = FusedAdam(model.parameters(), model.flat, lr=1e-3)
    sched = WarmupLR(opt, warmup_steps=10)
    return (Trainer(model, opt, sched, TrainerOptions(grad_clip=5.0, accum_grad=accum), cuda_graph=graph),
            model, opt, sched)


def _batch(dev):
    speech, slen, text, tlen = O.synthetic_batch(3, 96, 80, 32, [96, 80, 71], [6, 5, 4], 12)
    return dict(speech=speech.to(dev), speech_lengths=slen, text=text, text_lengths=tlen)


def test_graph_replay_matches_eager(dev):
    te, me, oe, se = _trainer(dev, False)
    tg, mg, og, sg = _trainer(dev, True)
    losses_e, losses_g = [], []
    for _ in range(4):
        losses_e.append(te.train_one_step(_batch(dev))["loss"].item())
        losses_g.append(tg.train_one_step(_batch(dev))["loss"].item())
    te.resolve_pending()
    tg.sync_host_state()
    assert len(tg._graphs) == 1
    for a, b in zip(losses_e, losses_g):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(a)), (losses_e, losses_g)
    assert torch.allclose(me.flat.flat, mg.flat.flat, rtol=0, atol=1e-6)
    assert og.n_steps == oe.n_steps == 4
    assert sg.last_epoch == se.last_epoch
    assert abs(og.param_groups[0]["lr"] - oe.param_groups[0]["lr"]) < 1e-12


def test_graph_new_batch_values_same_shapes(dev):
    """A replay re-targeted at another batch of the same shapes (new lengths / targets)."""
    te, me, _, _ = _trainer(dev, False)
    tg, mg, _, _ = _trainer(dev, True)
    b1 = _batch(dev)
    speech, slen, text, tlen = O.synthetic_batch(3, 96, 80, 32, [90, 96, 60], [6, 3, 5], 13)
    b2 = dict(speech=speech.to(dev), speech_lengths=slen, text=text, text_lengths=tlen)
    for b in (b1, b2, b1):
        # UtteranceMVN normalises the batch in place (utterance_mvn.py:66-69): fresh copies
        le = te.train_one_step(dict(b, speech=b["speech"].clone(), text=b["text"].clone()))["loss"].item()
        lg = tg.train_one_step(dict(b, speech=b["speech"].clone(), text=b["text"].clone()))["loss"].item()
        assert abs(le - lg) <= 1e-6 * max(1.0, abs(le)), (le, lg)
    assert len(tg._graphs) == 1


def test_graph_dropout_masks_fresh_and_reproducible(dev):
    runs = []
    for _ in range(2):
        torch.manual_seed(5)
        tg, _, _, _ = _trainer(dev, True, dropout=0.1)
        runs.append([tg.train_one_step(_batch(dev))["loss"].item() for _ in range(3)])
    assert runs[0] == runs[1]  # same CPU seed -> same device key sequence
    assert len(set(runs[0][1:])) == 2 or runs[0][1] != runs[0][2]


def test_graph_distributed_world1(dev):
    """The DDP graph path (replayed forward+backward, eager exchange + update) on a 1-rank RCCL
    group equals the single-GPU graph step."""
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
        from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR
        from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions
        cfg = small_cfg("latest")
        model = build_model(cfg, dev)
        load_seeded(model, cfg, 11)
        model.train()
        opt = FusedAdam(model.parameters(), model.flat, lr=1e-3)
        td = Trainer(model, opt, WarmupLR(opt, 10), TrainerOptions(grad_clip=5.0), distributed=True, cuda_graph=True)
        tg, mg, _, _ = _trainer(dev, True)
        for _ in range(3):
            a = td.train_one_step(_batch(dev))["loss"].item()
            b = tg.train_one_step(_batch(dev))["loss"].item()
            assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (a, b)
        assert torch.allclose(model.flat.flat, mg.flat.flat, rtol=0, atol=1e-5)
    finally:
        dist.destroy_process_group()


def test_eager_distributed_world1_rccl(dev):
    """The eager DDP path on a 1-rank RCCL ("nccl") group: the bucket hooks launch
    ReduceOp.AVG all-reduces (the branch the gloo tests cannot reach, distributed.py) while the
    explicit backward runs; the steps equal the single-GPU eager steps."""
    import socket

    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
        from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR
        from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions
        cfg = small_cfg("latest")
        model = build_model(cfg, dev)
        load_seeded(model, cfg, 11)
        model.train()
        opt = FusedAdam(model.parameters(), model.flat, lr=1e-3)
        td = Trainer(model, opt, WarmupLR(opt, 10), TrainerOptions(grad_clip=5.0), distributed=True,
                     bucket_mb=0.02)
        assert td.reducer is not None and td.reducer.backend == "nccl" and len(td.reducer.buckets) > 2
        te, me, _, _ = _trainer(dev, False)
        for _ in range(3):
            a = td.train_one_step(_batch(dev))["loss"].item()
            b = te.train_one_step(_batch(dev))["loss"].item()
            assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (a, b)
        td.resolve_pending()
        te.resolve_pending()
        assert torch.allclose(model.flat.flat, me.flat.flat, rtol=0, atol=1e-6)
    finally:
        dist.destroy_process_group()


def _batches_same_shapes(dev):
    """Two batches with identical padded shapes but different lengths / target counts."""
    out = []
    for lens, ulens, seed in (([96, 80, 71], [6, 5, 4], 12), ([90, 96, 60], [6, 2, 1], 13)):
        speech, slen, text, tlen = O.synthetic_batch(3, 96, 80, 32, lens, ulens, seed)
        out.append(dict(speech=speech.to(dev), speech_lengths=slen, text=text, text_lengths=tlen))
    return out


def _copy(b):
    return dict(b, speech=b["speech"].clone(), text=b["text"].clone())


def test_graph_length_normalized_loss_not_baked(dev):
    """length_normalized_loss: the denominator (non-ignored targets) differs between two
    batches of the same shapes; the replayed graph must use the new batch's count."""
    te, me, _, _ = _trainer(dev, False, lnorm=True)
    tg, mg, _, _ = _trainer(dev, True, lnorm=True)
    b1, b2 = _batches_same_shapes(dev)
    for b in (b1, b2, b1, b2):
        le = te.train_one_step(_copy(b))["loss"].item()
        lg = tg.train_one_step(_copy(b))["loss"].item()
        assert abs(le - lg) <= 1e-6 * max(1.0, abs(le)), (le, lg)
    te.resolve_pending()
    assert len(tg._graphs) == 1
    assert torch.allclose(me.flat.flat, mg.flat.flat, rtol=0, atol=1e-6)


def test_graph_accum_grad_matches_eager(dev):
    """accum_grad=2 in graph mode (a micro-batch graph and an update graph) equals eager."""
    te, me, oe, _ = _trainer(dev, False, accum=2)
    tg, mg, og, _ = _trainer(dev, True, accum=2)
    b1, b2 = _batches_same_shapes(dev)
    for b in (b1, b2, b2, b1, b1, b2):
        le = te.train_one_step(_copy(b))["loss"].item()
        lg = tg.train_one_step(_copy(b))["loss"].item()
        assert abs(le - lg) <= 1e-6 * max(1.0, abs(le)), (le, lg)
    te.resolve_pending()
    tg.sync_host_state()
    assert len(tg._graphs) == 2
    assert og.n_steps == oe.n_steps == 3 and tg.n_updates == te.n_updates == 3
    assert torch.allclose(me.flat.flat, mg.flat.flat, rtol=0, atol=1e-6)


def test_skipped_steps_counted_in_graph_mode(dev):
    """A non-finite gradient norm skips the update on device; the trainer counts it
    (all_steps_are_invalid of trainer.py:436-440) in graph and eager mode alike."""
    for graph in (False, True):
        t, m, o, _ = _trainer(dev, graph)
        b = _batches_same_shapes(dev)[0]
        t.train_one_step(_copy(b))
        bad = _copy(b)
        bad["speech"][0, 0, 0] = float("inf")
        t.train_one_step(bad)
        t.resolve_pending()
        t.sync_host_state()
        assert t.n_updates == 2 and t.n_skipped == 1, (graph, t.n_updates, t.n_skipped)
        assert o.n_steps == 1
        assert t.train_one_epoch([(None, bad)]) is True
        assert t.train_one_epoch([(None, _copy(b))]) is False


@pytest.mark.parametrize("dp,cond", [(False, False), (True, False), (False, True), (True, True)])
def test_graph_interctc_matches_eager(dev, dp, cond):
    """Intermediate CTC (ConformerEncoder interctc_layer_idx, interctc_weight) under the HIP graph, plain and
    through the data-parallel segmented capture on a 1-rank RCCL group (the module-done hooks of ctc /
    after_norm wait for the intermediate branches): losses, the per-layer loss_interctc stats and the
    parameters after 3 steps equal the eager steps'."""
    import torch.distributed as dist
    if dp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29573")
        dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        te, me, _, _ = _trainer(dev, False, interctc=True, cond=cond)
        tg, mg, _, _ = _trainer(dev, True, interctc=True, cond=cond)
        if dp:
            from espnet_slurp_amd.train.trainer import Trainer
            tg = Trainer(mg, tg.optimizer, tg.scheduler, tg.options, distributed=True, cuda_graph=True)
        for _ in range(3):
            se = te.train_one_step(_batch(dev))
            sg = tg.train_one_step(_batch(dev))
            for k in ("loss", "loss_ctc", "loss_interctc_layer1", "loss_interctc_layer2"):
                a, b = se[k].item(), sg[k].item()
                assert abs(a - b) <= (1e-5 if dp else 1e-6) * max(1.0, abs(a)), (k, a, b)
        te.resolve_pending()
        tg.sync_host_state()
        assert torch.allclose(me.flat.flat, mg.flat.flat, rtol=0, atol=1e-5 if dp else 1e-6)
    finally:
        if dp:
            dist.destroy_process_group()
