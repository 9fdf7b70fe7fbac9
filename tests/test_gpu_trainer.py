"""Trainer-step parity (VERDICT r1 'missing' 4 and 7; A1 and B5 of SURVEY.md §8):

* Trainer.train_one_step, eager and HIP-graph, against the reference's own two optimizer
  steps (tests/golden/train_step.npz: clip_grad_norm_(5) + Adam + WarmupLR(10),
  espnet2/train/trainer.py:594-690): loss, gradient norm, learning rate, final parameters.
* The reference's own loop shape on this model (trainer.py:554-690 with a plain
  torch.optim.Adam over model.parameters() and torch.nn.utils.clip_grad_norm_): the flat
  parameter / gradient views must behave like ordinary parameters, including
  optimizer.zero_grad()'s set_to_none."""
import numpy as np
import pytest
import torch

from oracle import espnet_cpu as O
from tests.helpers import build_model, golden, load_seeded, small_cfg

pytestmark = pytest.mark.gpu


def _setup(dev):
    cfg = small_cfg("latest", D=32, blocks=1, V=16)
    model = build_model(cfg, dev)
    load_seeded(model, cfg, 3)
    model.train()
    return cfg, model


def _batches(cfg, dev):
    out = []
    for step in range(2):
        speech, slen, text, tlen = O.synthetic_batch(2, 64, 80, cfg.vocab_size, [64, 50], [5, 3], 100 + step)
        out.append(dict(speech=speech.to(dev), speech_lengths=slen, text=text, text_lengths=tlen))
    return out


def _check_params(model, g):
    # Adam's first steps are sign-like (m/sqrt(v) ~ +-1): elements whose gradient is at fp32
    # noise level move by +-lr with an arbitrary sign (same criterion as the oracle pin,
    # tests/test_cpu.py::test_oracle_train_step_fixture)
    lr_sum = float(g["lr0"]) + float(g["lr1"])
    diffs = np.concatenate([np.abs(p.detach().cpu().numpy() - g["param/" + n]).ravel()
                            for n, p in model.named_parameters()])
    assert (diffs < 2e-6).mean() > 0.995, (diffs < 2e-6).mean()
    assert diffs.max() <= 2 * lr_sum + 1e-6


@pytest.mark.parametrize("graph", [False, True])
def test_trainer_two_steps_vs_reference(dev, graph):
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions
    g = golden("train_step")
    cfg, model = _setup(dev)
    opt = FusedAdam(model.parameters(), model.flat, lr=0.002, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-6)
    sch = WarmupLR(opt, warmup_steps=10)
    tr = Trainer(model, opt, sch, TrainerOptions(grad_clip=5.0), cuda_graph=graph)
    for step, b in enumerate(_batches(cfg, dev)):
        stats = tr.train_one_step(b)
        assert abs(stats["loss"].item() - float(g[f"loss{step}"])) < 1e-4
        assert abs(stats["grad_norm"].item() - float(g[f"gradnorm{step}"])) < 1e-4 * max(1.0, float(g[f"gradnorm{step}"]))
        # the lr this step used: the scheduler's batch step lands once the step's finite flag
        # is read (eager) / on device (graph)
        tr.resolve_pending()
        tr.sync_host_state()
        if step == 0:
            assert abs(opt.param_groups[0]["lr"] - float(g["lr1"])) < 1e-12
    tr.resolve_pending()
    tr.sync_host_state()
    assert opt.n_steps == 2 and sch.last_epoch == 2
    assert len(tr._graphs) == (1 if graph else 0)
    _check_params(model, g)


def test_reference_style_loop_on_flat_parameters(dev):
    """trainer.py:554-690 verbatim in shape: model(**batch) -> loss.backward() ->
    clip_grad_norm_(model.parameters()) -> torch.optim.Adam.step() -> WarmupLR.step() ->
    zero_grad() (set_to_none) — no FusedAdam, no Trainer."""
    from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR
    g = golden("train_step")
    cfg, model = _setup(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.002, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-6)
    sch = WarmupLR(opt, warmup_steps=10)
    for step, b in enumerate(_batches(cfg, dev)):
        assert abs(opt.param_groups[0]["lr"] - float(g[f"lr{step}"])) < 1e-12
        loss, stats, weight = model(**b)
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0, norm_type=2.0)
        assert abs(loss.item() - float(g[f"loss{step}"])) < 1e-4
        assert abs(gn.item() - float(g[f"gradnorm{step}"])) < 1e-4 * max(1.0, float(g[f"gradnorm{step}"]))
        opt.step()
        sch.step()
        opt.zero_grad()
        assert all(p.grad is None for p in model.parameters())
    _check_params(model, g)
    # the parameters are still views of the flat buffer the kernels read
    assert all(p.data_ptr() == model.flat.view(p).data_ptr() for p in model.parameters())


@pytest.mark.parametrize("graph", [False, True])
def test_trainer_amp_scaler_state(dev, graph):
    """use_amp's GradScaler state (trainer.py:181-195, 613-682): after every optimizer step the scale grows by
    growth_factor once growth_interval consecutive steps were finite and backs off (the step skipped) on a
    non-finite gradient norm -- the reference's scaler.update() sequence, here driven on device by the step's
    finite flag (eager and inside the captured step).  Its state_dict is torch's, so checkpoint.pth's
    "scaler" entry round-trips."""
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions
    cfg = small_cfg("latest")
    model = build_model(cfg, dev, dropout=0.0)
    load_seeded(model, cfg, 11)
    model.train()
    opt = FusedAdam(model.parameters(), model.flat, lr=1e-3)
    tr = Trainer(model, opt, None, TrainerOptions(grad_clip=5.0, use_amp=True), cuda_graph=graph)
    scaler = torch.amp.GradScaler("cuda", init_scale=1024.0, growth_interval=2)
    tr.set_scaler(scaler)
    speech, slen, text, tlen = O.synthetic_batch(3, 96, 80, 32, [96, 80, 71], [6, 5, 4], 12)
    good = dict(speech=speech.to(dev), speech_lengths=slen, text=text, text_lengths=tlen)
    finite = [True, True, False, True, True, True]
    want_scale, tracker = 1024.0, 0
    for step, ok in enumerate(finite):
        b = dict(good, speech=good["speech"].clone(), text=good["text"].clone())
        if not ok:
            b["speech"][0, 3, 5] = float("nan")
        tr.train_one_step(b)
        tr.resolve_pending()
        tr.sync_host_state()
        if ok:
            tracker += 1
            if tracker == 2:
                want_scale, tracker = want_scale * 2.0, 0
        else:
            want_scale, tracker = want_scale * 0.5, 0
        st = scaler.state_dict()
        assert st["scale"] == want_scale and st["_growth_tracker"] == tracker, (step, st)
    assert tr.n_skipped == 1 and tr.n_updates == len(finite)
    again = torch.amp.GradScaler("cuda")
    again.load_state_dict(scaler.state_dict())
    assert again.state_dict() == scaler.state_dict()
