"""Checkpoint interop, CPU: the reference's checkpoint.pth
(tests/golden/checkpoint_ref.pth, written by the reference's own Trainer objects, see
make_golden.checkpoint_fixture, which also checks ours -> reference with the reference's
Trainer.resume) resumes into this framework bit-exactly; our checkpoints have the reference's
layout; Reporter, average_nbest_models, save_epoch and load_pretrained_model follow the
reference's semantics (cases modelled on test/espnet2/train/test_reporter.py and
test/espnet2/main_funcs/test_average_nbest_models.py)."""
import json
import os
import uuid

import numpy as np
import pytest
import torch

from tests.helpers import GOLDEN, build_model, small_cfg

REF_CKPT = os.path.join(GOLDEN, "checkpoint_ref.pth")


def _meta():
    with open(os.path.join(GOLDEN, "checkpoint_ref_meta.json")) as f:
        return json.load(f)


def _ours(device="cpu", dropout=None):
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR
    from espnet_slurp_amd.train.reporter import Reporter
    m = _meta()["cfg"]
    model = build_model(small_cfg("latest", D=m["D"], blocks=m["blocks"], V=m["V"]), torch.device(device),
                        dropout=dropout)
    opt = FusedAdam(model.parameters(), model.flat, lr=0.002, betas=(0.9, 0.98), eps=1e-9, weight_decay=1e-6)
    sch = WarmupLR(opt, warmup_steps=10)
    return model, opt, sch, Reporter()


def test_resume_reference_checkpoint():
    from espnet_slurp_amd.train import checkpoint as CK
    meta = _meta()
    ref = CK.safe_load(REF_CKPT)
    model, opt, sch, rep = _ours()
    assert [n for n, _ in model.named_parameters()] == meta["param_names"]  # optimizer index order
    CK.resume(REF_CKPT, model, rep, [opt], [sch], None, ngpu=0)
    sd = model.state_dict()
    for k, v in ref["model"].items():
        assert torch.equal(sd[k], v), k
    params = dict(model.named_parameters())
    for i, name in enumerate(meta["param_names"]):
        st = ref["optimizers"][0]["state"][i]
        assert torch.equal(opt.exp_avg[slice(*_span(opt, params[name]))], st["exp_avg"].reshape(-1))
        assert torch.equal(opt.exp_avg_sq[slice(*_span(opt, params[name]))], st["exp_avg_sq"].reshape(-1))
    assert opt.n_steps == int(meta["adam_step"]) == 2
    assert opt.param_groups[0]["lr"] == meta["lr"]
    assert sch.last_epoch == meta["last_epoch"] and sch.state_dict() == ref["schedulers"][0]
    assert rep.get_epoch() == 1
    assert rep.get_value("train", "loss") == meta["train_loss"]
    assert rep.get_value("valid", "acc") == meta["valid_acc"]


def _span(opt, p):
    o, n = opt.flat.slots[id(p)]
    return o, o + n


def test_saved_checkpoint_has_reference_layout(tmp_path):
    """ours -> file: identical to the reference's file entry by entry (model tensors each in their
    own storage, Adam state / param_groups, WarmupLR state, reporter)."""
    from espnet_slurp_amd.train import checkpoint as CK
    ref = CK.safe_load(REF_CKPT)
    model, opt, sch, rep = _ours()
    CK.resume(REF_CKPT, model, rep, [opt], [sch], None)
    out = tmp_path / "checkpoint.pth"
    CK.save_checkpoint(out, model, rep, [opt], [sch])
    got = CK.safe_load(out)
    assert list(got) == list(ref) == ["model", "reporter", "optimizers", "schedulers", "scaler"]
    assert list(got["model"]) == list(ref["model"])
    for k, v in got["model"].items():
        assert torch.equal(v, ref["model"][k]) and v.dtype == ref["model"][k].dtype, k
        assert v.untyped_storage().nbytes() == v.numel() * v.element_size(), k  # not the flat buffer
    go, ro = got["optimizers"][0], ref["optimizers"][0]
    assert go["param_groups"] == ro["param_groups"]
    assert sorted(go["state"]) == sorted(ro["state"])
    for i in ro["state"]:
        assert list(go["state"][i]) == list(ro["state"][i])
        for k, v in ro["state"][i].items():
            assert torch.equal(go["state"][i][k], v) and go["state"][i][k].dtype == v.dtype, (i, k)
    assert got["schedulers"] == ref["schedulers"]
    assert got["reporter"] == ref["reporter"]
    assert got["scaler"] is None


def test_fused_adam_state_loads_into_torch_adam():
    """Our optimizer state is a valid torch.optim.Adam state (the reference's optimizer class)."""
    from espnet_slurp_amd.train import checkpoint as CK
    model, opt, sch, rep = _ours()
    CK.resume(REF_CKPT, model, rep, [opt], [sch], None)
    tadam = torch.optim.Adam(model.parameters(), lr=1.0)
    tadam.load_state_dict(opt.state_dict())
    back = tadam.state_dict()
    mine = opt.state_dict()
    assert back["param_groups"] == mine["param_groups"]
    for i, st in mine["state"].items():
        for k in st:
            assert torch.equal(back["state"][i][k], st[k])
    # and FusedAdam refuses mismatching / per-parameter-step states
    bad = opt.state_dict()
    bad["state"][0]["step"] = torch.tensor(5.0)
    with pytest.raises(ValueError):
        opt.load_state_dict(bad)


# ------------------------------------------------------------------------------- Reporter
def _reporter_with(values, key="valid", key2="acc"):
    from espnet_slurp_amd.train.reporter import Reporter
    r = Reporter()
    for e, v in enumerate(values, start=1):
        r.set_epoch(e)
        with r.observe(key) as sub:
            sub.register({key2: v})
            sub.next()
    return r


@pytest.mark.parametrize("w1,w2", [(None, None), (19, np.array(9))])
def test_reporter_register_and_aggregate(w1, w2):
    from espnet_slurp_amd.train.reporter import Reporter
    r = Reporter()
    r.set_epoch(1)
    s1 = {"float": 0.6, "int": 6, "np": 0.25, "torch": torch.tensor([0.75])}
    s2 = {"float": 0.3, "int": 100, "np": 0.5, "torch": torch.tensor([0.125])}
    with r.observe("train") as sub:
        sub.register(s1, w1)
        sub.next()
        sub.register(s2, w2)
        sub.next()
    with pytest.raises(RuntimeError):
        sub.register({})
    for k in s1:
        a, b = float(s1[k]), float(s2[k])
        want = (a + b) / 2 if w1 is None else (float(w1) * a + float(w2) * b) / (float(w1) + float(w2))
        np.testing.assert_allclose(r.get_value("train", k), want)


def test_reporter_sort_best_early_stopping_state():
    from espnet_slurp_amd.train.reporter import Reporter
    r = _reporter_with([0.3, 0.5, 0.2])
    assert r.sort_epochs_and_values("valid", "acc", "min") == [(3, 0.2), (1, 0.3), (2, 0.5)]
    assert r.sort_epochs("valid", "acc", "max") == [2, 1, 3]
    assert r.get_best_epoch("valid", "acc", "max") == 2
    with pytest.raises(ValueError):
        r.sort_epochs_and_values("valid", "acc", "foo")
    with pytest.raises(KeyError):
        r.sort_epochs_and_values("valid", "nope", "min")
    assert r.check_early_stopping(0, "valid", "acc", "max")  # epoch 3 - best 2 > 0
    assert not r.check_early_stopping(1, "valid", "acc", "max")
    assert r.has("valid", "acc") and not r.has("train", "acc")
    r2 = Reporter()
    r2.load_state_dict(r.state_dict())
    assert r2.state_dict() == r.state_dict()
    assert "3epoch results: [valid] acc=0.200" in r.log_message()


def test_reporter_edge_cases():
    from espnet_slurp_amd.train.reporter import Average, Reporter, aggregate
    r = Reporter()
    with r.observe("train", 1) as sub:
        with pytest.raises(ValueError):
            sub.register({"a": np.array([0, 1])})
        with pytest.raises(ValueError):
            sub.register({"b": 1}, weight=np.array([1, 2]))
    with pytest.raises(RuntimeError):
        with r.observe("train", 2) as sub:
            sub.register({"time": 2})
    with pytest.raises(ValueError):  # mixed Average / WeightedAverage for one key
        with r.observe("train", 3) as sub:
            sub.register({"a": 2}, weight=1)
            sub.next()
            sub.register({"a": 3})
            sub.next()
    with pytest.raises(RuntimeError):
        with r.observe("train", 4):
            r.set_epoch(5)
    r = Reporter()
    with r.observe("train", 1) as sub:  # keys missing from a step are nan-filled
        sub.register({"a": 1.0})
        sub.next()
        sub.register({"b": 2.0})
        sub.next()
    assert r.get_value("train", "a") == 1.0 and r.get_value("train", "b") == 2.0
    assert r.get_value("train", "total_count") == 2
    assert aggregate([Average(0.1), Average(0.3)]) == pytest.approx(0.2)
    assert aggregate([]) is np.nan


# -------------------------------------------------------------------- model-file management
def _epoch_files(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    for e in (1, 2, 3):
        torch.manual_seed(e)
        m = torch.nn.Sequential(torch.nn.Conv2d(1, 1, 3), torch.nn.BatchNorm2d(1), torch.nn.Linear(1, 1))
        m[1].num_batches_tracked.fill_(e)
        torch.save(m.state_dict(), out / f"{e}epoch.pth")
    return out


@pytest.mark.parametrize("nbest", [0, 1, 2, 3, 4, [1, 2, 3, 5], []])
def test_average_nbest_models(tmp_path, nbest):
    from espnet_slurp_amd.train import checkpoint as CK
    out = _epoch_files(tmp_path)
    rep = _reporter_with([0.4, 0.5, 0.6])
    for _ in range(2):  # existing files / links are replaced
        CK.average_nbest_models(output_dir=out, reporter=rep, best_model_criterion=[("valid", "acc", "max")],
                                nbest=nbest)
    ns = [nbest] if isinstance(nbest, int) else (nbest or [1])
    _n = [i for i in ns if i <= 3] or [1]
    assert os.readlink(out / "valid.acc.ave.pth") == f"valid.acc.ave_{max(_n)}best.pth"
    for n in _n:
        if n == 1:
            assert os.readlink(out / "valid.acc.ave_1best.pth") == "3epoch.pth"
        elif n > 1:
            avg = torch.load(out / f"valid.acc.ave_{n}best.pth", weights_only=True)
            eps = [3, 2, 1][:n]
            src = [torch.load(out / f"{e}epoch.pth", weights_only=True) for e in eps]
            for k, v in avg.items():
                if k.endswith("num_batches_tracked"):  # integers are summed, not averaged
                    assert int(v) == sum(eps)
                else:
                    assert torch.allclose(v, sum(s[k] for s in src) / n)


def test_average_nbest_models_empty_reporter(tmp_path):
    from espnet_slurp_amd.train import checkpoint as CK
    from espnet_slurp_amd.train.reporter import Reporter
    out = _epoch_files(tmp_path)
    CK.average_nbest_models(output_dir=out, reporter=Reporter(), best_model_criterion=[("valid", "acc", "max")],
                            nbest=2)
    assert not list(out.glob("valid.*"))


def test_save_epoch_links_and_pruning(tmp_path):
    from espnet_slurp_amd.train import checkpoint as CK
    from espnet_slurp_amd.train.reporter import Reporter
    model = torch.nn.Linear(2, 2)
    rep = Reporter()
    out = tmp_path
    accs = [0.5, 0.7, 0.6, 0.4]
    for e, a in enumerate(accs, start=1):
        rep.set_epoch(e)
        with rep.observe("valid") as sub:
            sub.register({"acc": a})
            sub.next()
        improved = CK.save_epoch(out, e, model, rep, [("valid", "acc", "max")], keep_nbest_models=2)
        assert improved == (["valid.acc"] if e in (1, 2) else [])
        assert os.readlink(out / "latest.pth") == f"{e}epoch.pth"
    assert os.readlink(out / "valid.acc.best.pth") == "2epoch.pth"
    # n-best {2, 3} and the latest epoch survive
    assert sorted(p.name for p in out.glob("*epoch.pth")) == ["2epoch.pth", "3epoch.pth", "4epoch.pth"]


def test_load_pretrained_model_keys(tmp_path):
    from espnet_slurp_amd.train import checkpoint as CK
    src = torch.nn.ModuleDict({"encoder": torch.nn.Linear(3, 3), "decoder": torch.nn.Linear(3, 4)})
    path = tmp_path / "src.pth"
    torch.save(src.state_dict(), path)
    # whole model
    dst = torch.nn.ModuleDict({"encoder": torch.nn.Linear(3, 3), "decoder": torch.nn.Linear(3, 4)})
    CK.load_pretrained_model(str(path), dst, ignore_init_mismatch=False)
    assert torch.equal(dst["decoder"].weight, src["decoder"].weight)
    # src_key -> dst_key
    dst = torch.nn.ModuleDict({"enc2": torch.nn.Linear(3, 3)})
    CK.load_pretrained_model(f"{path}:encoder:enc2", dst, ignore_init_mismatch=False)
    assert torch.equal(dst["enc2"].weight, src["encoder"].weight)
    # excludes + size-mismatch filtering
    dst = torch.nn.ModuleDict({"encoder": torch.nn.Linear(3, 3), "decoder": torch.nn.Linear(3, 5)})
    before = dst["encoder"].weight.detach().clone()
    CK.load_pretrained_model(f"{path}:::encoder", dst, ignore_init_mismatch=True)
    assert torch.equal(dst["encoder"].weight, before)  # excluded
    with pytest.raises(RuntimeError):  # size mismatch without ignore_init_mismatch
        CK.load_pretrained_model(str(path), dst, ignore_init_mismatch=False)


def test_unique_key_registration():
    from espnet_slurp_amd.train.reporter import Reporter
    r = Reporter()
    r.set_epoch(1)
    key = uuid.uuid4().hex
    with r.observe(key) as sub:
        sub.register({"x": 1.0})
        with pytest.raises(RuntimeError):
            sub.register({"x": 2.0})
        sub.next()
    assert r.get_all_keys()[0] == (key, "x")


def test_trainer_run_no_forward_run_all_epochs(tmp_path):
    """no_forward_run (trainer.py:515-517, 530-532): every batch is passed over and the epoch counts
    as VALID (all_steps_are_invalid = False), so Trainer.run goes through every epoch instead of
    stopping after the first with 'gradients at all steps are invalid'; the reporter gets one
    iter_time entry per batch.  Host only: no forward runs."""
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions
    model, opt, sch, _ = _ours()
    tr = Trainer(model, opt, sch, TrainerOptions(no_forward_run=True, max_epoch=2, output_dir=str(tmp_path)))

    class _It:
        def build_iter(self, epoch, shuffle=None):
            return [([f"u{i}"], {}) for i in range(3)]

    rep = tr.run(_It(), _It())
    assert rep.get_epoch() == 2
    assert tr.n_updates == 0 and tr.n_skipped == 0
    assert (tmp_path / "2epoch.pth").exists()
