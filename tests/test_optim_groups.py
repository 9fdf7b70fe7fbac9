"""FusedAdam beyond the espnet2 default (VERDICT r4 missing 3): several param groups and amsgrad, as
torch.optim.Adam takes them from optim_conf (espnet2/tasks/abs_task.py:856-880).  Host logic only here:
which runs of the flat buffer each group's launches cover, and the checkpoint format against
torch.optim.Adam's own state_dict (the GPU step is tests/test_gpu_optim.py)."""
import torch
from torch import nn

from espnet_slurp_amd.flat import FlatParams
from espnet_slurp_amd.optimizers.fused_adam import FusedAdam


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(5, 7), nn.LayerNorm(7), nn.Linear(7, 3), nn.Linear(3, 9))


def _groups(model):
    decay = [p for p in model.parameters() if p.dim() == 2]
    rest = [p for p in model.parameters() if p.dim() != 2]
    return [{"params": decay, "weight_decay": 0.01}, {"params": rest, "weight_decay": 0.0, "amsgrad": True, "lr": 5e-4}]


def test_single_group_is_one_run_over_the_buffer():
    model = _model()
    flat = FlatParams(model, "cpu")
    opt = FusedAdam(model.parameters(), flat, lr=1e-3)
    assert opt.group_ranges() == [[(0, flat.flat.numel())]]
    assert opt.max_exp_avg_sq is None


def test_group_runs_cover_exactly_their_parameters():
    model = _model()
    flat = FlatParams(model, "cpu")
    opt = FusedAdam(_groups(model), flat, lr=1e-3)
    runs = opt.group_ranges()
    assert opt.max_exp_avg_sq is not None and opt.max_exp_avg_sq.numel() == flat.flat.numel()
    for gi, g in enumerate(opt.param_groups):
        mine = [flat.slots[id(p)] for p in g["params"]]
        others = [flat.slots[id(p)] for h, og in enumerate(opt.param_groups) if h != gi for p in og["params"]]
        for o, k in mine:  # every element of the group's parameters is in one of its runs
            assert sum(1 for (ro, rk) in runs[gi] if ro <= o and o + k <= ro + rk) == 1
        for ro, rk in runs[gi]:  # no run touches another group's parameter
            assert all(o + k <= ro or ro + rk <= o for o, k in others)
    # flat order L1.w L1.b LN.w LN.b L2.w L2.b L3.w L3.b: the weights one run each, the rest three runs
    # (L1.b + LN.w + LN.b adjacent)
    assert len(runs[0]) == 3 and len(runs[1]) == 3


def test_state_dict_matches_torch_adam_with_groups_and_amsgrad():
    model = _model()
    flat = FlatParams(model, "cpu")
    opt = FusedAdam(_groups(model), flat, lr=1e-3, betas=(0.9, 0.98), eps=1e-9)
    g = torch.Generator().manual_seed(1)
    for buf in (opt.exp_avg, opt.exp_avg_sq, opt.max_exp_avg_sq):
        buf.copy_(torch.rand(buf.numel(), generator=g))
    opt.n_steps = 3
    mine = opt.state_dict()
    assert [len(x["params"]) for x in mine["param_groups"]] == [3, 5]
    assert [x["amsgrad"] for x in mine["param_groups"]] == [False, True]
    assert all(("max_exp_avg_sq" in mine["state"][i]) == (i >= 3) for i in range(8))
    tadam = torch.optim.Adam(_groups(model), lr=1.0)
    tadam.load_state_dict(mine)
    back = tadam.state_dict()
    assert back["param_groups"] == mine["param_groups"]
    for i, st in mine["state"].items():
        assert set(back["state"][i]) == set(st)
        for k in st:
            assert torch.equal(back["state"][i][k], st[k])
    # and back into a fresh FusedAdam built with amsgrad off: the checkpoint turns it on for group 1
    model2 = _model()
    flat2 = FlatParams(model2, "cpu")
    opt2 = FusedAdam(_groups(model2)[:1] + [{"params": _groups(model2)[1]["params"]}], flat2, lr=1e-3)
    assert opt2.max_exp_avg_sq is None
    opt2.load_state_dict(back)
    assert opt2.n_steps == 3 and [x["amsgrad"] for x in opt2.param_groups] == [False, True]
    for gi in range(2):
        for p, q in zip(opt.param_groups[gi]["params"], opt2.param_groups[gi]["params"]):
            o, k = flat.slots[id(p)]
            o2, k2 = flat2.slots[id(q)]
            bufs = [(opt.exp_avg, opt2.exp_avg), (opt.exp_avg_sq, opt2.exp_avg_sq)]
            if gi == 1:
                bufs.append((opt.max_exp_avg_sq, opt2.max_exp_avg_sq))
            for a, b in bufs:
                assert torch.equal(a[o:o + k], b[o2:o2 + k2])
