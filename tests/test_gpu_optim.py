"""FusedAdam's GPU step with several param groups and amsgrad (esp_adam / esp_adam_amsgrad per run,
and the device-resident form esp_adam_dev(_amsgrad) the HIP-graph trainer captures) against
torch.optim.Adam with the same groups, on the same gradients (torch fp32 reference of the same op)."""
import pytest
import torch
from torch import nn

from espnet_slurp_amd.flat import FlatParams
from espnet_slurp_amd.optimizers.fused_adam import FusedAdam

pytestmark = pytest.mark.gpu


def _model(dev):
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(50, 70), nn.LayerNorm(70), nn.Linear(70, 30), nn.Linear(30, 90)).to(dev)


def _groups(model):
    decay = [p for p in model.parameters() if p.dim() == 2]
    rest = [p for p in model.parameters() if p.dim() != 2]
    return [{"params": decay, "weight_decay": 0.01},
            {"params": rest, "weight_decay": 1e-4, "amsgrad": True, "lr": 5e-3, "betas": (0.8, 0.99)}]


@pytest.mark.parametrize("device_step", [False, True])
def test_fused_adam_groups_amsgrad_vs_torch(dev, device_step):
    ref = _model(dev)
    ours = _model(dev)
    flat = FlatParams(ours, dev)
    opt = FusedAdam(_groups(ours), flat, lr=2e-3, eps=1e-7)
    topt = torch.optim.Adam(_groups(ref), lr=2e-3, eps=1e-7)
    clip = torch.tensor([0.0, 1.0, 1.0], device=dev)  # coefficient 1, finite
    g = torch.Generator(device=dev).manual_seed(3)
    for step in range(4):
        grads = [torch.randn(p.shape, generator=g, device=dev) * (10.0 if step == 1 else 0.1) for p in ref.parameters()]
        for p, q, gr in zip(ref.parameters(), ours.parameters(), grads):
            p.grad = gr.clone()
            flat.gview(q).copy_(gr)
        topt.step()
        if device_step:
            opt.step_device(clip)
        else:
            opt.step(clip=clip)
    torch.cuda.synchronize()
    for p, q in zip(ref.parameters(), ours.parameters()):
        assert torch.allclose(q, p, rtol=1e-5, atol=1e-6), (p - q).abs().max().item()
    sd = opt.state_dict()
    tsd = topt.state_dict()
    for i, st in tsd["state"].items():
        for k in ("exp_avg", "exp_avg_sq", "max_exp_avg_sq"):
            if k in st:
                assert torch.allclose(sd["state"][i][k], st[k], rtol=1e-5, atol=1e-9), (i, k)
    assert ("max_exp_avg_sq" in sd["state"][7]) and ("max_exp_avg_sq" not in sd["state"][0])
