"""Flash rel-pos attention (csrc/flash_relpos.hip), latest AND legacy rel_shift, d_k = 64:
forward (scores + softmax + dropout + P.V in one kernel) and backward (recomputed scores,
in-kernel dq, dK / dV GEMMs over the dS / P_drop it writes, linear_pos gradient from dS
along its diagonals) against the fp64 oracle restatement of attention.py:117-308, at block
sizes from one partial 32-row block up to the full-size T' = 374; and against the
materialised-probability path with attention dropout on (same counter-RNG masks)."""
import pytest
import torch

from espnet_slurp_amd import kernels as K
from espnet_slurp_amd.asr.encoder.abs_encoder import pos_table
from espnet_slurp_amd.blocks import RelPositionMultiHeadedAttention, Seeds
from espnet_slurp_amd.flat import FlatParams
from oracle import espnet_cpu as O
from tests.helpers import rel_err
from tests.test_gpu_blocks import _check_grads, _params64

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _flash_on(monkeypatch):
    monkeypatch.setattr(K, "FLASH_ATTN", True)


def _block(dev, legacy, D, H, seed, std=0.1):
    torch.manual_seed(seed)
    mod = RelPositionMultiHeadedAttention(H, D, 0.0, legacy).to(dev)
    with torch.no_grad():
        for p in mod.parameters():
            p.normal_(0, std)
    mod.flat = FlatParams(mod, dev)
    return mod


def _run(mod, dev, x, res, dout, pos, klen, B, T, p_attn=0.0, seed=1):
    mod.p = p_attn
    out, c = mod.fwd(x.to(dev), res.to(dev), pos, klen.int().to(dev), B, T, 0.0, Seeds(seed), True)
    assert c.flash == K.flash_ok(T, mod.d_k)
    dx = mod.bwd(c, dout.to(dev))
    torch.cuda.synchronize()
    return out, dx


@pytest.mark.parametrize("legacy", [False, True])
@pytest.mark.parametrize("T,klens", [(29, [29, 23, 15]), (77, [77, 40, 9]), (130, [130, 129, 64]),
                                     (374, [374, 301])])
def test_flash_relpos_vs_oracle(dev, legacy, T, klens):
    assert K.flash_ok(T, 64)
    B, D, H = len(klens), 256, 4
    klen = torch.tensor(klens)
    mod = _block(dev, legacy, D, H, 3)
    x, res, dout = torch.randn(B * T, D), torch.randn(B * T, D), torch.randn(B * T, D)
    pos = pos_table("legacy" if legacy else "latest", T, D, dev)
    out, dx = _run(mod, dev, x, res, dout, pos, klen, B, T)
    P = _params64(mod, "a")
    xt = x.double().view(B, T, D).requires_grad_(True)
    mask = (~O.make_pad_mask(klen, T))[:, None, :]
    ref = O.rel_mha(P, "a", xt, pos.cpu().double()[None], mask, H, legacy) + res.double().view(B, T, D)
    ref.backward(dout.double().view(B, T, D))
    assert rel_err(out.cpu(), ref.detach().reshape(B * T, D)) < 1e-5
    assert rel_err(dx.cpu(), xt.grad.reshape(B * T, D)) < 1e-5
    _check_grads(mod, P, "a")


@pytest.mark.parametrize("legacy", [False, True])
@pytest.mark.parametrize("T", [77, 374])
def test_flash_matches_materialised_path_with_dropout(dev, legacy, T, monkeypatch):
    """Attention dropout 0.1: the flash kernels regenerate the materialised path's masks
    (index (z*T + i)*T + j of the same seed), so outputs and every gradient agree."""
    B, D, H = 2, 256, 4
    klen = torch.tensor([T, T - 20])
    x, res, dout = torch.randn(B * T, D), torch.randn(B * T, D), torch.randn(B * T, D)
    pos = pos_table("legacy" if legacy else "latest", T, D, dev)
    outs = []
    for flash in (True, False):
        monkeypatch.setattr(K, "FLASH_ATTN", flash)
        mod = _block(dev, legacy, D, H, 5)
        out, dx = _run(mod, dev, x, res, dout, pos, klen, B, T, p_attn=0.1, seed=7)
        outs.append((out.cpu(), dx.cpu(), {n: p.grad.detach().cpu().clone() for n, p in mod.named_parameters()}))
    (o1, d1, g1), (o2, d2, g2) = outs
    assert rel_err(o1, o2) < 1e-5
    assert rel_err(d1, d2) < 1e-5
    scale = max(float(v.abs().max()) for v in g2.values())
    for n in g1:
        gm = float(g2[n].abs().max())
        if gm < 1e-5 * scale:  # exactly-zero gradients (key bias): fp32 noise on both sides
            assert float(g1[n].abs().max()) < 1e-5 * scale, n
            continue
        assert float((g1[n] - g2[n]).abs().max()) <= 2e-5 * gm, (n, float((g1[n] - g2[n]).abs().max()), gm)


def test_flash_graph_replay_deterministic(dev):
    """Two runs of the flash forward + backward give bit-identical results (no atomics)."""
    B, T, D, H = 3, 130, 256, 4
    klen = torch.tensor([130, 99, 64])
    x, res, dout = torch.randn(B * T, D), torch.randn(B * T, D), torch.randn(B * T, D)
    pos = pos_table("latest", T, D, dev)
    runs = []
    for _ in range(2):
        mod = _block(dev, False, D, H, 9)
        out, dx = _run(mod, dev, x, res, dout, pos, klen, B, T, p_attn=0.1, seed=3)
        runs.append((out.cpu(), dx.cpu(), mod.flat.grad.cpu().clone()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])
    assert torch.equal(runs[0][2], runs[1][2])
