"""Full-size parity (VERDICT r1 'missing' 1 and 3): the C2 training step at T=1500, 12 blocks
with every parameter gradient (latest and legacy rel-pos: the fused attention kernels at
T'=374), the C4 shape (d=512, H=8, 17 blocks) forward loss and every gradient, all against fp32 AND fp64
reference results (tests/golden/make_golden.py fullgrad c4), gated like SURVEY.md §8(d)."""
import pytest
import torch

from oracle import espnet_cpu as O
from tests.helpers import build_model, c2_cfg, golden, grad_gate, load_seeded, loss_gate

pytestmark = pytest.mark.gpu


def _batch(g, F_, V):
    return O.synthetic_batch(int(g["B"]), int(g["T"]), F_, V, list(g["lens"]), list(g["ulens"]), int(g["seed"]) + 1)


@pytest.mark.parametrize("rel", ["latest", "legacy"])
def test_fullsize_c2_train_step_grads(dev, rel):
    g = golden(f"fullsize_c2_grad_{rel}")
    cfg = c2_cfg(rel)
    model = build_model(cfg, dev)
    load_seeded(model, cfg, int(g["seed"]))
    speech, slen, text, tlen = _batch(g, 80, 600)
    model.train()
    loss, stats, _ = model(speech.to(dev), slen, text, tlen)
    loss.backward()
    torch.cuda.synchronize()
    for key, got, slack in (("loss", loss.item(), 0.0), ("loss_att", stats["loss_att"].item(), 0.0),
                            ("loss_ctc", stats["loss_ctc"].item(), 2e-4)):
        ok, info = loss_gate(got, g, key, slack)
        assert ok, info
    assert abs(stats["acc"].item() - float(g["acc_f64"])) < 1e-6
    bad = grad_gate(model, g)
    assert not bad, bad


def _c4_cfg():
    return O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=512, attention_heads=8, linear_units=2048,
                                                   num_blocks=17, rel_pos_type="latest"),
                      dec=O.DecCfg(attention_heads=8, linear_units=2048, num_blocks=6))


def test_fullsize_c4_train_step_grads(dev):
    """C4 shape (d=512, H=8, d_k=64, FF 2048, 17 blocks, latest rel-pos) with every parameter
    gradient against the reference (VERDICT r2 'missing' 3: the latest rel-pos backward at
    H=8 was pinned by no fixture; attention.py:240-263)."""
    g = golden("fullsize_c4_grad_latest")
    cfg = _c4_cfg()
    model = build_model(cfg, dev)
    load_seeded(model, cfg, int(g["seed"]))
    speech, slen, text, tlen = _batch(g, 80, 600)
    model.train()
    loss, stats, _ = model(speech.to(dev), slen, text, tlen)
    loss.backward()
    torch.cuda.synchronize()
    for key, got, slack in (("loss", loss.item(), 0.0), ("loss_att", stats["loss_att"].item(), 0.0),
                            ("loss_ctc", stats["loss_ctc"].item(), 2e-4)):
        ok, info = loss_gate(got, g, key, slack)
        assert ok, info
    assert abs(stats["acc"].item() - float(g["acc_f64"])) < 1e-6
    bad = grad_gate(model, g)
    assert not bad, bad


def test_fullsize_c4_forward_loss(dev):
    g = golden("fullsize_c4_loss")
    cfg = _c4_cfg()
    model = build_model(cfg, dev)
    load_seeded(model, cfg, int(g["seed"]))
    speech, slen, text, tlen = _batch(g, 80, 600)
    model.train()
    with torch.no_grad():
        loss, stats, _ = model(speech.to(dev), slen, text, tlen)
    ok, info = loss_gate(loss.item(), g)
    assert ok, info
    ok, info = loss_gate(stats["loss_ctc"].item(), g, "loss_ctc", 2e-4)
    assert ok, info
