"""Long utterances (VERDICT r5 'missing' 1): the reference's positional tables extend to any length
(embedding.py:59,196 extend_pe), so an utterance past the rel-pos probabilities kernel's T' <= 512 must
train through the materialised kernels (the ac / bd MFMA GEMMs, the register-resident softmax and
softmax / rel_shift adjoints up to T' = 1024) and past T' = 1024 through their looped forms
(softmax_fwd_loop_kernel, softmax_bwd_loop_kernel) -- nothing raises.  A C2-shaped model (d = 256, H = 4,
d_k = 64, FF 1024; 2 encoder / 2 decoder blocks) at T' = 875 (the longest LibriSpeech-960 utterances,
~35 s) latest and legacy, and at T' = 1100 (~44 s) latest, one training step against the reference's fp32
and fp64 steps (tests/golden/make_golden.py long), gated like every full-size test: loss / loss_ctc /
loss_att within max(1e-4, 2 e_ref), every gradient's norm, slice and whole-tensor fingerprint."""
import pytest
import torch

from oracle import espnet_cpu as O
from tests.helpers import FlipProbe, build_model, golden, grad_gate, load_seeded, loss_gate

pytestmark = pytest.mark.gpu


def long_cfg(rel):
    return O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=256, attention_heads=4, linear_units=1024,
                                                    num_blocks=2, rel_pos_type=rel),
                      dec=O.DecCfg(attention_heads=4, linear_units=1024, num_blocks=2))


@pytest.mark.parametrize("name,rel", [("long_t875_latest", "latest"), ("long_t875_legacy", "legacy"),
                                      ("long_t1100_latest", "latest")])
def test_long_utterance_train_step(dev, name, rel):
    g = golden(name)
    cfg = long_cfg(rel)
    model = build_model(cfg, dev)
    load_seeded(model, cfg, int(g["seed"]))
    speech, slen, text, tlen = O.synthetic_batch(int(g["B"]), int(g["T"]), 80, 600, list(g["lens"]),
                                                 list(g["ulens"]), int(g["seed"]) + 1)
    model.train()
    with FlipProbe(model) as fp:
        loss, stats, _ = model(speech.to(dev), slen, text, tlen)
    loss.backward()
    torch.cuda.synchronize()
    Tp = model.encoder.embed.out_frames(int(g["T"]))
    assert Tp == {"long_t875_latest": 875, "long_t875_legacy": 875, "long_t1100_latest": 1100}[name]
    fails = []
    for key, got in (("loss", loss.item()), ("loss_att", stats["loss_att"].item()),
                     ("loss_ctc", stats["loss_ctc"].item())):
        ok, info = loss_gate(got, g, key)
        if not ok:
            fails.append(info)
    assert abs(stats["acc"].item() - float(g["acc_f64"])) < 1e-6
    bad = grad_gate(model, g, flips=fp)
    assert not fails and not bad, (fails, bad)
