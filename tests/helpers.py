"""Shared test helpers: build the espnet_slurp_amd model for an oracle ModelCfg, load the
oracle's seeded parameters, fixture loading and tolerance checks."""
import os

import numpy as np
import torch

from oracle import espnet_cpu as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def token_list(V):
    return ["<blank>", "<unk>"] + [f"t{i}" for i in range(V - 3)] + ["<sos/eos>"]


def small_cfg(rel_pos_type="latest", D=64, blocks=2, V=32):
    return O.ModelCfg(vocab_size=V,
                      enc=O.EncCfg(output_size=D, attention_heads=4, linear_units=128, num_blocks=blocks,
                                   rel_pos_type=rel_pos_type),
                      dec=O.DecCfg(attention_heads=4, linear_units=128, num_blocks=2), ctc_weight=0.3, lsm_weight=0.1)


def c1_cfg():
    return O.ModelCfg(vocab_size=30, enc=O.EncCfg(kind="transformer", output_size=256, attention_heads=4,
                                                   linear_units=1024, num_blocks=4), dec=None, ctc_weight=1.0)


def c2_cfg(rel_pos_type="latest", blocks=12):
    return O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=256, attention_heads=4, linear_units=1024,
                                                    num_blocks=blocks, rel_pos_type=rel_pos_type),
                      dec=O.DecCfg(attention_heads=4, linear_units=2048, num_blocks=6))


def build_model(cfg: O.ModelCfg, device, specaug=None, dropout=None, frontend=None):
    from espnet_slurp_amd.asr.ctc import CTC
    from espnet_slurp_amd.asr.decoder.transformer_decoder import TransformerDecoder
    from espnet_slurp_amd.asr.encoder.conformer_encoder import ConformerEncoder
    from espnet_slurp_amd.asr.encoder.transformer_encoder import TransformerEncoder
    from espnet_slurp_amd.asr.espnet_model import ESPnetASRModel
    from espnet_slurp_amd.layers.utterance_mvn import UtteranceMVN
    e = cfg.enc
    p = e.dropout_rate if dropout is None else dropout
    if e.kind == "conformer":
        enc = ConformerEncoder(input_size=e.input_size, output_size=e.output_size, attention_heads=e.attention_heads,
                               linear_units=e.linear_units, num_blocks=e.num_blocks, dropout_rate=p,
                               positional_dropout_rate=p, attention_dropout_rate=p, macaron_style=e.macaron_style,
                               rel_pos_type=e.rel_pos_type, use_cnn_module=e.use_cnn_module,
                               cnn_module_kernel=e.cnn_module_kernel)
    else:
        enc = TransformerEncoder(input_size=e.input_size, output_size=e.output_size, attention_heads=e.attention_heads,
                                 linear_units=e.linear_units, num_blocks=e.num_blocks, dropout_rate=p,
                                 positional_dropout_rate=p, attention_dropout_rate=p)
    dec = None
    if cfg.dec is not None and cfg.ctc_weight != 1.0:
        d = cfg.dec
        dec = TransformerDecoder(vocab_size=cfg.vocab_size, encoder_output_size=e.output_size,
                                 attention_heads=d.attention_heads, linear_units=d.linear_units,
                                 num_blocks=d.num_blocks, dropout_rate=p, positional_dropout_rate=p,
                                 self_attention_dropout_rate=p, src_attention_dropout_rate=p)
    ctc = CTC(odim=cfg.vocab_size, encoder_output_size=e.output_size)
    m = ESPnetASRModel(vocab_size=cfg.vocab_size, token_list=token_list(cfg.vocab_size), frontend=frontend,
                       specaug=specaug, normalize=UtteranceMVN(), preencoder=None, encoder=enc, postencoder=None,
                       decoder=dec, ctc=ctc, joint_network=None, ctc_weight=cfg.ctc_weight,
                       lsm_weight=cfg.lsm_weight, length_normalized_loss=cfg.length_normalized_loss,
                       report_cer=False, report_wer=False)
    m = m.to(device)
    m.flatten()
    return m


def load_seeded(model, cfg, seed):
    P = O.deterministic_params(cfg, seed)
    missing, unexpected = model.load_state_dict(P, strict=True)
    return P


def keep_scale(p: float) -> float:
    """The inverted-dropout rescale the C ABI applies: 1 / (1 - p rounded to 1/65536)
    (include/espnet_mi355.h, esp_gemm_f32)."""
    return 65536.0 / (65536.0 - max(1, round(p * 65536)))


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


def slurp_config():
    """egs2/slurp/asr1 training config as resolved by the reference (fixture written by
    tests/golden/make_golden.py slurp from the recipe YAML; the GPU box has no reference)."""
    import json
    with open(os.path.join(GOLDEN, "slurp_asr_conformer_config.json")) as f:
        return json.load(f)


def slurp_args(conf, dropout_zero=False, specaug=True):
    """argparse.Namespace with the fields ASRTask.build_model reads (asr.py:439-562)."""
    import argparse
    import copy
    conf = copy.deepcopy(conf)
    if dropout_zero:
        for sec in ("encoder_conf", "decoder_conf"):
            for k in conf[sec]:
                if k.endswith("dropout_rate"):
                    conf[sec][k] = 0.0
    return argparse.Namespace(
        token_list=token_list(conf["token_list_size"]), input_size=conf["input_size"],
        frontend=None, frontend_conf={}, specaug=conf["specaug"] if specaug else None,
        specaug_conf=conf["specaug_conf"], normalize=conf["normalize"], normalize_conf=conf["normalize_conf"],
        preencoder=None, encoder=conf["encoder"], encoder_conf=conf["encoder_conf"], postencoder=None,
        decoder=conf["decoder"], decoder_conf=conf["decoder_conf"], ctc_conf=conf["ctc_conf"],
        model="espnet", model_conf=conf["model_conf"], init=None)


def cfg_from_config(conf, dropout_zero=False):
    """The oracle ModelCfg of a resolved config (parameter shapes / seeded values)."""
    e, d = conf["encoder_conf"], conf["decoder_conf"]
    z = (lambda x: 0.0) if dropout_zero else (lambda x: x)
    return O.ModelCfg(
        vocab_size=conf["token_list_size"],
        enc=O.EncCfg(input_size=conf["input_size"], output_size=e["output_size"], attention_heads=e["attention_heads"],
                     linear_units=e["linear_units"], num_blocks=e["num_blocks"], dropout_rate=z(e["dropout_rate"]),
                     positional_dropout_rate=z(e["positional_dropout_rate"]),
                     attention_dropout_rate=z(e["attention_dropout_rate"]),
                     rel_pos_type=e.get("rel_pos_type", "legacy"), macaron_style=e["macaron_style"],
                     use_cnn_module=e["use_cnn_module"], cnn_module_kernel=e["cnn_module_kernel"]),
        dec=O.DecCfg(attention_heads=d["attention_heads"], linear_units=d["linear_units"], num_blocks=d["num_blocks"]),
        ctc_weight=conf["model_conf"]["ctc_weight"], lsm_weight=conf["model_conf"]["lsm_weight"],
        length_normalized_loss=conf["model_conf"]["length_normalized_loss"])


# Conv2dSubsampling's first conv sits below two ReLUs whose pre-activations come within
# fp32 rounding of 0 at full size (tools/relu_flip_diag.py: 53 conv2 outputs within 1e-5 of 0
# at C2, B=2; the GPU's fp32 sum lands on the other side of 0 than fp64 for 1 of them): one
# such discrete mask decision moves single elements of conv.0's gradient by ~3e-4 of its
# max.  The reference's own fp32 run flips different ones (its slice error is 1e-4), so the
# slice gate for these two tensors is 2e-3; their norm gate stays at max(1e-4, 2 e_ref).
RELU_FLIP_SLICE_TOL = {"encoder.embed.conv.0.weight": 2e-3, "encoder.embed.conv.0.bias": 2e-3}


def grad_gate(model, g, skip_rel=1e-6):
    """Per-tensor gradient gate of a full-size fixture (make_golden.fullsize_train_fixture):
    the L2 norm and a fixed element slice must be as close to the fp64 reference as the
    reference's own fp32 result is (x2), or within 1e-4 relative.  A fixture may carry, per
    tensor, "flipb/<name>": a computed bound on how far the slice elements can move when ReLU
    decisions within fp32 rounding of 0 flip (make_bench_fixture.flip_bounds: the decoder's
    norm3 feeds a ReLU FFN); it is added to the slice gate.  Returns the failures."""
    scale = max(float(g["gmax_f64/" + n]) for n, _ in model.named_parameters())
    bad = []
    for n, p in model.named_parameters():
        got = p.grad.detach().double().reshape(-1).cpu()
        gm = float(g["gmax_f64/" + n])
        if gm < skip_rel * scale:  # exactly-zero gradients: fp32 noise on both sides
            if float(got.abs().max()) > 1e-5 * scale:
                bad.append((n, "nonzero", float(got.abs().max())))
            continue
        gn64, gn32 = float(g["gn_f64/" + n]), float(g["gn_f32/" + n])
        e_gpu = abs(float(got.norm()) - gn64) / gn64
        e_ref = abs(gn32 - gn64) / gn64
        if e_gpu > max(1e-4, 2 * e_ref):
            bad.append((n, "norm", e_gpu, e_ref))
        s = got[torch.from_numpy(g["gidx/" + n])].numpy()
        es = float(np.abs(s - g["gs_f64/" + n]).max()) / gm
        er = float(np.abs(g["gs_f32/" + n] - g["gs_f64/" + n]).max()) / gm
        flip = float(g["flipb/" + n]) / gm if ("flipb/" + n) in g else 0.0
        if es > max(1e-4, 2 * er, RELU_FLIP_SLICE_TOL.get(n, 0.0)) + flip:
            bad.append((n, "slice", es, er))
    return bad


def loss_gate(got, g, key="loss", slack=0.0):
    """|build - ref64| <= max(1e-4, 2 |ref32 - ref64|) (+ slack)."""
    l64, l32 = float(g[f"{key}_f64"]), float(g[f"{key}_f32"])
    tol = max(1e-4, 2 * abs(l32 - l64)) + slack
    return abs(got - l64) <= tol, (key, got, l64, tol)
