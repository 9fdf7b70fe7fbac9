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
                               cnn_module_kernel=e.cnn_module_kernel, input_layer=e.input_layer,
                               interctc_layer_idx=list(e.interctc_layer_idx),
                               interctc_use_conditioning=e.interctc_use_conditioning)
    else:
        enc = TransformerEncoder(input_size=e.input_size, output_size=e.output_size, attention_heads=e.attention_heads,
                                 linear_units=e.linear_units, num_blocks=e.num_blocks, dropout_rate=p,
                                 positional_dropout_rate=p, attention_dropout_rate=p, input_layer=e.input_layer)
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
                       interctc_weight=cfg.interctc_weight, lsm_weight=cfg.lsm_weight, length_normalized_loss=cfg.length_normalized_loss,
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
                     use_cnn_module=e["use_cnn_module"], cnn_module_kernel=e["cnn_module_kernel"],
                     input_layer=e.get("input_layer", "conv2d")),
        dec=O.DecCfg(attention_heads=d["attention_heads"], linear_units=d["linear_units"], num_blocks=d["num_blocks"]),
        ctc_weight=conf["model_conf"]["ctc_weight"], lsm_weight=conf["model_conf"]["lsm_weight"],
        length_normalized_loss=conf["model_conf"]["length_normalized_loss"])


class FlipProbe:
    """The GPU model's ReLU decisions at the flip sites of tests/golden/flipfix.py, read from the
    tensors the forward keeps for its backward: conv1 from z1 (NHWC [B, T1, F1, D], post-ReLU), conv2
    from z2 ([B*T2*F2, D], post-ReLU), decoder layer l from its FFN's dh/dv (dact: keep * scale *
    (v > 0), rows b * L + position).  Use around the forward: `with FlipProbe(model) as fp: ...`."""

    def __init__(self, model, copies=1):
        self.model = model
        self.ctx = {}
        # copies > 1: the batch is the fixture's utterances repeated `copies` times (utterance-mean
        # losses: each copy carries 1/copies of every per-utterance contribution), so a site's
        # decision is the mean of its copies' decisions -- (mean - s64) x c is the exact correction
        self.copies = copies

    def __enter__(self):
        from espnet_slurp_amd import blocks
        self._b = blocks
        self._sub, self._ffn = blocks.Conv2dSubsampling.fwd, blocks.PositionwiseFeedForward.fwd
        self._sub6 = blocks.Conv2dSubsampling6.fwd
        probe = self

        def sub(mod, *a, **k):
            x, c = probe._sub(mod, *a, **k)
            probe.ctx["conv"] = c
            return x, c

        def sub6(mod, *a, **k):  # conv2d6 (its own fwd): the same z1 / z2 decisions
            x, c = probe._sub6(mod, *a, **k)
            probe.ctx["conv"] = c
            return x, c
        blocks.Conv2dSubsampling6.fwd = sub6

        def ffn(mod, *a, **k):
            out, c = probe._ffn(mod, *a, **k)
            probe.ctx[id(mod)] = c
            return out, c
        blocks.Conv2dSubsampling.fwd, blocks.PositionwiseFeedForward.fwd = sub, ffn
        return self

    def __exit__(self, *exc):
        self._b.Conv2dSubsampling.fwd, self._b.PositionwiseFeedForward.fwd = self._sub, self._ffn
        self._b.Conv2dSubsampling6.fwd = self._sub6

    def decisions(self, site: str, idx: np.ndarray) -> np.ndarray:
        if self.copies == 1:
            return self._decisions(site, idx)
        nb = self.ctx["conv"].B // self.copies
        out = np.zeros(len(idx), dtype=np.float64)
        for k in range(self.copies):
            ik = idx.copy()
            ik[:, 0] += k * nb  # the utterance index of copy k
            out += self._decisions(site, ik)
        return out / self.copies

    def _decisions(self, site: str, idx: np.ndarray) -> np.ndarray:
        c = self.ctx["conv"]
        ix = torch.from_numpy(idx).to(c.z1.device)
        if site == "conv1":
            z = c.z1.view(c.B, c.T1, c.F1, -1)
            b, ch, t, f = ix.unbind(1)
            return (z[b, t, f, ch] > 0).to(torch.int8).cpu().numpy()
        if site == "conv2":
            z = c.z2.view(c.B, c.T2, c.F2, -1)
            b, o, t, f = ix.unbind(1)
            return (z[b, t, f, o] > 0).to(torch.int8).cpu().numpy()
        assert site.startswith("dec"), site
        ff = self.model.decoder.decoders[int(site[3:])].feed_forward
        dact = self.ctx[id(ff)].dact
        L = dact.shape[0] // c.B
        b, p, u = ix.unbind(1)
        return (dact[b * L + p, u] > 0).to(torch.int8).cpu().numpy()


def flip_corrected_slice(name, got_slice, g, flips):
    """got_slice with every recorded ReLU decision near 0 set to the fp64 one (flipfix.py): minus
    (s_gpu - s64) x contribution per site; (slice, the fixture's corrected fp32 slice or None)."""
    pre = f"flip/{name}/"
    sites = sorted({k[len(pre):].split("/")[0] for k in g if k.startswith(pre)})
    if not sites:
        return got_slice, None
    assert flips is not None, f"{name}: the fixture holds ReLU flip records, pass flips=FlipProbe(...)"
    s = got_slice.astype(np.float64).copy()
    for site in sites:
        idx = g[f"{pre}{site}/idx"]
        if len(idx) == 0:
            continue
        sg = flips.decisions(site, idx).astype(np.float64)
        s -= ((sg - g[f"{pre}{site}/s64"].astype(np.float64))[:, None] * g[f"{pre}{site}/c"]).sum(0)
    return s, g[f"gs_f32c/{name}"]


def grad_gate(model, g, skip_rel=1e-6, flips=None):
    """Per-tensor gradient gate of a full-size fixture (make_golden.fullsize_train_fixture): the L2
    norm and a fixed element slice must be as close to the fp64 reference as the reference's own
    fp32 result is (x2), or within 1e-4 relative.  Slices of tensors right below a ReLU
    (Conv2dSubsampling's conv.0, the decoder layers' norm3) are compared after the ReLU decisions
    within fp32 rounding of 0 are set to the fp64 ones on both sides -- the GPU's read by `flips`
    (FlipProbe), the reference fp32 run's stored -- with their exact contributions from the fixture
    (tests/golden/flipfix.py).  Returns the failures."""
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
        s, s32 = flip_corrected_slice(n, s, g, flips)
        s32 = g["gs_f32/" + n] if s32 is None else s32
        es = float(np.abs(s - g["gs_f64/" + n]).max()) / gm
        er = float(np.abs(s32 - g["gs_f64/" + n]).max()) / gm
        if es > max(1e-4, 2 * er):
            bad.append((n, "slice", es, er))
        bad += fingerprint_gate(n, p.grad, g, gn64, flips)
    return bad


def fingerprint_gate(n, grad, g, gn64, flips=None):
    """The whole-tensor fingerprint of a full-size fixture (tests/golden/fingerprint.py, round 6): the 8 fp64
    projections on fixed +-1 vectors, relative to the fp64 norm, and for rank >= 2 tensors every row's L2 norm,
    relative to the largest fp64 row norm -- each within max(1e-4, 2 e_ref), e_ref the reference fp32 run's own
    error.  Projections of the ReLU-flip tensors are corrected like their slices (flip/<n>/<site>/cp, exact:
    a projection is linear); their row norms are not gated (not linear; the corrected projections cover
    them).  Fixtures written before round 6 carry no fingerprint: nothing is checked then."""
    if "fp_f64/" + n not in g:
        return []
    import sys
    sys.path.insert(0, GOLDEN)
    import fingerprint as FP
    bad = []
    p64 = g["fp_f64/" + n].astype(np.float64)
    pg = FP.projections(n, grad).cpu().numpy()
    pre = f"flip/{n}/"
    sites = sorted({k[len(pre):].split("/")[0] for k in g if k.startswith(pre)})
    for site in sites:
        idx = g[f"{pre}{site}/idx"]
        if len(idx) == 0 or f"{pre}{site}/cp" not in g:
            continue
        assert flips is not None, f"{n}: the fixture holds ReLU flip records, pass flips=FlipProbe(...)"
        sg = flips.decisions(site, idx).astype(np.float64)
        pg = pg - ((sg - g[f"{pre}{site}/s64"].astype(np.float64))[:, None] * g[f"{pre}{site}/cp"]).sum(0)
    p32 = g["fp_f32c/" + n] if "fp_f32c/" + n in g else g["fp_f32/" + n]
    ep = float(np.abs(pg - p64).max()) / gn64
    er = float(np.abs(p32 - p64).max()) / gn64
    if ep > max(1e-4, 2 * er):
        bad.append((n, "projection", ep, er))
    # rows: every row of a tensor without flip sites; of a tensor whose sites each move one row (conv.2, the
    # decoder w_1: flip/<n>/<site>/rows), every row no recorded site touches; of the others (conv.0: a conv2 site
    # reaches every channel through relu1's mask) none -- their corrected projections cover them
    skip = None
    if sites:
        if all(f"{pre}{site}/rows" in g for site in sites):
            skip = np.unique(np.concatenate([g[f"{pre}{site}/rows"] for site in sites] + [np.zeros(0, np.int64)]))
        else:
            skip = "all"
    if "rn_f64/" + n in g and not (isinstance(skip, str)):
        r64 = g["rn_f64/" + n].astype(np.float64)
        rg = FP.row_norms(grad).cpu().numpy()
        er = float(g["rn_eref/" + n])
        d = np.abs(rg - r64)
        if skip is not None and len(skip):
            d[skip] = 0.0
        en = float(d.max()) / max(float(r64.max()), 1e-300)
        if en > max(1e-4, 2 * er):
            bad.append((n, "rows", en, er, int(d.argmax())))
    return bad


def loss_gate(got, g, key="loss", slack=0.0):
    """|build - ref64| <= max(1e-4, 2 |ref32 - ref64|) (+ slack) on the loss.
    The component losses (loss_ctc ~ 1.6e3-1.9e3, loss_att) are gated the same way with one more floor:
    one fp32 ulp of the value (1.22e-4 at loss_ctc's magnitude).  An fp32 number of that size is a
    multiple of its ulp, so an atol below one ulp demands the correctly rounded result, which no fp32
    pipeline promises -- the reference's own fp32 loss_ctc is off by 5.6e-6 .. 7.4e-4 (0.05 .. 6 ulp)
    across the committed fixtures; a 1-ulp difference is a rounding-order difference, not a defect.
    The total loss (~700, ulp 6.1e-5) keeps the plain max(1e-4, 2 e_ref)."""
    l64, l32 = float(g[f"{key}_f64"]), float(g[f"{key}_f32"])
    tol = max(1e-4, 2 * abs(l32 - l64)) + slack
    if key != "loss":
        tol = max(tol, float(np.spacing(np.float32(abs(l64)))))
    print(f"LOSS_GATE {key} err={abs(got - l64):.3e} e_ref={abs(l32 - l64):.3e} ulp32={float(np.spacing(np.float32(l64))):.3e} "
          f"tol={tol:.3e} got={got!r} l64={l64!r}")
    return abs(got - l64) <= tol, (key, got, l64, tol)
