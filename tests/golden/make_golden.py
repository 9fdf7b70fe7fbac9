"""Generate golden fixtures by running the REFERENCE implementation (this container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Imports BriansIDP/espnet_slurp from /root/reference through `refshim`,
builds the reference modules, loads the seeded parameters of
`oracle.espnet_cpu.deterministic_params`, runs them on seeded synthetic inputs and
stores inputs + outputs (+ gradients) as small .npz files next to this script.  The
fixtures are DATA; the reference's code never travels with them.  Each fixture is also
checked against the oracle restatement here, so a drift is caught at generation time.
"""
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import refshim  # noqa: E402

refshim.install()

from espnet2.asr.ctc import CTC  # noqa: E402
from espnet2.asr.decoder.transformer_decoder import TransformerDecoder  # noqa: E402
from espnet2.asr.encoder.conformer_encoder import ConformerEncoder  # noqa: E402
from espnet2.asr.encoder.transformer_encoder import TransformerEncoder  # noqa: E402
from espnet2.asr.espnet_model import ESPnetASRModel  # noqa: E402
from espnet2.asr.specaug.specaug import SpecAug  # noqa: E402
from espnet2.layers.utterance_mvn import UtteranceMVN  # noqa: E402
from espnet2.schedulers.warmup_lr import WarmupLR  # noqa: E402
from espnet2.layers.mask_along_axis import mask_along_axis  # noqa: E402
from espnet2.layers.time_warp import time_warp  # noqa: E402
from espnet.nets.pytorch_backend.ctc import CTC as CTC1  # noqa: E402

from oracle import espnet_cpu as O  # noqa: E402
from oracle import ctc_np  # noqa: E402

torch.set_num_threads(8)


def token_list(V):
    return ["<blank>", "<unk>"] + [f"t{i}" for i in range(V - 3)] + ["<sos/eos>"]


def build_reference(cfg: O.ModelCfg):
    e = cfg.enc
    if e.kind == "conformer":
        enc = ConformerEncoder(
            input_size=e.input_size, output_size=e.output_size, attention_heads=e.attention_heads,
            linear_units=e.linear_units, num_blocks=e.num_blocks, dropout_rate=e.dropout_rate,
            positional_dropout_rate=e.positional_dropout_rate,
            attention_dropout_rate=e.attention_dropout_rate, input_layer=e.input_layer,
            normalize_before=True, macaron_style=e.macaron_style, rel_pos_type=e.rel_pos_type,
            pos_enc_layer_type="rel_pos", selfattention_layer_type="rel_selfattn",
            activation_type="swish", use_cnn_module=e.use_cnn_module,
            cnn_module_kernel=e.cnn_module_kernel, interctc_layer_idx=list(e.interctc_layer_idx),
            interctc_use_conditioning=e.interctc_use_conditioning)
    else:
        enc = TransformerEncoder(
            input_size=e.input_size, output_size=e.output_size, attention_heads=e.attention_heads,
            linear_units=e.linear_units, num_blocks=e.num_blocks, dropout_rate=e.dropout_rate,
            positional_dropout_rate=e.positional_dropout_rate,
            attention_dropout_rate=e.attention_dropout_rate, input_layer="conv2d")
    dec = None
    if cfg.dec is not None and cfg.ctc_weight != 1.0:
        d = cfg.dec
        dec = TransformerDecoder(
            vocab_size=cfg.vocab_size, encoder_output_size=e.output_size,
            attention_heads=d.attention_heads, linear_units=d.linear_units, num_blocks=d.num_blocks,
            dropout_rate=d.dropout_rate, positional_dropout_rate=d.positional_dropout_rate,
            self_attention_dropout_rate=d.self_attention_dropout_rate,
            src_attention_dropout_rate=d.src_attention_dropout_rate)
    ctc = CTC(odim=cfg.vocab_size, encoder_output_size=e.output_size)
    model = ESPnetASRModel(
        vocab_size=cfg.vocab_size, token_list=token_list(cfg.vocab_size), frontend=None,
        specaug=None, normalize=UtteranceMVN(), preencoder=None, encoder=enc, postencoder=None,
        decoder=dec, ctc=ctc, joint_network=None, ctc_weight=cfg.ctc_weight,
        interctc_weight=cfg.interctc_weight, lsm_weight=cfg.lsm_weight, length_normalized_loss=cfg.length_normalized_loss,
        report_cer=False, report_wer=False)
    return model


def load_params(model, cfg, seed, dtype=torch.float32):
    P = O.deterministic_params(cfg, seed, dtype)
    sd = model.state_dict()
    assert set(sd.keys()) == set(P.keys()), (set(sd) ^ set(P))
    for k in sd:
        assert tuple(sd[k].shape) == tuple(P[k].shape), (k, sd[k].shape, P[k].shape)
    model.load_state_dict(P)
    return P


def small_cfg(rel_pos_type="latest", D=64, blocks=2, V=32):
    return O.ModelCfg(
        vocab_size=V,
        enc=O.EncCfg(output_size=D, attention_heads=4, linear_units=128, num_blocks=blocks,
                     rel_pos_type=rel_pos_type),
        dec=O.DecCfg(attention_heads=4, linear_units=128, num_blocks=2),
        ctc_weight=0.3, lsm_weight=0.1)


def model_fixture(name, cfg, B, T, lens, ulens, seed, with_grads=True, dtype=torch.float32):
    model = build_reference(cfg).to(dtype)
    load_params(model, cfg, seed, dtype)
    model.train()
    speech, slen, text, tlen = O.synthetic_batch(B, T, cfg.enc.input_size, cfg.vocab_size, lens, ulens, seed + 1)
    speech = speech.to(dtype)
    loss, stats, weight = model(speech.clone(), slen.clone(), text.clone(), tlen.clone())
    loss.backward()
    out = dict(speech=speech.float().numpy(), speech_lengths=slen.numpy(), text=text.numpy(),
               text_lengths=tlen.numpy(), seed=np.int64(seed), loss=np.float64(loss.item()))
    for k in ["loss_ctc", "loss_att"] + [k for k in stats if k.startswith("loss_interctc_layer")]:
        if stats.get(k) is not None:
            out[k] = np.float64(stats[k].item())
    if stats.get("acc") is not None:
        out["acc"] = np.float64(stats["acc"])
    sd = model.state_dict()
    if with_grads:
        for n, p in model.named_parameters():
            out["grad/" + n] = p.grad.float().numpy()
        for n, b in sd.items():
            if "running" in n:
                out["buf/" + n] = b.float().numpy()
    else:
        for n, p in model.named_parameters():
            out["gradnorm/" + n] = np.float64(p.grad.double().norm().item())
    # cross-check the oracle restatement against the reference right here
    P = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k)
         for k, v in O.deterministic_params(cfg, seed, dtype).items()}
    bn = {}
    oloss, ostats, _ = O.asr_forward(P, speech, slen, text, tlen, cfg, bn_state=bn)
    oloss.backward()
    err = abs(oloss.item() - loss.item())
    gerr = max(float((P[n].grad - p.grad).abs().max()) for n, p in model.named_parameters())
    if with_grads:
        berr = max(float((bn[n] - b).abs().max()) for n, b in sd.items() if "running" in n)
        assert berr < 1e-5, berr
    print(f"{name}: ref loss {loss.item():.6f} oracle {oloss.item():.6f} |dl|={err:.2e} max|dg|={gerr:.2e}")
    assert err < 1e-5 * max(1.0, abs(loss.item())), err
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


def ctc_fixture():
    rng = np.random.Generator(np.random.PCG64(7))
    T, B, V = 40, 4, 12
    logits = (2.0 * rng.standard_normal((T, B, V))).astype(np.float32)
    ilens = np.array([40, 33, 20, 5], dtype=np.int64)
    tlens = np.array([10, 7, 6, 9], dtype=np.int64)    # utt 3 infeasible -> inf -> zero_infinity
    targets = rng.integers(1, V, size=(B, 10)).astype(np.int64)
    targets[1, 2] = targets[1, 1]                        # repeated label
    targets[2, :6] = [3, 3, 3, 4, 4, 5]
    ref = CTC(odim=V, encoder_output_size=V)
    th = torch.from_numpy(logits).requires_grad_(True)
    ys_true = torch.cat([torch.from_numpy(targets[i, :l]) for i, l in enumerate(tlens)])
    loss = ref.loss_fn(th, ys_true, torch.from_numpy(ilens), torch.from_numpy(tlens))
    loss.backward()
    per = torch.nn.functional.ctc_loss(torch.from_numpy(logits).log_softmax(2), ys_true,
                                       torch.from_numpy(ilens), torch.from_numpy(tlens),
                                       reduction="none", zero_infinity=True)
    nll, g = ctc_np.ctc_loss_np(logits, ilens, targets, tlens)
    print("ctc: ref", per.numpy(), "np", nll, "max|dgrad|", np.abs(g / B - th.grad.numpy()).max())
    np.savez_compressed(os.path.join(HERE, "ctc.npz"), logits=logits, ilens=ilens, tlens=tlens,
                        targets=targets, nll=per.double().numpy(), loss=np.float64(loss.item()),
                        grad=th.grad.numpy())


def align_fixture():
    rng = np.random.Generator(np.random.PCG64(11))
    V = 10
    ctc1 = CTC1(odim=V, eprojs=V, dropout_rate=0.0)
    with torch.no_grad():
        ctc1.ctc_lo.weight.copy_(torch.eye(V))
        ctc1.ctc_lo.bias.zero_()
    cases = {}
    for ci, (T, U, peaked) in enumerate([(30, 6, True), (25, 8, False), (12, 5, False), (40, 3, True)]):
        y = rng.integers(1, V, size=U).astype(np.int64)
        if ci == 2:
            y[1] = y[0]
        h = rng.standard_normal((T, V)).astype(np.float32)
        if peaked:   # a plausible trained-model shape: a monotone path dominates
            pos = np.sort(rng.choice(np.arange(1, T - 1), size=U, replace=False))
            h[:, 0] += 3.0
            for u, p in enumerate(pos):
                h[p, y[u]] += 6.0
        with torch.no_grad():
            ali = ctc1.forced_align(torch.from_numpy(h)[None], torch.from_numpy(y), blank_id=0)
            lpz = ctc1.log_softmax(torch.from_numpy(h)[None])[0].numpy()
        ali = np.array([int(a) for a in ali], dtype=np.int64)
        mine = np.array(ctc_np.forced_align_np(lpz, y), dtype=np.int64)
        assert (mine == ali).all(), (ci, mine, ali)
        cases[f"h{ci}"] = h
        cases[f"lpz{ci}"] = lpz
        cases[f"y{ci}"] = y
        cases[f"ali{ci}"] = ali
        cases[f"argmax{ci}"] = torch.argmax(torch.from_numpy(h), dim=-1).numpy()
    print("align: ok", {k: v.tolist() for k, v in cases.items() if k.startswith("ali")})
    np.savez_compressed(os.path.join(HERE, "align.npz"), **cases)


def align_c2_fixture():
    """forced_align / argmax at the C2 workload shape (VERDICT r5 'next' 1a): T' = 374 frames, V = 600,
    U in {20, 40}, through the reference's own espnet1 CTC (ctc_lo = identity, so h is the logits).
    Cases: 0 trained-like (a monotone label path dominates), 1 / 2 random logits (U = 40 / 20), where
    the s = 0 candidate s-1 = Python's index -1 (the last state) wins on some frames of the returned
    path, 3 logits quantised to {0, 1, 2} (exact fp32 ties in lpz, the path sums and argmax), 4 all-zero
    logits (every path sum ties), 5 runs of repeated labels.  The generator asserts the oracle equals the
    reference on every case and records how many frames of each alignment came through the wrap."""
    rng = np.random.Generator(np.random.PCG64(374))
    T, V = 374, 600
    ctc1 = CTC1(odim=V, eprojs=V, dropout_rate=0.0)
    with torch.no_grad():
        ctc1.ctc_lo.weight.copy_(torch.eye(V))
        ctc1.ctc_lo.bias.zero_()
    cases = {}
    wraps = []
    specs = [(40, "peaked"), (40, "random"), (20, "random"), (40, "quant"), (40, "zeros"), (40, "repeats")]
    for ci, (U, kind) in enumerate(specs):
        y = rng.integers(1, V - 1, size=U).astype(np.int64)
        if kind == "repeats":
            y[5:9] = y[4]
            y[20:22] = y[19]
        if kind == "peaked":
            h = rng.standard_normal((T, V)).astype(np.float32)
            pos = np.sort(rng.choice(np.arange(1, T - 1), size=U, replace=False))
            h[:, 0] += 4.0
            for u, p in enumerate(pos):
                h[p, y[u]] += 8.0
        elif kind in ("random", "repeats"):
            h = (2.0 * rng.standard_normal((T, V))).astype(np.float32)
        elif kind == "quant":
            h = rng.integers(0, 3, size=(T, V)).astype(np.float32)
        else:
            h = np.zeros((T, V), dtype=np.float32)
        with torch.no_grad():
            ali = ctc1.forced_align(torch.from_numpy(h)[None], torch.from_numpy(y), blank_id=0)
            lpz = ctc1.log_softmax(torch.from_numpy(h)[None])[0].numpy()
        ali = np.array([int(a) for a in ali], dtype=np.int64)
        mine, states = ctc_np.forced_align_np(lpz, y, return_states=True)
        assert (np.array(mine) == ali).all(), (ci, kind)
        wraps.append(int(sum(1 for s_ in states if s_ < 0)))
        cases[f"lpz{ci}"] = lpz
        cases[f"y{ci}"] = y
        cases[f"ali{ci}"] = ali
        # argmax (ctc.py:119-127 is torch.argmax over the logits): on lpz for every case, and on the logits
        # themselves where they hold exact ties (kept small: the integer / zero logits compress to nothing)
        cases[f"argmax{ci}"] = torch.argmax(torch.from_numpy(lpz), dim=-1).numpy()
        if kind in ("quant", "zeros"):
            cases[f"h{ci}"] = h
            cases[f"argmax_h{ci}"] = torch.argmax(torch.from_numpy(h), dim=-1).numpy()
    cases["wrap_frames"] = np.array(wraps, dtype=np.int64)
    cases["kinds"] = np.array([k for _, k in specs])
    print("align_c2: ok; frames through the s=0 wrap per case", wraps)
    assert any(w > 0 for w in wraps), "no case exercises the s=0 wrap"
    np.savez_compressed(os.path.join(HERE, "align_c2.npz"), **cases)


def specaug_fixture():
    B, T, F_ = 2, 100, 80
    rng = np.random.Generator(np.random.PCG64(5))
    x = rng.standard_normal((B, T, F_)).astype(np.float32)
    out = dict(x=x)
    # time warp (window 5, bicubic): replicate the reference's two torch.randint draws
    for s in (3, 4):
        torch.manual_seed(s)
        y = time_warp(torch.from_numpy(x).clone(), window=5, mode="bicubic")
        torch.manual_seed(s)
        center = int(torch.randint(5, T - 5, (1,))[0])
        warped = int(torch.randint(center - 5, center + 5, (1,))[0] + 1)
        mine = O.time_warp_fixed(torch.from_numpy(x), center, warped)
        assert torch.allclose(mine, y, atol=1e-6), float((mine - y).abs().max())
        out[f"tw{s}_center"] = np.int64(center)
        out[f"tw{s}_warped"] = np.int64(warped)
        out[f"tw{s}_y"] = y.numpy()
    for dim, rng_w, key in ((2, (0, 30), "freq"), (1, (0, 40), "time")):
        torch.manual_seed(9)
        y, _ = mask_along_axis(torch.from_numpy(x).clone(), None, rng_w, dim, 2)
        torch.manual_seed(9)
        ml = torch.randint(rng_w[0], rng_w[1], (B, 2))
        mp = torch.randint(0, max(1, x.shape[dim] - int(ml.max())), (B, 2))
        mine = O.mask_along_axis_fixed(torch.from_numpy(x), mp, ml, dim)
        assert torch.equal(mine, y)
        out[f"{key}_pos"] = mp.numpy()
        out[f"{key}_len"] = ml.numpy()
        out[f"{key}_y"] = y.numpy()
    lens = torch.tensor([100, 71])
    xm = torch.from_numpy(x).clone()
    xm[1, 71:] = 0
    y, _ = UtteranceMVN()(xm.clone(), lens)
    assert torch.allclose(O.utterance_mvn(xm, lens), y)
    out["mvn_x"] = xm.numpy()
    out["mvn_lens"] = lens.numpy()
    out["mvn_y"] = y.numpy()
    # whole SpecAug module under a fixed seed, for the full-module shape contract
    sa = SpecAug(apply_time_warp=True, time_warp_window=5, time_warp_mode="bicubic",
                 freq_mask_width_range=(0, 30), num_freq_mask=2,
                 time_mask_width_range=(0, 40), num_time_mask=2)
    torch.manual_seed(21)
    y, _ = sa(torch.from_numpy(x).clone(), torch.tensor([T, T]))
    out["specaug_seed21_y"] = y.numpy()
    print("specaug: ok")
    np.savez_compressed(os.path.join(HERE, "specaug.npz"), **out)


def train_step_fixture():
    """Two reference optimizer steps: clip_grad_norm_(5) + Adam + WarmupLR (trainer.py:642-686)."""
    cfg = small_cfg("latest", D=32, blocks=1, V=16)
    model = build_reference(cfg)
    load_params(model, cfg, 3)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=0.002, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-6)
    sch = WarmupLR(opt, warmup_steps=10)
    out = {}
    for step in range(2):
        speech, slen, text, tlen = O.synthetic_batch(2, 64, 80, cfg.vocab_size, [64, 50], [5, 3], 100 + step)
        loss, stats, weight = model(speech, slen, text, tlen)
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0, norm_type=2.0)
        out[f"loss{step}"] = np.float64(loss.item())
        out[f"gradnorm{step}"] = np.float64(gn.item())
        out[f"lr{step}"] = np.float64(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
        opt.zero_grad()
    for n, p in model.named_parameters():
        out["param/" + n] = p.detach().numpy()
    print("train_step: losses", out["loss0"], out["loss1"], "gn", out["gradnorm0"], out["gradnorm1"])
    np.savez_compressed(os.path.join(HERE, "train_step.npz"), **out)


def fullsize_fixture():
    """C2 shape (d=256, 12L, T=1500, B=2): fp32 vs fp64 reference loss (SURVEY.md §0.4 gate)."""
    cfg = O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=256, attention_heads=4, linear_units=1024,
                                                   num_blocks=12, rel_pos_type="latest"),
                     dec=O.DecCfg(attention_heads=4, linear_units=2048, num_blocks=6))
    out = {}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        model = build_reference(cfg).to(dt)
        load_params(model, cfg, 42, dt)
        model.train()
        speech, slen, text, tlen = O.synthetic_batch(2, 1500, 80, 600, [1500, 1337], [40, 27], 43)
        with torch.no_grad():
            loss, stats, _ = model(speech.to(dt), slen, text, tlen)
        out[f"loss_{tag}"] = np.float64(loss.item())
        out[f"loss_ctc_{tag}"] = np.float64(stats["loss_ctc"].item())
        out[f"loss_att_{tag}"] = np.float64(stats["loss_att"].item())
        print("fullsize", tag, loss.item())
    out.update(lens=np.array([1500, 1337]), ulens=np.array([40, 27]), seed=np.int64(42))
    np.savez_compressed(os.path.join(HERE, "fullsize_c2.npz"), **out)


N_SLICE = 16


def slice_indices(name: str, numel: int) -> np.ndarray:
    """Fixed element indices per tensor (first 4, last 4, 8 seeded by the name)."""
    import zlib
    rng = np.random.Generator(np.random.PCG64(zlib.crc32(name.encode())))
    k = min(numel, N_SLICE)
    if numel <= N_SLICE:
        return np.arange(numel, dtype=np.int64)
    idx = np.concatenate([np.arange(4), np.arange(numel - 4, numel), rng.integers(4, numel - 4, size=k - 8)])
    return idx.astype(np.int64)


def grad_summary(model, tag: str, out: dict, rows=None):
    """Per-tensor gradient L2 norm (fp64), max |g|, a fixed slice of elements and (rows: a dict kept across
    the fp32 and fp64 runs, fingerprint.finish_rows after both) the whole-tensor fingerprint."""
    import fingerprint as FP
    for n, p in model.named_parameters():
        g = p.grad.detach().double().reshape(-1)
        idx = slice_indices(n, g.numel())
        out[f"gn_{tag}/{n}"] = np.float64(g.norm().item())
        out[f"gmax_{tag}/{n}"] = np.float64(g.abs().max().item())
        out[f"gidx/{n}"] = idx
        out[f"gs_{tag}/{n}"] = g[torch.from_numpy(idx)].numpy()
        if rows is not None:
            FP.summarize(n, p.grad.detach(), tag, out, rows)


def oracle_vs_reference(cfg, seed, speech, slen, text, tlen, ref_loss, ref_grads, name, log=print):
    """VERDICT r5 'next' 1d: the oracle restatement (oracle/espnet_cpu.py) run in fp64 on the fixture's own
    inputs and parameters must equal the reference's fp64 step -- the loss and EVERY parameter gradient
    (max |g_oracle - g_ref| relative to the largest gradient element of the model) -- to fp64 rounding, so
    the oracle-generated fixtures at other batch sizes (make_bench_fixture.py) rest on a pinned oracle."""
    P = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k)
         for k, v in O.deterministic_params(cfg, seed, torch.float64).items()}
    oloss, _, _ = O.asr_forward(P, speech.to(torch.float64), slen, text, tlen, cfg, bn_state={})
    oloss.backward()
    scale = max(float(g.abs().max()) for g in ref_grads.values())
    dl = abs(oloss.item() - ref_loss) / max(1.0, abs(ref_loss))
    worst = max((float((P[n].grad - g).abs().max()) / scale, n) for n, g in ref_grads.items())
    log(f"{name}: oracle vs reference fp64: |dloss| {dl:.2e} relative, worst gradient {worst[0]:.2e} ({worst[1]})")
    assert dl < 1e-10, dl
    assert worst[0] < 1e-9, worst
    return dl, worst[0]


def fullsize_train_fixture(name: str, cfg, B=2, T=1500, lens=(1500, 1337), ulens=(40, 27), seed=42,
                           with_grads=True, build=None, train=True, oracle_check=True):
    """Full-size fp32 AND fp64 reference step (SURVEY.md §8(d) gate judged against fp64): loss,
    loss_ctc / loss_att / acc and, with_grads, every parameter's gradient norm, a fixed
    slice of its elements and its whole-tensor fingerprint (fingerprint.py).  train=False runs the
    reference in eval mode (validation step: no dropout, no SpecAug, BatchNorm from its running
    statistics).  With grads and oracle_check, the oracle's fp64 step is asserted equal to the
    reference's (loss and every gradient, oracle_vs_reference) before the fixture is written."""
    import time as _t
    import flipfix
    import fingerprint as FP
    build = build or (lambda: build_reference(cfg))
    out = {}
    recs = {}
    rows = {}
    shapes = {}
    F_ = cfg.enc.input_size
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        t0 = _t.time()
        model = build().to(dt)
        load_params(model, cfg, seed, dt)
        model.train(train)
        speech, slen, text, tlen = O.synthetic_batch(B, T, F_, cfg.vocab_size, list(lens), list(ulens), seed + 1)
        if with_grads:
            # the ReLU decisions near 0 and their slice contributions (flipfix.py)
            with flipfix.ReferenceProbe(model) as probe:
                loss, stats, _ = model(speech.to(dt), slen, text, tlen)
            loss.backward()
            recs[tag] = probe.rec.detach()
            grad_summary(model, tag, out, rows)
            shapes = {n: p.numel() for n, p in model.named_parameters()}
            if tag == "f64" and oracle_check and train:
                ref_grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
                ref_loss = loss.item()
        else:
            with torch.no_grad():
                loss, stats, _ = model(speech.to(dt), slen, text, tlen)
        out[f"loss_{tag}"] = np.float64(loss.item())
        for k in ("loss_ctc", "loss_att", "acc", "cer_ctc", "cer", "wer"):
            if stats.get(k) is not None:
                out[f"{k}_{tag}"] = np.float64(float(stats[k]))
        if not train:  # the greedy sequences the eval-mode error calculator scored
            with torch.no_grad():
                hs, hl = model.encode(speech.to(dt), slen)
                out[f"ctc_argmax_{tag}"] = model.ctc.argmax(hs).numpy()
        print(f"{name} {tag}: loss {loss.item():.6f} ({_t.time() - t0:.1f} s)", flush=True)
        del model
    if with_grads:
        FP.finish_rows(out, rows)
        gs32 = {k[len("gs_f32/"):]: v for k, v in out.items() if k.startswith("gs_f32/")}
        flipfix.flip_records(recs["f64"], recs["f32"], lambda n: out["gidx/" + n], out, gs32,
                             log=lambda m: print(f"{name}: {m}", flush=True), shapes=shapes)
        del recs
        if oracle_check and train:
            speech, slen, text, tlen = O.synthetic_batch(B, T, F_, cfg.vocab_size, list(lens), list(ulens), seed + 1)
            t0 = _t.time()
            dl, dg = oracle_vs_reference(cfg, seed, speech, slen, text, tlen, ref_loss, ref_grads, name,
                                         log=lambda m: print(m, flush=True))
            print(f"{name}: oracle check {_t.time() - t0:.1f} s", flush=True)
            out["oracle_ref64_dloss"] = np.float64(dl)
            out["oracle_ref64_dgrad"] = np.float64(dg)
    out.update(lens=np.array(lens), ulens=np.array(ulens), seed=np.int64(seed), B=np.int64(B), T=np.int64(T))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


def amp_reference_fixture(name: str, cfg, B=2, T=1500, lens=(1500, 1337), ulens=(40, 27), seed=57):
    """The reference's own reduced-precision step at a full-size shape (VERDICT r3 'next' 1a): the
    fp64 step's gradient vs the same step under torch.autocast(bfloat16) (the reference trains with
    autocast under use_amp, trainer.py:181-195,554; here the CPU's bf16 autocast: GEMM / conv inputs
    and outputs in bf16).  Stored per tensor: the cosine of the autocast gradient to the fp64 one and
    the relative norm difference ("cos_amp/<n>", "dn_amp/<n>"), and the autocast loss -- the bar the
    GPU's bf16 step is held to (tests/test_gpu_fullsize.py)."""
    import time as _t
    out = {}
    F_ = cfg.enc.input_size
    speech, slen, text, tlen = O.synthetic_batch(B, T, F_, cfg.vocab_size, list(lens), list(ulens), seed + 1)
    grads = {}
    for tag in ("f64", "amp"):
        t0 = _t.time()
        dt = torch.float64 if tag == "f64" else torch.float32
        model = build_reference(cfg).to(dt)
        load_params(model, cfg, seed, dt)
        model.train()
        if tag == "f64":
            loss, stats, _ = model(speech.to(dt), slen, text, tlen)
        else:
            # shim: attention.py:79-81 takes the masking constant from numpy.finfo of the scores' dtype,
            # and numpy has no bfloat16 -- the scores enter the unchanged masking + softmax in fp32
            # (where autocast runs softmax anyway); P.V and every projection stay bf16 autocast ops
            from espnet.nets.pytorch_backend.transformer.attention import MultiHeadedAttention as _MHA
            fa = _MHA.forward_attention
            _MHA.forward_attention = lambda self, v, s, m: fa(self, v, s.float(), m)
            try:
                with torch.autocast("cpu", dtype=torch.bfloat16):
                    loss, stats, _ = model(speech.to(dt), slen, text, tlen)
            finally:
                _MHA.forward_attention = fa
        loss.backward()
        out[f"loss_{tag}"] = np.float64(loss.item())
        for n, p in model.named_parameters():
            gg = p.grad.detach().double().reshape(-1)
            if tag == "f64":
                grads[n] = gg
            else:
                ref = grads[n]
                den = float(gg.norm() * ref.norm())
                out[f"cos_amp/{n}"] = np.float64(float(gg @ ref) / den if den > 0 else 1.0)
                out[f"dn_amp/{n}"] = np.float64(abs(float(gg.norm()) - float(ref.norm())) / max(float(ref.norm()), 1e-300))
        print(f"{name} {tag}: loss {loss.item():.6f} ({_t.time() - t0:.1f} s)", flush=True)
        del model
    worst = min((float(v), k) for k, v in out.items() if k.startswith("cos_amp/"))
    print(f"{name}: worst autocast cosine {worst}", flush=True)
    out.update(lens=np.array(lens), ulens=np.array(ulens), seed=np.int64(seed), B=np.int64(B), T=np.int64(T))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


def c2_cfg(rel_pos_type):
    return O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=256, attention_heads=4, linear_units=1024,
                                                   num_blocks=12, rel_pos_type=rel_pos_type),
                      dec=O.DecCfg(attention_heads=4, linear_units=2048, num_blocks=6))


def long_cfg(rel_pos_type):
    """The long-utterance fixtures' model: C2's layer shapes (d = 256, H = 4, d_k = 64, FF 1024), 2 encoder and
    2 decoder blocks (tests/helpers.long_cfg)."""
    return O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=256, attention_heads=4, linear_units=1024,
                                                   num_blocks=2, rel_pos_type=rel_pos_type),
                      dec=O.DecCfg(attention_heads=4, linear_units=1024, num_blocks=2))


SLURP_YAML = "egs2/slurp/asr1/conf/tuning/train_asr_conformer.yaml"


def slurp_config():
    """The SLURP recipe's training config as the reference resolves it (config.yaml fields).

    egs2/slurp/asr1/run.sh:14-31 trains with --feats_type fbank_pitch (83-dim Kaldi fbank +
    pitch, so asr.sh passes --input_size=83, asr.sh:1034-1042) and --feats_normalize
    utterance_mvn (the default normalize, asr.sh:1046-1049); the YAML has no rel_pos_type, so
    ConformerEncoder's default "legacy" applies (conformer_encoder.py:98,116-120)."""
    import yaml
    with open(os.path.join(refshim.REF, SLURP_YAML)) as f:
        conf = yaml.safe_load(f)
    keys = ("encoder", "encoder_conf", "decoder", "decoder_conf", "model_conf", "specaug", "specaug_conf",
            "optim", "optim_conf", "scheduler", "scheduler_conf", "max_epoch", "best_model_criterion",
            "keep_nbest_models")
    resolved = {k: conf[k] for k in keys if k in conf}
    resolved.update(input_size=83, normalize="utterance_mvn", normalize_conf={}, ctc_conf={}, frontend=None,
                    token_list_size=600, source=SLURP_YAML + " + egs2/slurp/asr1/run.sh (fbank_pitch, utterance_mvn)")
    return resolved


def build_reference_from_config(conf, V):
    """ASRTask.build_model (espnet2/tasks/asr.py:439-562) steps 1-7 replayed on the reference's
    own classes: espnet2.tasks.asr itself does not import in this fork (asr.py:27 imports
    espnet/nets/pytorch_backend/conformer/contextual_block_encoder_layer.py, which is absent)."""
    enc_cls = {"conformer": ConformerEncoder, "transformer": TransformerEncoder}[conf["encoder"]]
    spec = SpecAug(**conf["specaug_conf"]) if conf.get("specaug") == "specaug" else None
    norm = UtteranceMVN(**conf["normalize_conf"]) if conf.get("normalize") == "utterance_mvn" else None
    enc = enc_cls(input_size=conf["input_size"], **conf["encoder_conf"])
    dec = TransformerDecoder(vocab_size=V, encoder_output_size=enc.output_size(), **conf["decoder_conf"])
    ctc = CTC(odim=V, encoder_output_size=enc.output_size(), **conf["ctc_conf"])
    return ESPnetASRModel(vocab_size=V, frontend=None, specaug=spec, normalize=norm, preencoder=None, encoder=enc,
                          postencoder=None, decoder=dec, ctc=ctc, joint_network=None, token_list=token_list(V),
                          **conf["model_conf"])


def slurp_cfg_from_config(conf, V, dropout_zero=False):
    e, d = conf["encoder_conf"], conf["decoder_conf"]
    z = (lambda x: 0.0) if dropout_zero else (lambda x: x)
    return O.ModelCfg(
        vocab_size=V,
        enc=O.EncCfg(input_size=conf["input_size"], output_size=e["output_size"], attention_heads=e["attention_heads"],
                     linear_units=e["linear_units"], num_blocks=e["num_blocks"], dropout_rate=z(e["dropout_rate"]),
                     positional_dropout_rate=z(e["positional_dropout_rate"]),
                     attention_dropout_rate=z(e["attention_dropout_rate"]),
                     rel_pos_type=e.get("rel_pos_type", "legacy"), macaron_style=e["macaron_style"],
                     use_cnn_module=e["use_cnn_module"], cnn_module_kernel=e["cnn_module_kernel"],
                     input_layer=e.get("input_layer", "conv2d")),
        dec=O.DecCfg(attention_heads=d["attention_heads"], linear_units=d["linear_units"], num_blocks=d["num_blocks"],
                     dropout_rate=z(d["dropout_rate"]), positional_dropout_rate=z(d["positional_dropout_rate"]),
                     self_attention_dropout_rate=z(d["self_attention_dropout_rate"]),
                     src_attention_dropout_rate=z(d["src_attention_dropout_rate"])),
        ctc_weight=conf["model_conf"]["ctc_weight"], lsm_weight=conf["model_conf"]["lsm_weight"],
        length_normalized_loss=conf["model_conf"]["length_normalized_loss"])


def slurp_yaml_fixture():
    """The SLURP recipe config end to end (VERDICT r1 'missing' 1): the resolved config as JSON
    (data: the GPU box has no /root/reference), the reference model's state_dict key/shape
    list, and full-size (B=2, T=1500, 83-dim) fp32/fp64 reference results for
      * the YAML model exactly as configured, in eval mode (validate_one_epoch: dropout and
        SpecAug off, BatchNorm running statistics);
      * the same architecture with every dropout rate 0 and SpecAug off, in train mode
        (BatchNorm batch statistics), with every parameter gradient summarised."""
    import json
    V = 600
    conf = slurp_config()
    ref = build_reference_from_config(conf, V)
    sd = ref.state_dict()
    cfg = slurp_cfg_from_config(conf, V)
    P = O.deterministic_params(cfg, 0)
    assert set(P) == set(sd), set(P) ^ set(sd)
    conf["reference_state_dict"] = [[k, list(v.shape)] for k, v in sd.items()]
    conf["reference_num_params"] = int(sum(p.numel() for p in ref.parameters()))
    conf["reference_modules"] = {"encoder.encoders.0.self_attn": type(ref.encoder.encoders[0].self_attn).__name__,
                                 "encoder.embed.1": type(ref.encoder.embed.out[1]).__name__
                                 if hasattr(ref.encoder.embed, "out") else ""}
    with open(os.path.join(HERE, "slurp_asr_conformer_config.json"), "w") as f:
        json.dump(conf, f, indent=1)
    print("slurp config:", conf["reference_num_params"], "params", conf["reference_modules"])
    del ref
    fullsize_train_fixture("slurp_yaml_eval", cfg, seed=61, with_grads=False, train=False,
                           build=lambda: build_reference_from_config(conf, V))
    conf0 = json.loads(json.dumps(conf))
    for sec in ("encoder_conf", "decoder_conf"):
        for k in list(conf0[sec]):
            if k.endswith("dropout_rate"):
                conf0[sec][k] = 0.0
    conf0["specaug"] = None
    fullsize_train_fixture("slurp_yaml_train", slurp_cfg_from_config(conf, V, dropout_zero=True), seed=62,
                           build=lambda: build_reference_from_config(conf0, V))


LIBRISPEECH_YAML = "egs2/librispeech/asr1/conf/tuning/train_asr_conformer.yaml"


def librispeech_config():
    """The LibriSpeech-960 Conformer recipe's training config (the C4 corpus; run.sh's asr_config): d = 512,
    H = 8, FF 2048, 12 blocks, input_layer conv2d6, macaron_style false, no rel_pos_type (the legacy default),
    nbpe 5000 (run.sh).  asr.sh feeds it raw audio through DefaultFrontend (80 log-mel) + global_mvn; here the
    80-dim features are the input and utterance_mvn the normalisation (the front end and GlobalMVN have their
    own fixture, frontend.npz)."""
    import yaml
    with open(os.path.join(refshim.REF, LIBRISPEECH_YAML)) as f:
        conf = yaml.safe_load(f)
    keys = ("encoder", "encoder_conf", "decoder", "decoder_conf", "model_conf", "specaug", "specaug_conf",
            "optim", "optim_conf", "scheduler", "scheduler_conf", "max_epoch", "best_model_criterion",
            "keep_nbest_models", "accum_grad")
    resolved = {k: conf[k] for k in keys if k in conf}
    resolved.update(input_size=80, normalize="utterance_mvn", normalize_conf={}, ctc_conf={}, frontend=None,
                    token_list_size=5000, source=LIBRISPEECH_YAML + " + egs2/librispeech/asr1/run.sh (nbpe 5000)")
    return resolved


def librispeech_yaml_fixture():
    """The LibriSpeech Conformer recipe config end to end: the resolved config + the reference model's
    state_dict layout as JSON, and the dropout-free / SpecAug-off architecture's full-size (B=2, T=1500) fp32 /
    fp64 training step with every gradient summarised (input_layer conv2d6, no macaron FFN, legacy rel-pos)."""
    import json
    V = 5000
    conf = librispeech_config()
    ref = build_reference_from_config(conf, V)
    sd = ref.state_dict()
    cfg = slurp_cfg_from_config(conf, V)
    P = O.deterministic_params(cfg, 0)
    assert set(P) == set(sd), set(P) ^ set(sd)
    conf["reference_state_dict"] = [[k, list(v.shape)] for k, v in sd.items()]
    conf["reference_num_params"] = int(sum(p.numel() for p in ref.parameters()))
    conf["reference_modules"] = {"encoder.embed": type(ref.encoder.embed).__name__,
                                 "encoder.encoders.0.self_attn": type(ref.encoder.encoders[0].self_attn).__name__}
    with open(os.path.join(HERE, "librispeech_asr_conformer_config.json"), "w") as f:
        json.dump(conf, f, indent=1)
    print("librispeech config:", conf["reference_num_params"], "params", conf["reference_modules"])
    del ref
    conf0 = json.loads(json.dumps(conf))
    for sec in ("encoder_conf", "decoder_conf"):
        for k in list(conf0[sec]):
            if k.endswith("dropout_rate"):
                conf0[sec][k] = 0.0
    conf0["specaug"] = None
    fullsize_train_fixture("librispeech_yaml_train", slurp_cfg_from_config(conf, V, dropout_zero=True), seed=64,
                           ulens=(60, 45), build=lambda: build_reference_from_config(conf0, V))


def frontend_fixture():
    """Front end: the reference Stft, the LogMel forward (with the
    oracle's restated mel matrix injected: librosa is absent) and GlobalMVN on seeded audio."""
    import tempfile

    from espnet2.layers.global_mvn import GlobalMVN
    from espnet2.layers.log_mel import LogMel
    from espnet2.layers.stft import Stft

    from oracle import frontend_cpu as FE
    g = torch.Generator().manual_seed(77)
    lens = torch.tensor([3000, 2571, 1234])
    x = torch.randn(3, 3000, generator=g) * 0.3
    for b, n in enumerate(lens.tolist()):
        x[b, n:] = 0.0
    st = Stft(n_fft=512, hop_length=128)
    spec, olens = st(x, lens)
    ospec, oolens = FE.stft(x, lens, 512, 128)
    assert torch.equal(olens, oolens) and torch.allclose(spec, ospec, rtol=0, atol=1e-5)
    power = spec[..., 0] ** 2 + spec[..., 1] ** 2
    melmat = torch.from_numpy(FE.mel_filters(16000, 512, 80, 0.0, 8000.0).T).float()
    lm = LogMel.__new__(LogMel)
    torch.nn.Module.__init__(lm)
    lm.register_buffer("melmat", melmat)
    lm.log_base = None
    lm.mel_options = {}
    feats, flens = lm(power, olens)
    assert torch.allclose(feats, FE.log_mel(power, olens, melmat), rtol=0, atol=1e-5)
    stats = {"count": np.float64(1234.0), "sum": np.random.RandomState(3).randn(80) * 50.0,
             "sum_square": np.random.RandomState(4).rand(80) * 9e4 + 2e4}
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "feats_stats.npz")
        np.savez(path, **stats)
        gm = GlobalMVN(path)
        normed, _ = gm(feats.clone(), flens)
    mean, std = FE.global_mvn_stats(stats)
    assert torch.allclose(normed, FE.global_mvn(feats, flens, mean, std), rtol=0, atol=1e-5)
    np.savez_compressed(os.path.join(HERE, "frontend.npz"), x=x.numpy(), lens=lens.numpy(),
                        spec=spec.numpy(), olens=olens.numpy(), melmat=melmat.numpy(), feats=feats.numpy(),
                        stat_count=stats["count"], stat_sum=stats["sum"], stat_sum_square=stats["sum_square"],
                        normed=normed.numpy())
    print("frontend", tuple(spec.shape), tuple(feats.shape))


def checkpoint_fixture():
    """Checkpoint interop.  checkpoint_ref.pth is what the reference's
    Trainer writes after an epoch (trainer.py:340-352): a tiny Conformer after two steps of the
    reference's own clip + Adam + WarmupLR, and a Reporter holding one epoch of train / valid
    stats.  checkpoint_ref_meta.json: the parameter names in optimizer order and the values
    the tests check.  The reverse direction is checked here (the reference cannot be imported
    by the tests): our resume() of that file followed by our save_checkpoint() is loaded back
    by the reference's own Trainer.resume into fresh reference objects, and every tensor,
    the optimizer / scheduler state and the reporter must come back identical."""
    import json
    import tempfile

    from espnet2.train.reporter import Reporter
    from espnet2.train.trainer import Trainer as RefTrainer

    cfg = small_cfg("latest", D=16, blocks=1, V=12)
    model = build_reference(cfg)
    load_params(model, cfg, 7)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=0.002, betas=(0.9, 0.98), eps=1e-9, weight_decay=1e-6)
    sch = WarmupLR(opt, warmup_steps=10)
    rep = Reporter()
    rep.set_epoch(1)
    with rep.observe("train") as sub:
        for step in range(2):
            speech, slen, text, tlen = O.synthetic_batch(2, 48, 80, cfg.vocab_size, [48, 40], [4, 3], 200 + step)
            loss, stats, weight = model(speech, slen, text, tlen)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0)
            opt.step()
            sch.step()
            opt.zero_grad()
            sub.register({k: v for k, v in stats.items() if v is not None}, weight)
            sub.next()
    with rep.observe("valid") as sub:
        sub.register({"acc": 0.25, "loss": 3.5})
        sub.next()
    ckpt = {"model": model.state_dict(), "reporter": rep.state_dict(), "optimizers": [opt.state_dict()],
            "schedulers": [sch.state_dict()], "scaler": None}
    path = os.path.join(HERE, "checkpoint_ref.pth")
    torch.save(ckpt, path)
    names = [n for n, _ in model.named_parameters()]
    meta = {"param_names": names, "cfg": {"D": 16, "blocks": 1, "V": 12}, "lr": opt.param_groups[0]["lr"],
            "last_epoch": sch.last_epoch, "adam_step": float(opt.state_dict()["state"][0]["step"]),
            "train_loss": float(rep.get_value("train", "loss")), "valid_acc": float(rep.get_value("valid", "acc"))}
    with open(os.path.join(HERE, "checkpoint_ref_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)

    # reverse direction: ours -> reference
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from tests.helpers import build_model
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR as OurWarmupLR
    from espnet_slurp_amd.train import checkpoint as CK
    from espnet_slurp_amd.train.reporter import Reporter as OurReporter
    ours = build_model(cfg, torch.device("cpu"))
    oopt = FusedAdam(ours.parameters(), ours.flat, lr=0.002, betas=(0.9, 0.98), eps=1e-9, weight_decay=1e-6)
    osch = OurWarmupLR(oopt, warmup_steps=10)
    orep = OurReporter()
    CK.resume(path, ours, orep, [oopt], [osch], None, ngpu=0)
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "checkpoint.pth")
        CK.save_checkpoint(out, ours, orep, [oopt], [osch])
        m2 = build_reference(cfg)
        o2 = torch.optim.Adam(m2.parameters(), lr=0.1)
        s2 = WarmupLR(o2, warmup_steps=99)
        r2 = Reporter()
        # torch >= 2.6 loads weights_only by default: the reference's own resume needs the
        # reporter's timedelta / numpy stat types allow-listed even for its own checkpoints
        with torch.serialization.safe_globals(CK._safe_globals()):
            RefTrainer.resume(out, m2, r2, [o2], [s2], None, ngpu=0)
    for k, v in model.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k
    a, b = opt.state_dict(), o2.state_dict()
    assert a["param_groups"] == b["param_groups"], (a["param_groups"], b["param_groups"])
    for i in a["state"]:
        for k in ("step", "exp_avg", "exp_avg_sq"):
            assert torch.equal(a["state"][i][k], b["state"][i][k]), (i, k)
    assert sch.state_dict() == s2.state_dict(), (sch.state_dict(), s2.state_dict())
    assert rep.state_dict() == r2.state_dict()
    print("checkpoint: ref -> ours -> ref round trip identical;", os.path.getsize(path), "bytes")


TRAINRUN_TRAIN = [([96, 90, 71], [6, 5, 4], 300), ([96, 96, 80], [6, 3, 5], 301), ([88, 70, 64], [5, 5, 2], 302)]
TRAINRUN_VALID = [([96, 81, 77], [6, 4, 5], 310), ([90, 60, 50], [3, 5, 4], 311)]


def trainrun_batches(spec, epoch=0):
    """(utt_ids, batch) lists of the Trainer.run fixture; the train order rotates per epoch."""
    out = []
    for i, (lens, ulens, seed) in enumerate(spec):
        speech, slen, text, tlen = O.synthetic_batch(len(lens), max(lens), 80, 32, lens, ulens, seed)
        out.append(([f"u{seed}_{k}" for k in range(len(lens))],
                    dict(speech=speech, speech_lengths=slen, text=text, text_lengths=tlen)))
    r = epoch % len(out)
    return out[r:] + out[:r]


TRAINRUN_OPTS = dict(max_epoch=3, seed=0, keep_nbest_models=[1, 2], nbest_averaging_interval=2, patience=None,
                     early_stopping_criterion=("valid", "loss", "min"),
                     best_model_criterion=[("valid", "acc", "max"), ("valid", "loss", "min"), ("train", "loss", "min")],
                     val_scheduler_criterion=("valid", "loss"))


def trainrun_fixture():
    """The reference's epoch driver (VERDICT r2 'next' 6): Trainer.run (trainer.py:154-447) with
    train_one_epoch + validate_one_epoch (:724-772) on the small golden model (dropout 0, no
    SpecAug), 3 epochs of 3 train / 2 valid batches, Adam + WarmupLR + clip 5, best-model links,
    n-best pruning (keep 1 and 2) and n-best averaging every 2 epochs.  Stored (JSON): the
    reporter's per-epoch train / valid values, the files Trainer.run left in output_dir and the
    targets of its links."""
    import json
    import tempfile
    from pathlib import Path

    from espnet2.iterators.abs_iter_factory import AbsIterFactory
    from espnet2.train.distributed_utils import DistributedOption
    from espnet2.train.trainer import Trainer as RefTrainer
    from espnet2.train.trainer import TrainerOptions as RefOptions

    class Factory(AbsIterFactory):
        def __init__(self, spec, dtype):
            self.spec, self.dtype = spec, dtype

        def build_iter(self, epoch, shuffle=None):
            return [(ids, dict(b, speech=b["speech"].to(self.dtype))) for ids, b in trainrun_batches(self.spec, epoch)]

    cfg = small_cfg("latest")
    runs = {}
    # the same run in fp32 (the fixture) and in fp64 (round 6: the bar the GPU's values are gated against,
    # with the fp32 run's own distance to it as the allowance -- the rule of every other gate)
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        model = build_reference(cfg).to(dt)
        load_params(model, cfg, 21, dt)
        opt = torch.optim.Adam(model.parameters(), lr=0.002, betas=(0.9, 0.98), eps=1e-9, weight_decay=1e-6)
        sch = WarmupLR(opt, warmup_steps=10)
        with tempfile.TemporaryDirectory() as td:
            o = RefOptions(ngpu=0, resume=True, use_amp=False, train_dtype=str(dt).split(".")[1], grad_noise=False,
                           accum_grad=1, grad_clip=5.0, grad_clip_type=2.0, log_interval=None, no_forward_run=False,
                           use_matplotlib=False, use_tensorboard=False, use_wandb=False, output_dir=td,
                           sharded_ddp=False, unused_parameters=False, wandb_model_log_interval=-1,
                           create_graph_in_tensorboard=False, **TRAINRUN_OPTS)
            RefTrainer.run(model=model, optimizers=[opt], schedulers=[sch],
                           train_iter_factory=Factory(TRAINRUN_TRAIN, dt), valid_iter_factory=Factory(TRAINRUN_VALID, dt),
                           plot_attention_iter_factory=None, trainer_options=o,
                           distributed_option=DistributedOption(distributed=False, ngpu=0))
            out = Path(td)
            from espnet_slurp_amd.train.checkpoint import safe_load
            rep = safe_load(out / "checkpoint.pth")["reporter"]
            values = {}
            for e, per in rep["stats"].items():
                values[str(e)] = {ph: {k: float(v) for k, v in d.items() if k in ("loss", "loss_att", "loss_ctc",
                                                                                    "acc", "optim0_lr0")}
                                  for ph, d in per.items() if ph in ("train", "valid")}
            runs[tag] = (values, sorted(p.name for p in out.iterdir()),
                         {p.name: str(p.readlink()) for p in out.iterdir() if p.is_symlink()})
    values, files, links = runs["f32"]
    assert runs["f64"][1] == files and runs["f64"][2] == links, (runs["f64"][1:], files, links)
    meta = {"values": values, "values_f64": runs["f64"][0], "files": files, "links": links, "seed": 21,
            "opts": TRAINRUN_OPTS,
            "adam": {"lr": 0.002, "betas": [0.9, 0.98], "eps": 1e-9, "weight_decay": 1e-6}, "warmup_steps": 10}
    for e, per in values.items():
        for ph, vals in per.items():
            print(e, ph, {k: f"{abs(v - runs['f64'][0][e][ph][k]):.2e}" for k, v in vals.items()})
    with open(os.path.join(HERE, "trainrun_ref.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("trainrun:", files, links)
    print(json.dumps(values, indent=1)[:1500])


if __name__ == "__main__":
    which = sys.argv[1:] or ["ctc", "align", "specaug", "small", "c1", "train", "full", "frontend", "checkpoint"]
    if "frontend" in which:
        frontend_fixture()
    if "checkpoint" in which:
        checkpoint_fixture()
    if "ctc" in which:
        ctc_fixture()
    if "align" in which:
        align_fixture()
    if "align_c2" in which:
        align_c2_fixture()
    if "specaug" in which:
        specaug_fixture()
    if "small" in which:
        model_fixture("model_small_latest", small_cfg("latest"), 3, 120, [120, 97, 64], [9, 5, 7], 1)
        model_fixture("model_small_legacy", small_cfg("legacy"), 3, 120, [120, 97, 64], [9, 5, 7], 2)
    if "long" in which:  # long utterances (VERDICT r5 'missing' 1): T' = 875 latest / legacy, T' = 1100 latest,
        # d_k = 64 (the rel-pos kernels' head size), 2 encoder / 2 decoder blocks
        for name, rel, T, lens in (("long_t875_latest", "latest", 3503, (3503, 3000)),
                                   ("long_t875_legacy", "legacy", 3503, (3503, 3000)),
                                   ("long_t1100_latest", "latest", 4403, (4403, 3803))):
            fullsize_train_fixture(name, long_cfg(rel), B=2, T=T, lens=lens, ulens=(60, 45), seed=91)
    if "interctc" in which:  # intermediate CTC (conformer_encoder.py:283-285,333-350; espnet_model.py:222-245)
        cfg = small_cfg("latest", blocks=3)
        cfg.enc.interctc_layer_idx = (1, 2)
        cfg.interctc_weight = 0.3
        model_fixture("model_small_interctc", cfg, 3, 120, [120, 97, 64], [9, 5, 7], 8)
        cfg.enc.interctc_use_conditioning = True  # + self-conditioning (conformer_encoder.py:343-350)
        model_fixture("model_small_interctc_cond", cfg, 3, 120, [120, 97, 64], [9, 5, 7], 9)
    if "conv2d6" in which:  # input_layer conv2d6 (Conv2dSubsampling6, the LibriSpeech Conformer recipe's)
        cfg = small_cfg("latest")
        cfg.enc.input_layer = "conv2d6"
        model_fixture("model_small_conv2d6", cfg, 3, 120, [120, 97, 64], [9, 5, 7], 6)
    if "lnorm" in which:  # length_normalized_loss=True (LabelSmoothingLoss normalize_length)
        cfg = small_cfg("latest")
        cfg.length_normalized_loss = True
        model_fixture("model_small_lnorm", cfg, 3, 120, [120, 97, 64], [9, 5, 7], 4)
    if "c1" in which:
        c1 = O.ModelCfg(vocab_size=30, enc=O.EncCfg(kind="transformer", output_size=256, attention_heads=4,
                                                     linear_units=1024, num_blocks=4),
                        dec=None, ctc_weight=1.0)
        model_fixture("model_c1_transformer_ctc", c1, 2, 200, [200, 173], [10, 7], 5, with_grads=False)
    if "train" in which:
        train_step_fixture()
    if "full" in which:
        fullsize_fixture()
    if "fullgrad" in which:  # full-size C2 gradients, latest and legacy (round 2)
        fullsize_train_fixture("fullsize_c2_grad_latest", c2_cfg("latest"), seed=42)
        fullsize_train_fixture("fullsize_c2_grad_legacy", c2_cfg("legacy"), seed=44)
    if "c4" in which:  # C4 shape: d=512, H=8, FF=2048, 17 blocks, latest; forward loss
        c4 = O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=512, attention_heads=8, linear_units=2048,
                                                     num_blocks=17, rel_pos_type="latest"),
                        dec=O.DecCfg(attention_heads=8, linear_units=2048, num_blocks=6))
        fullsize_train_fixture("fullsize_c4_loss", c4, seed=51, with_grads=False)
    if "c4grad" in which:  # C4 shape with every parameter gradient (VERDICT r2 'missing' 3)
        c4 = O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=512, attention_heads=8, linear_units=2048,
                                                     num_blocks=17, rel_pos_type="latest"),
                        dec=O.DecCfg(attention_heads=8, linear_units=2048, num_blocks=6))
        fullsize_train_fixture("fullsize_c4_grad_latest", c4, seed=53)
    if "c5grad" in which:  # C5 shape (SLURP-entity: d=512, H=8, FF 2048, 12 blocks, latest) with every
        # parameter gradient (VERDICT r3 'next' 1a): the fp32 step and the bf16 step are gated against it
        c5 = O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=512, attention_heads=8, linear_units=2048,
                                                     num_blocks=12, rel_pos_type="latest"),
                        dec=O.DecCfg(attention_heads=8, linear_units=2048, num_blocks=6))
        fullsize_train_fixture("fullsize_c5_grad_latest", c5, seed=57)
    if "c5amp" in which:  # the reference's bf16-autocast step at the C5 shape (the bf16 gate's bar)
        c5 = O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=512, attention_heads=8, linear_units=2048,
                                                     num_blocks=12, rel_pos_type="latest"),
                        dec=O.DecCfg(attention_heads=8, linear_units=2048, num_blocks=6))
        amp_reference_fixture("fullsize_c5_amp_ref", c5, seed=57)
    if "slurp" in which:
        slurp_yaml_fixture()
    if "trainrun" in which:
        trainrun_fixture()
    if "librispeech" in which:
        librispeech_yaml_fixture()
