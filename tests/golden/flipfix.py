"""ReLU-decision flip records for the full-size gradient fixtures (test infrastructure only).

At full size a few ReLU pre-activations sit within fp32 rounding of 0: Conv2dSubsampling's two
ReLUs (subsampling.py:53-87) and the decoder FFN's ReLU (positionwise_feed_forward.py:30-32,
transformer_decoder.py DecoderLayer).  Two correct fp32 implementations can land on opposite sides
of 0 there, and each such discrete decision moves single gradient elements of the tensors right
below it -- conv.0 (the first Conv2d) and the decoder layer's norm3 -- by far more than fp32
rounding.  Instead of widening the slice gate, the fixtures record every decision within tau of 0
(tau = 4x the largest |fp32 - fp64| pre-activation difference of the site in the reference's own
fp32 run) with its exact first-order contribution to the gated slice elements, computed from the
fp64 run:

  conv1 flip at (b, c, t1, f1), g1 = dL/d relu1:   d conv.0.weight[c, 0, i, j] = g1 x[b, 2t1+i, 2f1+j],
                                                  d conv.0.bias[c] = g1
  conv2 flip at (b, o, t2, f2), g2 = dL/d relu2:   d relu1[b, c, 2t2+kt, 2f2+kf] = g2 W2[o, c, kt, kf], through
                                                  relu1's (fp64) mask into conv.0 as above; and (round 6)
                                                  d conv.2.weight[o, c, kt, kf] = g2 relu1[b, c, 2t2+kt, 2f2+kf],
                                                  d conv.2.bias[o] = g2 (conv2d6: 5 x 5, stride 3)
  decoder flip at (b, l, u), g = dL/d relu:        d norm3.weight[c] = g W1[u, c] xhat[b, l, c],
                                                  d norm3.bias[c] = g W1[u, c]; and (round 6)
                                                  d w_1.weight[u, c] = g y[b, l, c], d w_1.bias[u] = g

The GPU test reads its own decisions at those positions (tests/helpers.FlipProbe) and subtracts
(s_gpu - s64) x contribution; the fixture's fp32 slices are corrected the same way with the fp32
run's decisions ("gs_f32c/<name>"), so the gate max(1e-4, 2 e_ref) compares like with like.

Fixture keys, per gated tensor n and site s (conv1, conv2, dec<l>):
  flip/<n>/<s>/idx  int64 [k, 3]   (b, c, t, f)->(b, c_or_o, t, f) for conv sites: [k, 4]; (b, l, u) for decoder
  flip/<n>/<s>/s64  int8 [k]       fp64 decision (pre > 0)
  flip/<n>/<s>/s32  int8 [k]       the reference's fp32 decision
  flip/<n>/<s>/c    float64 [k, S] contribution of an "on" decision to the S slice elements
  gs_f32c/<n>                      the fp32 slice with its own flips corrected to the fp64 decisions
  flip/<n>/<s>/cp   float64 [k, 8] (round 6) the contribution to the 8 fingerprint projections (fingerprint.py),
                                   formed over every element of the tensor; fp_f32c/<n> the fp32 projections
                                   corrected like gs_f32c.  (Row-norm fingerprints are not flip-corrected:
                                   the gate skips them on these tensors, whose projections it corrects.)
"""
import numpy as np
import torch

CONV_TENSORS = ("encoder.embed.conv.0.weight", "encoder.embed.conv.0.bias")
# round 6: a flip at the second ReLU also moves the second convolution's own gradient (row o of conv.2), and a
# decoder flip the FFN's w_1 row u -- single rows, which the whole-tensor row-norm fingerprint sees
CONV2_TENSORS = ("encoder.embed.conv.2.weight", "encoder.embed.conv.2.bias")


class Records:
    """Per-run (one precision) tensors of the sites, filled by a reference or an oracle adapter:
    conv: x [B, T, F] (subsampling input), pre1, out1, pre2, out2 (NCHW; out* keep .grad), W2;
    dec[l]: y [B, L, D] (FFN input = norm3 output), h [B, L, FF] (pre-activation), r (ReLU output,
    keeps .grad), W1 [FF, D], gamma / beta of norm3."""

    def __init__(self):
        self.conv = {}
        self.dec = {}

    def detach(self):
        """Drop the autograd graph after backward (keep the values and the ReLU-output grads)."""
        def dd(d):
            out = {}
            for k, v in d.items():
                if torch.is_tensor(v):
                    out[k] = v.detach()
                    if k.startswith("out") or k == "r":
                        out[k + "_grad"] = v.grad.detach() if v.grad is not None else torch.zeros_like(v)
                else:
                    out[k] = v
            return out
        self.conv = dd(self.conv)
        self.dec = {l: dd(d) for l, d in self.dec.items()}
        return self


class ReferenceProbe:
    """Module hooks on the reference ESPnetASRModel (encoder.embed Conv2dSubsampling, decoder
    layers' feed_forward)."""

    def __init__(self, model):
        self.model = model
        self.rec = Records()
        self.h = []

    def __enter__(self):
        rec = self.rec
        emb = self.model.encoder.embed
        seq = emb.conv
        self.h.append(emb.register_forward_pre_hook(lambda m, a: rec.conv.__setitem__("x", a[0])))

        def keep(name):
            def hook(m, a, out):
                rec.conv[name] = out
                if name.startswith("out") and out.requires_grad:
                    out.retain_grad()
            return hook
        for i, name in ((0, "pre1"), (1, "out1"), (2, "pre2"), (3, "out2")):
            self.h.append(seq[i].register_forward_hook(keep(name)))
        rec.conv["W2"] = seq[2].weight
        dec = getattr(self.model, "decoder", None)
        if dec is not None:
            # PositionwiseFeedForward's activation is a default argument (positionwise_feed_forward.py:22):
            # ONE torch.nn.ReLU instance shared by every layer, so its hook files the output under the
            # layer whose w_1 ran last
            cur = [None]
            acts = {}
            for l, layer in enumerate(dec.decoders):
                ff = layer.feed_forward
                d = rec.dec.setdefault(l, {})
                d["W1"], d["gamma"], d["beta"] = ff.w_1.weight, layer.norm3.weight, layer.norm3.bias

                def w1_hook(m, a, out, d=d):
                    d["y"], d["h"] = a[0], out
                    cur[0] = d
                self.h.append(ff.w_1.register_forward_hook(w1_hook))
                acts[id(ff.activation)] = ff.activation

            def act_hook(m, a, out):
                if cur[0] is not None:
                    cur[0]["r"] = out
                    cur[0] = None
                    if out.requires_grad:
                        out.retain_grad()
            for act in acts.values():
                self.h.append(act.register_forward_hook(act_hook))
        return self

    def __exit__(self, *exc):
        for h in self.h:
            h.remove()


class OracleProbe:
    """The same records from the oracle restatement (oracle/espnet_cpu.py): wraps
    O.conv2d_subsampling and the decoder's O.ffn with copies that keep the intermediate tensors."""

    def __init__(self, O, P):
        self.O, self.P = O, P
        self.rec = Records()

    def __enter__(self):
        O, P, rec = self.O, self.P, self.rec
        F = torch.nn.functional
        self._sub, self._ffn = O.conv2d_subsampling, O.ffn

        def sub(P_, pre, x, mask, input_layer="conv2d"):
            rec.conv["x"] = x
            pre1 = F.conv2d(x.unsqueeze(1), P_[pre + ".conv.0.weight"], P_[pre + ".conv.0.bias"], stride=2)
            out1 = F.relu(pre1)
            pre2 = F.conv2d(out1, P_[pre + ".conv.2.weight"], P_[pre + ".conv.2.bias"],
                            stride=2 if input_layer == "conv2d" else 3)
            out2 = F.relu(pre2)
            for v in (out1, out2):
                if v.requires_grad:
                    v.retain_grad()
            rec.conv.update(pre1=pre1, out1=out1, pre2=pre2, out2=out2, W2=P_[pre + ".conv.2.weight"])
            b, c, t, f = out2.size()
            y = O.linear(P_, pre + ".out.0", out2.transpose(1, 2).contiguous().view(b, t, c * f))
            if input_layer == "conv2d":
                return y, mask[:, :, :-2:2][:, :, :-2:2]
            return y, mask[:, :, :-2:2][:, :, :-4:3]

        def ffn(P_, pre, x, act, p_drop=0.0, training=True):
            if not (pre.startswith("decoder.") and act == "relu"):
                return self._ffn(P_, pre, x, act, p_drop, training)
            l = int(pre.split(".")[2])
            lay = pre[: -len(".feed_forward")]
            h = O.linear(P_, pre + ".w_1", x)
            r = F.relu(h)
            if r.requires_grad:
                r.retain_grad()
            rec.dec[l] = dict(y=x, h=h, r=r, W1=P_[pre + ".w_1.weight"], gamma=P_[lay + ".norm3.weight"],
                              beta=P_[lay + ".norm3.bias"])
            return O.linear(P_, pre + ".w_2", O.dropout(r, p_drop, training))
        O.conv2d_subsampling, O.ffn = sub, ffn
        return self

    def __exit__(self, *exc):
        self.O.conv2d_subsampling, self.O.ffn = self._sub, self._ffn


def _near(pre64, pre32, factor=4.0):
    tau = factor * float((pre32.double() - pre64.double()).abs().max())
    return (pre64.abs() < tau).nonzero(), tau


def flip_records(r64: Records, r32: Records, slice_idx, out: dict, gs32: dict, log=print, prefix="", corr=None,
                 shapes=None, corr_fp=None):
    """Compute the flip records of module docstring from the fp64 / fp32 Records of one fixture and
    write them (and the corrected fp32 slices gs_f32c/<n>) into `out`.  slice_idx(name) -> the
    fixture's slice element indices; gs32[name] -> the fp32 slice values.  prefix: site-name prefix
    (one forward of several whose gradients add, e.g. "r0:" per data-parallel rank); corr: a dict
    that accumulates the fp32 corrections over such calls (gs_f32c written from the running sum).
    shapes: {name: numel} of the gated tensors -- when given, each site's contribution is also formed for
    EVERY element of the tensor and projected on the fingerprint vectors (fingerprint.py): "cp" [k, 8], and
    fp_f32c/<n> = the fp32 projections with the fp32 run's flips corrected (corr_fp accumulates like corr)."""
    import fingerprint as FP
    corr = {} if corr is None else corr
    corr_fp = {} if corr_fp is None else corr_fp
    sg = {}

    def allidx(name):
        return np.arange(shapes[name], dtype=np.int64) if shapes else None

    def signs(name):
        if name not in sg:
            sg[name] = FP.signs(name, shapes[name])
        return sg[name]

    def add(name, site, idx, s64, s32, c, cfull=None, cp=None, rows=None):
        """c: [k, S] contributions to the slice; cfull: [k, numel] to every element (small tensors) or cp:
        [k, N_PROJ] directly to the projections; rows: the row each site moves (row-sparse tensors)."""
        site = prefix + site
        out[f"flip/{name}/{site}/idx"] = idx.numpy().astype(np.int64)
        out[f"flip/{name}/{site}/s64"] = s64.numpy().astype(np.int8)
        out[f"flip/{name}/{site}/s32"] = s32.numpy().astype(np.int8)
        out[f"flip/{name}/{site}/c"] = c.numpy().astype(np.float64)
        if rows is not None:
            out[f"flip/{name}/{site}/rows"] = rows.numpy().astype(np.int64)
        ds = (s32.double() - s64.double())[:, None]  # fp32's flips relative to fp64
        corr[name] = corr.get(name, 0.0) + (ds * c).sum(0)
        if cfull is not None:
            cp = cfull @ signs(name).T  # [k, N_PROJ]
        if cp is not None:
            out[f"flip/{name}/{site}/cp"] = cp.numpy().astype(np.float64)
            corr_fp[name] = corr_fp.get(name, 0.0) + (ds * cp).sum(0)

    def row_cp(name, rows, vals):
        """projection contributions of sites that each move one row: vals [k, R] the row's values, rows [k]"""
        sgn = signs(name).view(FP.N_PROJ, -1, vals.shape[1])  # [P, rows, R]
        cp = torch.zeros(len(rows), FP.N_PROJ, dtype=torch.float64)
        for a in range(0, len(rows), 256):
            r = rows[a:a + 256]
            cp[a:a + 256] = torch.einsum("kj,pkj->kp", vals[a:a + 256], sgn[:, r, :])
        return cp

    if r64.conv:
        c64, c32 = r64.conv, r32.conv
        x = c64["x"].double()                      # [B, T, F]
        pre1 = c64["pre1"].double()                # [B, C, T1, F1]
        g1 = c64["out1_grad"].double()
        g2 = c64["out2_grad"].double()
        W2 = c64["W2"].double()                    # [O, C, 3, 3]

        def conv1_contrib(b, c, t1, f1, gg, iw, ib):
            wc, wi, wj = iw // 9, (iw % 9) // 3, iw % 3  # weight [C, 1, 3, 3] flat
            xw = x[b[:, None], 2 * t1[:, None] + wi[None], 2 * f1[:, None] + wj[None]]  # [k, S]
            cw = torch.where(c[:, None] == wc[None], gg[:, None] * xw, torch.zeros_like(xw))
            cb = torch.where(c[:, None] == ib[None], gg[:, None].expand(-1, len(ib)),
                             torch.zeros(len(b), len(ib), dtype=torch.float64))
            return cw, cb

        # the second convolution: 3 x 3 stride 2 (conv2d) or 5 x 5 stride 3 (conv2d6, Conv2dSubsampling6)
        k2 = W2.shape[2]
        s2 = {3: 2, 5: 3}[k2]

        def conv2_contrib(b, o, t2, f2, gg, iw, ib):
            wc, wi, wj = iw // 9, (iw % 9) // 3, iw % 3
            cw = torch.zeros(len(b), len(iw), dtype=torch.float64)
            cb = torch.zeros(len(b), len(ib), dtype=torch.float64)
            for kt in range(k2):
                for kf in range(k2):
                    tt, ff = s2 * t2 + kt, s2 * f2 + kf
                    # weight elements (c', i, j)
                    m = (pre1[b[:, None], wc[None], tt[:, None], ff[:, None]] > 0).double()
                    wv = W2[o[:, None], wc[None], kt, kf]
                    xv = x[b[:, None], 2 * tt[:, None] + wi[None], 2 * ff[:, None] + wj[None]]
                    cw += gg[:, None] * wv * m * xv
                    mb = (pre1[b[:, None], ib[None], tt[:, None], ff[:, None]] > 0).double()
                    cb += gg[:, None] * W2[o[:, None], ib[None], kt, kf] * mb
            return cw, cb

        iw = torch.from_numpy(slice_idx(CONV_TENSORS[0]))
        ib = torch.from_numpy(slice_idx(CONV_TENSORS[1]))
        # conv1 flips
        near, tau1 = _near(c64["pre1"], c32["pre1"])
        b, c, t1, f1 = near.unbind(1) if len(near) else (torch.zeros(0, dtype=torch.long),) * 4
        gg = g1[b, c, t1, f1]
        s64 = c64["pre1"][b, c, t1, f1] > 0
        s32 = c32["pre1"][b, c, t1, f1] > 0
        cw, cb = conv1_contrib(b, c, t1, f1, gg, iw, ib)
        fw = fb = None
        if shapes:
            fw, fb = conv1_contrib(b, c, t1, f1, gg, torch.from_numpy(allidx(CONV_TENSORS[0])),
                                   torch.from_numpy(allidx(CONV_TENSORS[1])))
        add(CONV_TENSORS[0], "conv1", near, s64, s32, cw, fw)
        add(CONV_TENSORS[1], "conv1", near, s64, s32, cb, fb)
        log(f"conv1: tau {tau1:.3g}, {len(b)} decisions, {(s64 != s32).sum().item()} flipped in fp32")
        # conv2 flips: through relu1's fp64 mask into conv.0
        near, tau2 = _near(c64["pre2"], c32["pre2"])
        b, o, t2, f2 = near.unbind(1) if len(near) else (torch.zeros(0, dtype=torch.long),) * 4
        gg = g2[b, o, t2, f2]
        s64 = c64["pre2"][b, o, t2, f2] > 0
        s32 = c32["pre2"][b, o, t2, f2] > 0
        cw, cb = conv2_contrib(b, o, t2, f2, gg, iw, ib)
        fw = fb = None
        if shapes:
            fw, fb = conv2_contrib(b, o, t2, f2, gg, torch.from_numpy(allidx(CONV_TENSORS[0])),
                                   torch.from_numpy(allidx(CONV_TENSORS[1])))
        add(CONV_TENSORS[0], "conv2", near, s64, s32, cw, fw)
        add(CONV_TENSORS[1], "conv2", near, s64, s32, cb, fb)
        # the same sites' direct share of conv.2's gradient: d W2[o, c, kt, kf] = g2 out1[b, c, s2 t2 + kt,
        # s2 f2 + kf], d b2[o] = g2 -- row o only
        out1 = c64["out1"].double()
        C = out1.shape[1]
        CK = C * k2 * k2
        j = torch.arange(CK)
        jc, jt, jf = j // (k2 * k2), (j % (k2 * k2)) // k2, j % k2
        i2 = torch.from_numpy(slice_idx(CONV2_TENSORS[0]))
        eo, ec, et, ef = i2 // CK, (i2 % CK) // (k2 * k2), (i2 % (k2 * k2)) // k2, i2 % k2
        xv = out1[b[:, None], ec[None], s2 * t2[:, None] + et[None], s2 * f2[:, None] + ef[None]]
        cw2 = torch.where(o[:, None] == eo[None], gg[:, None] * xv, torch.zeros_like(xv))
        ib2 = torch.from_numpy(slice_idx(CONV2_TENSORS[1]))
        cb2 = torch.where(o[:, None] == ib2[None], gg[:, None].expand(-1, len(ib2)),
                          torch.zeros(len(b), len(ib2), dtype=torch.float64))
        cpw2 = cpb2 = None
        if shapes:
            vals = gg[:, None] * out1[b[:, None], jc[None], s2 * t2[:, None] + jt[None], s2 * f2[:, None] + jf[None]]
            cpw2 = row_cp(CONV2_TENSORS[0], o, vals)
            cpb2 = row_cp(CONV2_TENSORS[1], o, gg[:, None])
        add(CONV2_TENSORS[0], "conv2", near, s64, s32, cw2, cp=cpw2, rows=o)
        add(CONV2_TENSORS[1], "conv2", near, s64, s32, cb2, cp=cpb2, rows=o)
        log(f"conv2: tau {tau2:.3g}, {len(b)} decisions, {(s64 != s32).sum().item()} flipped in fp32")
    for l, d64 in sorted(r64.dec.items()):
        d32 = r32.dec[l]
        lay = f"decoder.decoders.{l}"
        near, tau = _near(d64["h"], d32["h"])
        b, p, u = near.unbind(1) if len(near) else (torch.zeros(0, dtype=torch.long),) * 3
        g = d64["r_grad"].double()[b, p, u]
        s64 = d64["h"][b, p, u] > 0
        s32 = d32["h"][b, p, u] > 0
        W1 = d64["W1"].double()
        y = d64["y"].double()
        gam, bet = d64["gamma"].double(), d64["beta"].double()

        def dec_contrib(name, ci):
            c = g[:, None] * W1[u[:, None], ci[None]]
            if name.endswith("weight"):
                xhat = (y[b[:, None], p[:, None], ci[None]] - bet[ci][None]) / gam[ci][None]
                c = c * xhat
            return c
        for name in (lay + ".norm3.weight", lay + ".norm3.bias"):
            c = dec_contrib(name, torch.from_numpy(slice_idx(name)))
            cf = dec_contrib(name, torch.from_numpy(allidx(name))) if shapes else None
            add(name, f"dec{l}", near, s64, s32, c, cf)
        # the FFN's w_1 row u: d w_1.weight[u, c] = g y[b, p, c], d w_1.bias[u] = g
        D = y.shape[2]
        wn, bn = lay + ".feed_forward.w_1.weight", lay + ".feed_forward.w_1.bias"
        iw1 = torch.from_numpy(slice_idx(wn))
        yv = y[b[:, None], p[:, None], (iw1 % D)[None]]
        cw1 = torch.where(u[:, None] == (iw1 // D)[None], g[:, None] * yv, torch.zeros_like(yv))
        ib1 = torch.from_numpy(slice_idx(bn))
        cb1 = torch.where(u[:, None] == ib1[None], g[:, None].expand(-1, len(ib1)),
                          torch.zeros(len(b), len(ib1), dtype=torch.float64))
        cpw1 = cpb1 = None
        if shapes:
            cpw1 = row_cp(wn, u, g[:, None] * y[b, p, :])
            cpb1 = row_cp(bn, u, g[:, None])
        add(wn, f"dec{l}", near, s64, s32, cw1, cp=cpw1, rows=u)
        add(bn, f"dec{l}", near, s64, s32, cb1, cp=cpb1, rows=u)
        log(f"{lay}: tau {tau:.3g}, {len(b)} decisions, {(s64 != s32).sum().item()} flipped in fp32")
    for name, d in corr.items():
        out[f"gs_f32c/{name}"] = np.asarray(gs32[name], dtype=np.float64) - d.numpy()
    for name, d in corr_fp.items():
        out[f"fp_f32c/{name}"] = np.asarray(out[f"fp_f32/{name}"], dtype=np.float64) - d.numpy()
