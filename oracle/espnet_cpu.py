"""CPU oracle: a plain-PyTorch (CPU, fp32/fp64) restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may import this module, and only as the checker / CPU baseline.
The product package `espnet_slurp_amd` never imports it (a test enforces this).

It restates, functionally over a flat `state_dict`-keyed parameter dict, the reference's
`ESPnetASRModel.forward` training step (BriansIDP/espnet_slurp, read-only at
/root/reference).  Every function cites the reference file:line it follows.  The
arithmetic primitives (matmul, conv2d, softmax, ctc_loss, interpolate) are PyTorch CPU
ATen ops, exactly the third-party engine the reference itself calls (SURVEY.md §8(c):
torch 2.10.0 in this image).  The restatement is pinned against golden vectors
produced by importing the reference itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]


# ----------------------------------------------------------------------------- config
@dataclass
class EncCfg:
    kind: str = "conformer"          # conformer | transformer
    input_size: int = 80
    output_size: int = 256
    attention_heads: int = 4
    linear_units: int = 1024
    num_blocks: int = 12
    dropout_rate: float = 0.0
    positional_dropout_rate: float = 0.0
    attention_dropout_rate: float = 0.0
    rel_pos_type: str = "latest"     # latest | legacy (conformer only)
    macaron_style: bool = True
    use_cnn_module: bool = True
    cnn_module_kernel: int = 31
    max_pos_emb_len: int = 5000
    input_layer: str = "conv2d"      # conv2d | conv2d6 (Conv2dSubsampling6, subsampling.py:101-146)
    interctc_layer_idx: Tuple[int, ...] = ()  # intermediate CTC layers (conformer_encoder.py:283-285,333-350)
    interctc_use_conditioning: bool = False   # self-conditioning (conformer_encoder.py:343-350)


@dataclass
class DecCfg:
    attention_heads: int = 4
    linear_units: int = 2048
    num_blocks: int = 6
    dropout_rate: float = 0.0
    positional_dropout_rate: float = 0.0
    self_attention_dropout_rate: float = 0.0
    src_attention_dropout_rate: float = 0.0


@dataclass
class ModelCfg:
    vocab_size: int = 600
    enc: EncCfg = field(default_factory=EncCfg)
    dec: Optional[DecCfg] = field(default_factory=DecCfg)
    ctc_weight: float = 0.3
    interctc_weight: float = 0.0     # espnet_model.py:54,222-245
    lsm_weight: float = 0.1
    ignore_id: int = -1
    length_normalized_loss: bool = False
    blank_id: int = 0
    sos: int = -1                    # default vocab_size-1 (espnet_model.py:74-82)
    eos: int = -1

    def __post_init__(self):
        if self.sos < 0:
            self.sos = self.vocab_size - 1
        if self.eos < 0:
            self.eos = self.vocab_size - 1


# ----------------------------------------------------------------------------- masks
def make_pad_mask(lengths, maxlen: Optional[int] = None) -> torch.Tensor:
    """True at padded positions; nets_utils.py:64-176 (xs=None form)."""
    lengths = torch.as_tensor(lengths).long().cpu()
    if maxlen is None:
        maxlen = int(lengths.max())
    ar = torch.arange(maxlen, dtype=torch.int64)
    return ar[None, :] >= lengths[:, None]


def subsequent_mask(n: int) -> torch.Tensor:
    """transformer/mask.py:20-38."""
    return torch.tril(torch.ones(n, n, dtype=torch.bool))


def subsampled_lengths(lengths: torch.Tensor, T: int, input_layer: str = "conv2d") -> torch.Tensor:
    """Length of `mask[:, :, :-2:2][:, :, :-2:2]` (subsampling.py:87; conv2d6: `[:, :, :-2:2][:, :, :-4:3]`,
    :146) as counts."""
    m = ~make_pad_mask(lengths, T)
    m = m[:, :-2:2][:, :-2:2] if input_layer == "conv2d" else m[:, :-2:2][:, :-4:3]
    return m.sum(1)


# ----------------------------------------------------------------------------- pos enc
def _pe_rows(positions: torch.Tensor, d: int) -> torch.Tensor:
    """embedding.py:66-80 / 209-221: sin/cos table in fp32 on CPU."""
    pe = torch.zeros(positions.numel(), d)
    position = positions.to(torch.float32).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe


def abs_pos_table(T: int, d: int, max_len: int = 5000) -> torch.Tensor:
    """PositionalEncoding (embedding.py:48-94): pe[:T] of a max_len table, shape (1,T,d)."""
    n = max(max_len, T)
    return _pe_rows(torch.arange(0, n, dtype=torch.float32), d)[:T].unsqueeze(0)


def rel_pos_table_latest(T: int, d: int, max_len: int = 5000) -> torch.Tensor:
    """RelPositionalEncoding (embedding.py:173-244): (1, 2T-1, d), row k = PE(T-1-k)."""
    n = max(max_len, T)
    position = torch.arange(0, n, dtype=torch.float32)
    pos = _pe_rows(position, d)
    neg = torch.zeros(n, d)
    pm = position.unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    neg[:, 0::2] = torch.sin(-1 * pm * div_term)
    neg[:, 1::2] = torch.cos(-1 * pm * div_term)
    pe = torch.cat([torch.flip(pos, [0]), neg[1:]], dim=0).unsqueeze(0)
    c = pe.size(1) // 2
    return pe[:, c - T + 1: c + T]


def rel_pos_table_legacy(T: int, d: int, max_len: int = 5000) -> torch.Tensor:
    """LegacyRelPositionalEncoding (embedding.py:133-170): reversed positions, (1,T,d)."""
    n = max(max_len, T)
    return _pe_rows(torch.arange(n - 1, -1, -1.0, dtype=torch.float32), d)[:T].unsqueeze(0)


# ----------------------------------------------------------------------------- blocks
def linear(P: Params, pre: str, x, bias: bool = True):
    y = x @ P[pre + ".weight"].t()
    if bias:
        y = y + P[pre + ".bias"]
    return y


def layer_norm(P: Params, pre: str, x, eps: float = 1e-12):
    """layer_norm.py:12-38 (torch.nn.LayerNorm, eps=1e-12)."""
    return F.layer_norm(x, (x.size(-1),), P[pre + ".weight"], P[pre + ".bias"], eps)


def dropout(x, p: float, training: bool = True):
    return F.dropout(x, p, training) if (p > 0 and training) else x


def conv2d_subsampling(P: Params, pre: str, x, mask, input_layer: str = "conv2d"):
    """Conv2dSubsampling.forward, subsampling.py:53-87 (returns pre-pos-enc features); input_layer
    "conv2d6": Conv2dSubsampling6.forward, subsampling.py:101-146 (second conv 5 x 5, stride 3)."""
    x = x.unsqueeze(1)
    x = F.relu(F.conv2d(x, P[pre + ".conv.0.weight"], P[pre + ".conv.0.bias"], stride=2))
    s2 = 2 if input_layer == "conv2d" else 3
    x = F.relu(F.conv2d(x, P[pre + ".conv.2.weight"], P[pre + ".conv.2.bias"], stride=s2))
    b, c, t, f = x.size()
    x = linear(P, pre + ".out.0", x.transpose(1, 2).contiguous().view(b, t, c * f))
    if input_layer == "conv2d":
        return x, mask[:, :, :-2:2][:, :, :-2:2]
    return x, mask[:, :, :-2:2][:, :, :-4:3]


def rel_shift_latest(x):
    """RelPositionMultiHeadedAttention.rel_shift, attention.py:240-263."""
    zero_pad = torch.zeros((*x.size()[:3], 1), dtype=x.dtype)
    x_padded = torch.cat([zero_pad, x], dim=-1)
    x_padded = x_padded.view(*x.size()[:2], x.size(3) + 1, x.size(2))
    return x_padded[:, :, 1:].view_as(x)[:, :, :, : x.size(-1) // 2 + 1]


def rel_shift_legacy(x):
    """LegacyRelPositionMultiHeadedAttention.rel_shift, attention.py:145-165."""
    zero_pad = torch.zeros((*x.size()[:3], 1), dtype=x.dtype)
    x_padded = torch.cat([zero_pad, x], dim=-1)
    x_padded = x_padded.view(*x.size()[:2], x.size(3) + 1, x.size(2))
    return x_padded[:, :, 1:].view_as(x)


def _attend(P, pre, v, scores, mask, p_drop, training):
    """MultiHeadedAttention.forward_attention, attention.py:64-96."""
    B = v.size(0)
    m = mask.unsqueeze(1).eq(0)
    minv = float(np.finfo(torch.tensor(0, dtype=scores.dtype).numpy().dtype).min)
    scores = scores.masked_fill(m, minv)
    attn = torch.softmax(scores, dim=-1).masked_fill(m, 0.0)
    x = torch.matmul(dropout(attn, p_drop, training), v)
    x = x.transpose(1, 2).contiguous().view(B, -1, v.size(1) * v.size(3))
    return linear(P, pre + ".linear_out", x)


def _qkv(P, pre, q_in, k_in, v_in, H):
    """MultiHeadedAttention.forward_qkv, attention.py:40-62."""
    B = q_in.size(0)
    D = P[pre + ".linear_q.weight"].size(0)
    dk = D // H
    q = linear(P, pre + ".linear_q", q_in).view(B, -1, H, dk).transpose(1, 2)
    k = linear(P, pre + ".linear_k", k_in).view(B, -1, H, dk).transpose(1, 2)
    v = linear(P, pre + ".linear_v", v_in).view(B, -1, H, dk).transpose(1, 2)
    return q, k, v


def mha(P, pre, q_in, k_in, v_in, mask, H, p_drop=0.0, training=True):
    """MultiHeadedAttention.forward, attention.py:98-114."""
    q, k, v = _qkv(P, pre, q_in, k_in, v_in, H)
    scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(q.size(-1))
    return _attend(P, pre, v, scores, mask, p_drop, training)


def rel_mha(P, pre, x, pos_emb, mask, H, legacy: bool, p_drop=0.0, training=True):
    """(Legacy)RelPositionMultiHeadedAttention.forward, attention.py:167-209 / 265-308."""
    q, k, v = _qkv(P, pre, x, x, x, H)
    q = q.transpose(1, 2)
    nbp = pos_emb.size(0)
    p = linear(P, pre + ".linear_pos", pos_emb, bias=False).view(nbp, -1, H, q.size(-1))
    p = p.transpose(1, 2)
    q_u = (q + P[pre + ".pos_bias_u"]).transpose(1, 2)
    q_v = (q + P[pre + ".pos_bias_v"]).transpose(1, 2)
    ac = torch.matmul(q_u, k.transpose(-2, -1))
    bd = torch.matmul(q_v, p.transpose(-2, -1))
    bd = rel_shift_legacy(bd) if legacy else rel_shift_latest(bd)
    scores = (ac + bd) / math.sqrt(q.size(-1))
    return _attend(P, pre, v, scores, mask, p_drop, training)


def ffn(P, pre, x, act: str, p_drop=0.0, training=True):
    """PositionwiseFeedForward.forward, positionwise_feed_forward.py:30-32."""
    h = linear(P, pre + ".w_1", x)
    h = h * torch.sigmoid(h) if act == "swish" else F.relu(h)
    return linear(P, pre + ".w_2", dropout(h, p_drop, training))


def conv_module(P, pre, x, kernel: int, bn_state: Optional[dict] = None, training=True):
    """ConvolutionModule.forward, conformer/convolution.py:56-79 (BN in training mode)."""
    x = x.transpose(1, 2)
    x = F.conv1d(x, P[pre + ".pointwise_conv1.weight"], P[pre + ".pointwise_conv1.bias"])
    x = F.glu(x, dim=1)
    D = x.size(1)
    x = F.conv1d(x, P[pre + ".depthwise_conv.weight"], P[pre + ".depthwise_conv.bias"],
                 padding=(kernel - 1) // 2, groups=D)
    st = bn_state if bn_state is not None else {}
    rm = st.setdefault(pre + ".norm.running_mean", P[pre + ".norm.running_mean"].detach().clone())
    rv = st.setdefault(pre + ".norm.running_var", P[pre + ".norm.running_var"].detach().clone())
    x = F.batch_norm(x, rm, rv, P[pre + ".norm.weight"], P[pre + ".norm.bias"],
                     training=training, momentum=0.1, eps=1e-5)
    x = x * torch.sigmoid(x)
    x = F.conv1d(x, P[pre + ".pointwise_conv2.weight"], P[pre + ".pointwise_conv2.bias"])
    return x.transpose(1, 2)


def conformer_layer(P, pre, x, pos_emb, mask, cfg: EncCfg, bn_state=None, training=True):
    """Conformer EncoderLayer.forward (macaron, pre-LN), encoder_layer.py:76-157."""
    p = cfg.dropout_rate
    ff_scale = 0.5 if cfg.macaron_style else 1.0
    if cfg.macaron_style:
        x = x + ff_scale * dropout(ffn(P, pre + ".feed_forward_macaron",
                                       layer_norm(P, pre + ".norm_ff_macaron", x), "swish", p, training), p, training)
    h = layer_norm(P, pre + ".norm_mha", x)
    x = x + dropout(rel_mha(P, pre + ".self_attn", h, pos_emb, mask, cfg.attention_heads,
                            cfg.rel_pos_type == "legacy", cfg.attention_dropout_rate, training), p, training)
    if cfg.use_cnn_module:
        h = layer_norm(P, pre + ".norm_conv", x)
        x = x + dropout(conv_module(P, pre + ".conv_module", h, cfg.cnn_module_kernel, bn_state, training), p, training)
    h = layer_norm(P, pre + ".norm_ff", x)
    x = x + ff_scale * dropout(ffn(P, pre + ".feed_forward", h, "swish", p, training), p, training)
    if cfg.use_cnn_module:
        x = layer_norm(P, pre + ".norm_final", x)
    return x


def transformer_enc_layer(P, pre, x, mask, cfg: EncCfg, training=True):
    """transformer/encoder_layer.py:57-110 (pre-LN, ReLU FFN)."""
    p = cfg.dropout_rate
    h = layer_norm(P, pre + ".norm1", x)
    x = x + dropout(mha(P, pre + ".self_attn", h, h, h, mask, cfg.attention_heads,
                        cfg.attention_dropout_rate, training), p, training)
    h = layer_norm(P, pre + ".norm2", x)
    x = x + dropout(ffn(P, pre + ".feed_forward", h, "relu", p, training), p, training)
    return x


def encoder(P, feats, lens, cfg: EncCfg, bn_state=None, training=True):
    """ConformerEncoder.forward (conformer_encoder.py:292-368) / TransformerEncoder.forward."""
    T = feats.size(1)
    lim = 7 if cfg.input_layer == "conv2d" else 11  # check_short_utt, subsampling.py:31-39
    if T < lim:
        raise ValueError(f"TooShortUttError: needs more than {lim} frames")
    masks = (~make_pad_mask(lens, T))[:, None, :]
    x, masks = conv2d_subsampling(P, "encoder.embed", feats, masks, cfg.input_layer)
    Tp = x.size(1)
    D = cfg.output_size
    if cfg.kind == "conformer":
        x = x * math.sqrt(D)
        if cfg.rel_pos_type == "legacy":
            pos = rel_pos_table_legacy(Tp, D, cfg.max_pos_emb_len)
        else:
            pos = rel_pos_table_latest(Tp, D, cfg.max_pos_emb_len)
        pos = pos.to(x.dtype)
        x = dropout(x, cfg.positional_dropout_rate, training)
        pos = dropout(pos, cfg.positional_dropout_rate, training)
        inter = []
        for i in range(cfg.num_blocks):
            x = conformer_layer(P, f"encoder.encoders.{i}", x, pos, masks, cfg, bn_state, training)
            if i + 1 in cfg.interctc_layer_idx:  # intermediate outputs are also normalised (:337-341)
                h = layer_norm(P, "encoder.after_norm", x)
                inter.append((i + 1, h))
                if cfg.interctc_use_conditioning:  # x + conditioning_layer(ctc.softmax(h)) (:343-350)
                    x = x + linear(P, "encoder.conditioning_layer", torch.softmax(linear(P, "ctc.ctc_lo", h), dim=-1))
        if inter:
            x = layer_norm(P, "encoder.after_norm", x)
            return (x, inter), masks.squeeze(1).sum(1)
    else:
        x = x * math.sqrt(D) + abs_pos_table(Tp, D).to(x.dtype)
        x = dropout(x, cfg.positional_dropout_rate, training)
        for i in range(cfg.num_blocks):
            x = transformer_enc_layer(P, f"encoder.encoders.{i}", x, masks, cfg, training)
    x = layer_norm(P, "encoder.after_norm", x)
    olens = masks.squeeze(1).sum(1)
    return x, olens


def decoder(P, hs, hlens, ys_in, ys_in_lens, cfg: DecCfg, training=True):
    """BaseTransformerDecoder.forward, transformer_decoder.py:92-145 + DecoderLayer.forward."""
    L = ys_in.size(1)
    tgt_mask = (~make_pad_mask(ys_in_lens, L))[:, None, :]
    tgt_mask = tgt_mask & subsequent_mask(L).unsqueeze(0)
    mem_mask = (~make_pad_mask(hlens, hs.size(1)))[:, None, :]
    D = hs.size(-1)
    x = P["decoder.embed.0.weight"][ys_in]
    x = x * math.sqrt(D) + abs_pos_table(L, D).to(x.dtype)
    x = dropout(x, cfg.positional_dropout_rate, training)
    p = cfg.dropout_rate
    H = cfg.attention_heads
    for j in range(cfg.num_blocks):
        pre = f"decoder.decoders.{j}"
        h = layer_norm(P, pre + ".norm1", x)
        x = x + dropout(mha(P, pre + ".self_attn", h, h, h, tgt_mask, H, cfg.self_attention_dropout_rate, training), p, training)
        h = layer_norm(P, pre + ".norm2", x)
        x = x + dropout(mha(P, pre + ".src_attn", h, hs, hs, mem_mask, H, cfg.src_attention_dropout_rate, training), p, training)
        h = layer_norm(P, pre + ".norm3", x)
        x = x + dropout(ffn(P, pre + ".feed_forward", h, "relu", p, training), p, training)
    x = layer_norm(P, "decoder.after_norm", x)
    return linear(P, "decoder.output_layer", x)


# ----------------------------------------------------------------------------- losses
def ctc_loss(P, hs, hlens, ys_pad, ys_lens, blank=0):
    """espnet2 CTC.forward + loss_fn (ctc.py:52-97): log_softmax + CTCLoss(none, zero_inf), sum/B."""
    ys_hat = linear(P, "ctc.ctc_lo", hs).transpose(0, 1)
    ys_true = torch.cat([ys_pad[i, :l] for i, l in enumerate(ys_lens)])
    lp = ys_hat.log_softmax(2)
    loss = F.ctc_loss(lp, ys_true, hlens, ys_lens, blank=blank, reduction="none", zero_infinity=True)
    return loss.sum() / lp.size(1)


def add_sos_eos(ys_pad, sos, eos, ignore_id):
    """add_sos_eos.py:12-31."""
    ys = [y[y != ignore_id] for y in ys_pad]
    L = max(len(y) for y in ys) + 1
    B = len(ys)
    ys_in = torch.full((B, L), eos, dtype=torch.long)
    ys_out = torch.full((B, L), ignore_id, dtype=torch.long)
    for i, y in enumerate(ys):
        ys_in[i, 0] = sos
        ys_in[i, 1: len(y) + 1] = y
        ys_out[i, : len(y)] = y
        ys_out[i, len(y)] = eos
    return ys_in, ys_out


def label_smoothing_loss(x, target, size, padding_idx, smoothing, normalize_length=False):
    """LabelSmoothingLoss.forward, label_smoothing_loss.py:41-63 (KL incl. t*log t)."""
    B = x.size(0)
    x = x.view(-1, size)
    target = target.view(-1)
    with torch.no_grad():
        true_dist = torch.full_like(x, smoothing / (size - 1))
        ignore = target == padding_idx
        total = len(target) - int(ignore.sum())
        t = target.masked_fill(ignore, 0)
        true_dist.scatter_(1, t.unsqueeze(1), 1.0 - smoothing)
    kl = F.kl_div(torch.log_softmax(x, dim=1), true_dist, reduction="none")
    denom = total if normalize_length else B
    return kl.masked_fill(ignore.unsqueeze(1), 0).sum() / denom


def th_accuracy(pad_outputs, pad_targets, ignore_label):
    """nets_utils.py:299-320."""
    pred = pad_outputs.view(pad_targets.size(0), pad_targets.size(1), pad_outputs.size(1)).argmax(2)
    mask = pad_targets != ignore_label
    num = torch.sum(pred.masked_select(mask) == pad_targets.masked_select(mask))
    return float(num) / float(torch.sum(mask))


# ----------------------------------------------------------------------------- frontend
def time_warp_fixed(x, center: int, warped: int):
    """time_warp.py:9-46 with (center, warped) given instead of drawn (x: (B,T,F))."""
    xx = x[:, None]
    t = xx.shape[2]
    left = F.interpolate(xx[:, :, :center], (warped, xx.shape[3]), mode="bicubic", align_corners=False)
    right = F.interpolate(xx[:, :, center:], (t - warped, xx.shape[3]), mode="bicubic", align_corners=False)
    return torch.cat([left, right], dim=-2)[:, 0]


def mask_along_axis_fixed(spec, mask_pos, mask_len, dim: int):
    """mask_along_axis.py:8-68 with (mask_pos, mask_len) (B,num_mask) given; fill 0."""
    D = spec.shape[dim]
    aran = torch.arange(D)[None, None, :]
    mask = (mask_pos[:, :, None] <= aran) & (aran < (mask_pos + mask_len)[:, :, None])
    mask = mask.any(dim=1)
    mask = mask.unsqueeze(2) if dim == 1 else mask.unsqueeze(1)
    return spec.masked_fill(mask, 0.0)


def utterance_mvn(x, ilens):
    """utterance_mvn.py:45-80, norm_means=True, norm_vars=False (pads become -mean)."""
    pm = make_pad_mask(ilens, x.size(1))[:, :, None]
    x = x.masked_fill(pm, 0.0)
    mean = x.sum(dim=1, keepdim=True) / ilens.to(x.dtype).view(-1, 1, 1)
    return x - mean


# ----------------------------------------------------------------------------- model
def asr_forward(P: Params, speech, speech_lengths, text, text_lengths, cfg: ModelCfg,
                specaug: Optional[dict] = None, bn_state=None, training=True):
    """ESPnetASRModel.forward, espnet_model.py:169-297 (+ encode :319-377).

    `specaug`, when given, holds the injected random draws:
    {"center","warped"} (time warp), {"freq_pos","freq_len"}, {"time_pos","time_len"}.
    Returns (loss, stats dict, weight) like the reference.
    """
    B = speech.size(0)
    text = text.clone()
    text[text == -1] = cfg.ignore_id
    text = text[:, : int(text_lengths.max())]
    feats = speech[:, : int(speech_lengths.max())]
    lens = speech_lengths
    if specaug is not None and training:
        if "center" in specaug:
            feats = time_warp_fixed(feats, int(specaug["center"]), int(specaug["warped"]))
        if "freq_pos" in specaug:
            feats = mask_along_axis_fixed(feats, specaug["freq_pos"], specaug["freq_len"], 2)
        if "time_pos" in specaug:
            feats = mask_along_axis_fixed(feats, specaug["time_pos"], specaug["time_len"], 1)
    feats = utterance_mvn(feats, lens)
    hs, hlens = encoder(P, feats, lens, cfg.enc, bn_state, training)
    inter = None
    if isinstance(hs, tuple):
        hs, inter = hs
    stats = {}
    loss_ctc = loss_att = acc = None
    if cfg.ctc_weight != 0.0:
        loss_ctc = ctc_loss(P, hs, hlens, text, text_lengths, cfg.blank_id)
        stats["loss_ctc"] = loss_ctc.detach()
    if cfg.interctc_weight != 0.0 and inter:  # espnet_model.py:222-245
        loss_ic = 0.0
        for idx, h in inter:
            l_ic = ctc_loss(P, h, hlens, text, text_lengths, cfg.blank_id)
            stats[f"loss_interctc_layer{idx}"] = l_ic.detach()
            loss_ic = loss_ic + l_ic
        loss_ctc = (1 - cfg.interctc_weight) * loss_ctc + cfg.interctc_weight * (loss_ic / len(inter))
    if cfg.ctc_weight != 1.0:
        ys_in, ys_out = add_sos_eos(text, cfg.sos, cfg.eos, cfg.ignore_id)
        dec_out = decoder(P, hs, hlens, ys_in, text_lengths + 1, cfg.dec, training)
        loss_att = label_smoothing_loss(dec_out, ys_out, cfg.vocab_size, cfg.ignore_id,
                                        cfg.lsm_weight, cfg.length_normalized_loss)
        acc = th_accuracy(dec_out.view(-1, cfg.vocab_size), ys_out, cfg.ignore_id)
        stats["loss_att"] = loss_att.detach()
        stats["acc"] = acc
    if cfg.ctc_weight == 0.0:
        loss = loss_att
    elif cfg.ctc_weight == 1.0:
        loss = loss_ctc
    else:
        loss = cfg.ctc_weight * loss_ctc + (1 - cfg.ctc_weight) * loss_att
    stats["loss"] = loss.detach()
    return loss, stats, torch.tensor([B])


# ----------------------------------------------------------------------------- params
def param_shapes(cfg: ModelCfg) -> Dict[str, Tuple[int, ...]]:
    """state_dict keys/shapes of the reference model, trainable + BN buffers."""
    e, V = cfg.enc, cfg.vocab_size
    D, FF, H = e.output_size, e.linear_units, e.attention_heads
    F2 = ((e.input_size - 1) // 2 - 1) // 2 if e.input_layer == "conv2d" else ((e.input_size - 1) // 2 - 2) // 3
    s: Dict[str, Tuple[int, ...]] = {}

    def lin(pre, i, o, bias=True):
        s[pre + ".weight"] = (o, i)
        if bias:
            s[pre + ".bias"] = (o,)

    def ln(pre):
        s[pre + ".weight"] = (D,)
        s[pre + ".bias"] = (D,)

    s["encoder.embed.conv.0.weight"] = (D, 1, 3, 3)
    s["encoder.embed.conv.0.bias"] = (D,)
    k2 = 3 if e.input_layer == "conv2d" else 5
    s["encoder.embed.conv.2.weight"] = (D, D, k2, k2)
    s["encoder.embed.conv.2.bias"] = (D,)
    lin("encoder.embed.out.0", D * F2, D)
    if e.interctc_use_conditioning:  # espnet_model.py:96-101 (registered on the encoder, after its layers)
        lin("encoder.conditioning_layer", V, D)
    for i in range(e.num_blocks):
        p = f"encoder.encoders.{i}"
        for n in ("q", "k", "v", "out"):
            lin(f"{p}.self_attn.linear_{n}", D, D)
        if e.kind == "conformer":
            lin(f"{p}.self_attn.linear_pos", D, D, bias=False)
            s[f"{p}.self_attn.pos_bias_u"] = (H, D // H)
            s[f"{p}.self_attn.pos_bias_v"] = (H, D // H)
            lin(f"{p}.feed_forward.w_1", D, FF)
            lin(f"{p}.feed_forward.w_2", FF, D)
            if e.macaron_style:
                lin(f"{p}.feed_forward_macaron.w_1", D, FF)
                lin(f"{p}.feed_forward_macaron.w_2", FF, D)
            if e.use_cnn_module:
                c = f"{p}.conv_module"
                s[f"{c}.pointwise_conv1.weight"] = (2 * D, D, 1)
                s[f"{c}.pointwise_conv1.bias"] = (2 * D,)
                s[f"{c}.depthwise_conv.weight"] = (D, 1, e.cnn_module_kernel)
                s[f"{c}.depthwise_conv.bias"] = (D,)
                s[f"{c}.norm.weight"] = (D,)
                s[f"{c}.norm.bias"] = (D,)
                s[f"{c}.norm.running_mean"] = (D,)
                s[f"{c}.norm.running_var"] = (D,)
                s[f"{c}.norm.num_batches_tracked"] = ()
                s[f"{c}.pointwise_conv2.weight"] = (D, D, 1)
                s[f"{c}.pointwise_conv2.bias"] = (D,)
            ln(f"{p}.norm_ff")
            ln(f"{p}.norm_mha")
            if e.macaron_style:
                ln(f"{p}.norm_ff_macaron")
            if e.use_cnn_module:
                ln(f"{p}.norm_conv")
                ln(f"{p}.norm_final")
        else:
            lin(f"{p}.feed_forward.w_1", D, FF)
            lin(f"{p}.feed_forward.w_2", FF, D)
            ln(f"{p}.norm1")
            ln(f"{p}.norm2")
    ln("encoder.after_norm")
    if cfg.dec is not None and cfg.ctc_weight != 1.0:
        d = cfg.dec
        s["decoder.embed.0.weight"] = (V, D)
        ln("decoder.after_norm")
        lin("decoder.output_layer", D, V)
        for j in range(d.num_blocks):
            p = f"decoder.decoders.{j}"
            for a in ("self_attn", "src_attn"):
                for n in ("q", "k", "v", "out"):
                    lin(f"{p}.{a}.linear_{n}", D, D)
            lin(f"{p}.feed_forward.w_1", D, d.linear_units)
            lin(f"{p}.feed_forward.w_2", d.linear_units, D)
            ln(f"{p}.norm1")
            ln(f"{p}.norm2")
            ln(f"{p}.norm3")
    if cfg.ctc_weight != 0.0:
        lin("ctc.ctc_lo", D, V)
    return s


def deterministic_params(cfg: ModelCfg, seed: int = 0, dtype=torch.float32) -> Params:
    """Seeded parameter values reproducible without the reference (numpy PCG64).

    Keys are sorted so the stream does not depend on construction order. Weights ~
    N(0, 1/fan_in); biases ~ 0.05 N; norm scales 1 + 0.1 N; BN running stats (0, 1).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    out: Params = {}
    for k in sorted(param_shapes(cfg)):
        shp = param_shapes(cfg)[k]
        if k.endswith("num_batches_tracked"):
            out[k] = torch.tensor(0, dtype=torch.long)
            continue
        if k.endswith("running_mean"):
            a = np.zeros(shp)
        elif k.endswith("running_var"):
            a = np.ones(shp)
        elif ("norm" in k.split(".")[-2] or k.split(".")[-2].startswith("norm")) and k.endswith(".weight") and len(shp) == 1:
            a = 1.0 + 0.1 * rng.standard_normal(shp)
        elif k.endswith("bias") or len(shp) == 1:
            a = 0.05 * rng.standard_normal(shp)
        elif k.endswith("pos_bias_u") or k.endswith("pos_bias_v"):
            a = 0.1 * rng.standard_normal(shp)
        elif k == "decoder.embed.0.weight":
            a = rng.standard_normal(shp)
        else:
            fan_in = int(np.prod(shp[1:]))
            a = rng.standard_normal(shp) / math.sqrt(fan_in)
        out[k] = torch.tensor(a, dtype=dtype)
    return out


def synthetic_batch(B: int, T: int, F_: int, V: int, lens: List[int], ulens: List[int], seed: int):
    """Seeded synthetic batch (numpy PCG64): fbank ~ N(0,1), text ~ U[2, V-2], padded -1."""
    rng = np.random.Generator(np.random.PCG64(seed))
    speech = rng.standard_normal((B, T, F_)).astype(np.float32)
    for i, l in enumerate(lens):
        speech[i, l:] = 0.0
    U = max(ulens)
    text = np.full((B, U), -1, dtype=np.int64)
    for i, u in enumerate(ulens):
        text[i, :u] = rng.integers(2, V - 1, size=u)
    return (torch.from_numpy(speech), torch.tensor(lens, dtype=torch.long),
            torch.from_numpy(text), torch.tensor(ulens, dtype=torch.long))
