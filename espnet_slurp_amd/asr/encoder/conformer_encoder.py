"""ConformerEncoder — drop-in for espnet2/asr/encoder/conformer_encoder.py:47-368.

Same constructor kwargs and state_dict keys; forward(xs_pad, ilens) -> (out, olens, None).
Computation: Conv2dSubsampling (implicit-im2col MFMA GEMM) -> x*sqrt(D) + rel-pos table
-> num_blocks macaron Conformer blocks -> after_norm, all in libespnet_mi355.so kernels
with an explicit backward (EncoderFn).  Supported configuration space = the one the
SLURP / LibriSpeech Conformer recipes use; anything else raises NotImplementedError.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple, Union

import torch
from torch import nn

from ... import kernels as K
from ...blocks import (ConvolutionModule, Ctx, make_subsampling, LayerNorm, PositionwiseFeedForward,
                       RelPositionMultiHeadedAttention, Seeds, empty)
from .abs_encoder import (AbsEncoder, EncoderFn, TooShortUttError, draw_seed, lengths_to_device, pos_table,
                          subsampled_lengths)


class EncoderLayer(nn.Module):
    """Conformer block (conformer/encoder_layer.py:17-157), normalize_before=True,
    concat_after=False:  x += ff_scale*drop(FFN_mac(LN(x))); x += drop(MHA(LN(x)));
    x += drop(Conv(LN(x))); x += ff_scale*drop(FFN(LN(x))); x = LN_final(x)."""

    def __init__(self, size, self_attn, feed_forward, feed_forward_macaron, conv_module, dropout_rate):
        super().__init__()
        self.self_attn = self_attn
        self.feed_forward = feed_forward
        self.feed_forward_macaron = feed_forward_macaron
        self.conv_module = conv_module
        self.norm_ff = LayerNorm(size)
        self.norm_mha = LayerNorm(size)
        if feed_forward_macaron is not None:
            self.norm_ff_macaron = LayerNorm(size)
            self.ff_scale = 0.5
        else:
            self.ff_scale = 1.0
        if conv_module is not None:
            self.norm_conv = LayerNorm(size)
            self.norm_final = LayerNorm(size)
        self.p = dropout_rate
        self.size = size

    def fwd(self, x, pos, klen, B, T, seeds: Seeds, training: bool, tvalid=None):
        c = Ctx()
        p = self.p
        if self.feed_forward_macaron is not None:
            h, c.ln_mac = self.norm_ff_macaron.fwd(x, gemm_only=True)
            x, c.ffm = self.feed_forward_macaron.fwd(h, x, self.ff_scale, p, seeds, training)
        h, c.ln_mha = self.norm_mha.fwd(x, gemm_only=True)
        x, c.mha = self.self_attn.fwd(h, x, pos, klen, B, T, p, seeds, training, tvalid=tvalid)
        if self.conv_module is not None:
            h, c.ln_conv = self.norm_conv.fwd(x, gemm_only=True)
            x, c.conv = self.conv_module.fwd(h, x, B, T, p, seeds, training, tvalid=tvalid)
        h, c.ln_ff = self.norm_ff.fwd(x, gemm_only=True)
        x, c.ff = self.feed_forward.fwd(h, x, self.ff_scale, p, seeds, training)
        if self.conv_module is not None:
            x, c.ln_final = self.norm_final.fwd(x)
        return x, c

    def bwd(self, c, d):
        if self.conv_module is not None:
            d = self.norm_final.bwd_new(c.ln_final, d)
        self.norm_ff.bwd(c.ln_ff, self.feed_forward.bwd(c.ff, d), d)
        if self.conv_module is not None:
            self.norm_conv.bwd(c.ln_conv, self.conv_module.bwd(c.conv, d), d)
        self.norm_mha.bwd(c.ln_mha, self.self_attn.bwd(c.mha, d), d)
        if self.feed_forward_macaron is not None:
            self.norm_ff_macaron.bwd(c.ln_mac, self.feed_forward_macaron.bwd(c.ffm, d), d)
        return d


class ConformerEncoder(AbsEncoder):
    def __init__(
        self,
        input_size: int,
        output_size: int = 256,
        attention_heads: int = 4,
        linear_units: int = 2048,
        num_blocks: int = 6,
        dropout_rate: float = 0.1,
        positional_dropout_rate: float = 0.1,
        attention_dropout_rate: float = 0.0,
        input_layer: str = "conv2d",
        normalize_before: bool = True,
        concat_after: bool = False,
        positionwise_layer_type: str = "linear",
        positionwise_conv_kernel_size: int = 3,
        macaron_style: bool = False,
        rel_pos_type: str = "legacy",
        pos_enc_layer_type: str = "rel_pos",
        selfattention_layer_type: str = "rel_selfattn",
        activation_type: str = "swish",
        use_cnn_module: bool = True,
        zero_triu: bool = False,
        cnn_module_kernel: int = 31,
        padding_idx: int = -1,
        interctc_layer_idx: List[int] = [],
        interctc_use_conditioning: bool = False,
        stochastic_depth_rate: Union[float, List[float]] = 0.0,
        layer_drop_rate: float = 0.0,
        max_pos_emb_len: int = 5000,
    ):
        super().__init__()
        self._output_size = output_size
        # rel_pos_type remap, conformer_encoder.py:116-125
        if rel_pos_type == "legacy":
            if pos_enc_layer_type == "rel_pos":
                pos_enc_layer_type = "legacy_rel_pos"
            if selfattention_layer_type == "rel_selfattn":
                selfattention_layer_type = "legacy_rel_selfattn"
        elif rel_pos_type == "latest":
            assert selfattention_layer_type != "legacy_rel_selfattn"
            assert pos_enc_layer_type != "legacy_rel_pos"
        else:
            raise ValueError("unknown rel_pos_type: " + rel_pos_type)
        unsupported = []
        if input_layer not in ("conv2d", "conv2d6"):
            unsupported.append(f"input_layer={input_layer}")
        if not normalize_before or concat_after:
            unsupported.append("normalize_before=False/concat_after=True")
        if positionwise_layer_type != "linear":
            unsupported.append(f"positionwise_layer_type={positionwise_layer_type}")
        if (pos_enc_layer_type, selfattention_layer_type) not in (("rel_pos", "rel_selfattn"),
                                                                  ("legacy_rel_pos", "legacy_rel_selfattn")):
            unsupported.append(f"{pos_enc_layer_type}/{selfattention_layer_type}")
        if activation_type != "swish":
            unsupported.append(f"activation_type={activation_type}")
        if zero_triu or layer_drop_rate:
            unsupported.append("zero_triu/layer_drop")
        sdr = stochastic_depth_rate if isinstance(stochastic_depth_rate, list) else [stochastic_depth_rate]
        if any(r != 0.0 for r in sdr):
            unsupported.append("stochastic_depth_rate")
        if unsupported:
            raise NotImplementedError("espnet_slurp_amd ConformerEncoder: unsupported " + ", ".join(unsupported))
        self.legacy = pos_enc_layer_type == "legacy_rel_pos"
        self.embed = make_subsampling(input_layer, input_size, output_size)
        self.encoders = nn.ModuleList([
            EncoderLayer(
                output_size,
                RelPositionMultiHeadedAttention(attention_heads, output_size, attention_dropout_rate, self.legacy),
                PositionwiseFeedForward(output_size, linear_units, dropout_rate, K.ACT_SWISH),
                PositionwiseFeedForward(output_size, linear_units, dropout_rate, K.ACT_SWISH) if macaron_style else None,
                ConvolutionModule(output_size, cnn_module_kernel) if use_cnn_module else None,
                dropout_rate,
            ) for _ in range(num_blocks)
        ])
        self.after_norm = LayerNorm(output_size)
        self.dropout_rate = dropout_rate
        self.positional_dropout_rate = positional_dropout_rate
        self.max_pos_emb_len = max_pos_emb_len
        if len(interctc_layer_idx) > 0:  # conformer_encoder.py:283-285
            assert 0 < min(interctc_layer_idx) and max(interctc_layer_idx) < num_blocks
        self.interctc_layer_idx = list(interctc_layer_idx)
        # self-conditioning (conformer_encoder.py:286-287, 343-350): the model creates conditioning_layer =
        # Linear(vocab, D) (espnet_model.py:96-101) and passes the CTC module to the forward
        self.conditioning_layer = None
        self.interctc_use_conditioning = interctc_use_conditioning
        self.flat = None
        self._seed_counter = 0

    def output_size(self) -> int:
        return self._output_size

    def attach_flat(self, flat):
        self.flat = flat
        for l in self.encoders:
            l.self_attn.flat = flat

    # ---------------------------------------------------------------- explicit passes
    def run_forward(self, feats, ilens_cpu, seeds: Seeds, training: bool, klen=None, tvalid=None, inter=None):
        """tvalid: optional device int32 (1,) = the reference batch's T' when feats are padded
        to a length bucket (frames beyond are excluded from the convolution module's depthwise
        padding and BatchNorm statistics, and the legacy rel_shift is taken at T'; every other op
        is per frame or masked by klen).
        inter: the model's intermediate-CTC request (ESPnetASRModel._inter_request) -- after each block in
        interctc_layer_idx the block output is normalised by after_norm (conformer_encoder.py:333-341) and its
        CTC loss and loss gradient are formed right here, like the heads' CTC (fused into the forward); the
        backward adds the gradient into the residual stream at that block (run_backward)."""
        B, T, _ = feats.shape
        lim = self.embed.min_frames  # check_short_utt (subsampling.py:31-39)
        if T < lim:
            raise TooShortUttError(
                f"has {T} frames and is too short for subsampling (it needs more than {lim} frames), return empty results",
                T, lim)
        D = self._output_size
        olens = subsampled_lengths(ilens_cpu, T, self.embed.input_layer)
        if klen is None:
            klen = lengths_to_device(olens, feats.device)
        x, c_emb = self.embed.fwd(feats, math.sqrt(D), self.positional_dropout_rate, seeds, training)
        T2 = c_emb.T2
        tab = pos_table("legacy" if self.legacy else "latest", T2, D, feats.device, self.max_pos_emb_len)
        pp = self.positional_dropout_rate if training else 0.0
        sp = seeds.next()
        if pp > 0:
            pos = torch.empty_like(tab)
            K.scale_dropout(tab, pos, drop_p=pp, seed=sp)
        else:
            pos = tab
        ctxs = []
        inters = []
        for li, layer in enumerate(self.encoders):
            x, c = layer.fwd(x, pos, klen, B, T2, seeds, training, tvalid=tvalid)
            ctxs.append(c)
            if inter is not None and li + 1 in self.interctc_layer_idx:
                x, ic = self._interctc_fwd(li + 1, x, B, T2, inter)
                inters.append(ic)
        hs, c_after = self.after_norm.fwd(x)
        return hs.view(B, T2, D), olens, Ctx(emb=c_emb, layers=ctxs, after=c_after, inter=inters)

    def _interctc_fwd(self, idx, x, B, T2, inter):
        """One intermediate branch: y = after_norm(x), its CTC nll (B,) and d(weighted loss)/d logits (when the
        model weights the branch), and with self-conditioning the new residual stream x + conditioning_layer(
        softmax(ctc_lo(y))) (conformer_encoder.py:343-350).  Returns (x, branch context)."""
        y, c_ln = self.after_norm.fwd(x)
        ctc = inter["ctc"]
        nll = grad = lp = None
        if inter["weighted"]:
            nll, grad, lp = ctc.loss_and_grad(y, B, T2, inter["hlens"], inter["ys"], inter["tlens"], inter["Umax"],
                                              inter["gscale"], want_grad=inter["want_grad"])
            inter["nll"].append((idx, nll))
            if grad is not None:
                inter["grads"].append(grad)
        prob = None
        if self.conditioning_layer is not None:
            if lp is None:
                logits = ctc.logits(y)
                lp = torch.empty_like(logits)
                K.log_softmax(logits, lp, logits.shape[0], logits.shape[1])
            prob = torch.exp(lp)  # ctc.softmax (ctc.py:100-108): exp of the log-softmax rows
            x = self.conditioning_layer.fwd(prob, R=x, beta=1.0)  # x + W p + b
        return x, Ctx(idx=idx, y=y, c_ln=c_ln, grad=grad, ctc=ctc, prob=prob,
                      live=grad is not None or (prob is not None and inter["want_grad"]))

    def run_backward(self, saved, dhs, grad_hook=None):
        B, T2, D = dhs.shape
        d = self.after_norm.bwd_new(saved.after, dhs.view(B * T2, D))
        inter = {c.idx: c for c in (saved.get("inter") or []) if c.live}
        # after_norm (and ctc_lo) receive more gradient from the intermediate branches below: their
        # module-done hooks (the DP bucket launches) wait until the last branch is done
        if grad_hook is not None and not inter:
            grad_hook(self.after_norm)
        for i in range(len(self.encoders) - 1, -1, -1):
            ic = inter.get(i + 1)
            if ic is not None:  # the intermediate branch read block i's output: its gradient joins d there
                if ic.prob is not None:
                    # self-conditioning: d (x + W p + b) / d p = W^T d -> softmax adjoint into the logits (+ the
                    # branch's CTC loss gradient), d x keeps d itself (the identity path)
                    rows, V = ic.prob.shape
                    dp = self.conditioning_layer.bwd(d, ic.prob)
                    dl = torch.empty_like(dp)
                    K.attn_softmax_bwd(ic.prob, dp, dl, 0.0, 0, 1.0, rows, V)
                    if ic.grad is not None:
                        dl.add_(ic.grad)
                else:
                    dl = ic.grad
                dy = torch.empty_like(ic.y)
                ic.ctc.backward_from_logits(dl, ic.y, dy)
                self.after_norm.bwd(ic.c_ln, dy, d)
            d = self.encoders[i].bwd(saved.layers[i], d)
            saved.layers[i] = None
            if grad_hook is not None:
                grad_hook(self.encoders[i])
        if grad_hook is not None and inter:
            grad_hook(self.after_norm)
            grad_hook(next(iter(inter.values())).ctc)
            if self.conditioning_layer is not None:
                grad_hook(self.conditioning_layer)
        saved.inter = None
        self.embed.bwd(saved.emb, d)
        if grad_hook is not None:
            grad_hook(self.embed)

    def forward(self, xs_pad: torch.Tensor, ilens: torch.Tensor, prev_states: torch.Tensor = None,
                ctc=None) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
        assert self.flat is not None, "call espnet_slurp_amd.flatten_model(model) before running"
        ilens_cpu = ilens.detach().cpu()
        feats = xs_pad.contiguous().float()
        olens = subsampled_lengths(ilens_cpu, feats.shape[1], self.embed.input_layer)
        hs = self.forward_prepared(feats, ilens_cpu, lengths_to_device(olens, feats.device), draw_seed())
        return hs, K.h2d(olens, xs_pad.device), None

    def forward_prepared(self, feats: torch.Tensor, ilens_cpu: torch.Tensor, klen: torch.Tensor, seed: int,
                         tvalid: torch.Tensor = None, inter=None):
        """Encoder output hs (B, T', D) from device-resident inputs only (klen: int32 output
        lengths on device): no host->device traffic, so it can be captured in a HIP graph.
        inter: the model's intermediate-CTC request (run_forward)."""
        anchor = self.after_norm.weight
        hook = getattr(self, "_grad_hook", None)
        if torch.is_grad_enabled() and anchor.requires_grad:
            return EncoderFn.apply(feats, anchor, self, ilens_cpu, seed, hook, klen, tvalid, inter)
        return self.run_forward(feats, ilens_cpu, Seeds(seed), self.training, klen=klen, tvalid=tvalid,
                                inter=inter)[0]

    def output_lengths(self, ilens_cpu: torch.Tensor, T: int) -> torch.Tensor:
        """Valid output frames per utterance (host, no device round trip)."""
        return subsampled_lengths(ilens_cpu, T, self.embed.input_layer)
