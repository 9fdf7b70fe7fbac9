"""TransformerEncoder — drop-in for espnet2/asr/encoder/transformer_encoder.py:59-228
(config C1, the mini_an4 plumbing case): Conv2dSubsampling + abs PositionalEncoding
(x*sqrt(D) + pe, dropout) + N pre-LN blocks [x += drop(MHA(LN x)); x += drop(FFN_relu(LN x))]
(transformer/encoder_layer.py:16-110) + after_norm."""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
from torch import nn

from ... import kernels as K
from ...blocks import Ctx, make_subsampling, LayerNorm, MultiHeadedAttention, PositionwiseFeedForward, Seeds
from .abs_encoder import (AbsEncoder, EncoderFn, TooShortUttError, draw_seed, lengths_to_device, pos_table,
                          subsampled_lengths)


class TransformerEncoderLayer(nn.Module):
    def __init__(self, size, self_attn, feed_forward, dropout_rate):
        super().__init__()
        self.self_attn = self_attn
        self.feed_forward = feed_forward
        self.norm1 = LayerNorm(size)
        self.norm2 = LayerNorm(size)
        self.p = dropout_rate
        self.size = size

    def fwd(self, x, klen, B, T, seeds, training):
        c = Ctx()
        h, c.ln1 = self.norm1.fwd(x)
        x, c.mha = self.self_attn.fwd(h, x, B, T, klen, False, self.p, seeds, training)
        h, c.ln2 = self.norm2.fwd(x)
        x, c.ff = self.feed_forward.fwd(h, x, 1.0, self.p, seeds, training)
        return x, c

    def bwd(self, c, d):
        self.norm2.bwd(c.ln2, self.feed_forward.bwd(c.ff, d), d)
        self.norm1.bwd(c.ln1, self.self_attn.bwd(c.mha, d), d)
        return d


class TransformerEncoder(AbsEncoder):
    def __init__(self, input_size: int, output_size: int = 256, attention_heads: int = 4, linear_units: int = 2048,
                 num_blocks: int = 6, dropout_rate: float = 0.1, positional_dropout_rate: float = 0.1,
                 attention_dropout_rate: float = 0.0, input_layer: Optional[str] = "conv2d", pos_enc_class=None,
                 normalize_before: bool = True, concat_after: bool = False, positionwise_layer_type: str = "linear",
                 positionwise_conv_kernel_size: int = 1, padding_idx: int = -1, interctc_layer_idx: List[int] = [],
                 interctc_use_conditioning: bool = False):
        super().__init__()
        if input_layer not in ("conv2d", "conv2d6") or not normalize_before or concat_after or positionwise_layer_type != "linear" \
                or interctc_layer_idx or interctc_use_conditioning:
            raise NotImplementedError("espnet_slurp_amd TransformerEncoder supports the conv2d / conv2d6, pre-LN, linear-FFN form")
        self._output_size = output_size
        self.embed = make_subsampling(input_layer, input_size, output_size)
        self.encoders = nn.ModuleList([
            TransformerEncoderLayer(output_size,
                                    MultiHeadedAttention(attention_heads, output_size, attention_dropout_rate),
                                    PositionwiseFeedForward(output_size, linear_units, dropout_rate, K.ACT_RELU),
                                    dropout_rate) for _ in range(num_blocks)])
        self.after_norm = LayerNorm(output_size)
        self.positional_dropout_rate = positional_dropout_rate
        self.flat = None

    def output_size(self) -> int:
        return self._output_size

    def attach_flat(self, flat):
        self.flat = flat
        for l in self.encoders:
            l.self_attn.flat = flat

    def run_forward(self, feats, ilens_cpu, seeds: Seeds, training: bool, klen=None, tvalid=None):
        # tvalid (length buckets) needs no handling here: every op is per frame or masked by klen
        B, T, _ = feats.shape
        lim = self.embed.min_frames  # check_short_utt (subsampling.py:31-39)
        if T < lim:
            raise TooShortUttError(f"has {T} frames and is too short for subsampling", T, lim)
        D = self._output_size
        olens = subsampled_lengths(ilens_cpu, T, self.embed.input_layer)
        if klen is None:
            klen = lengths_to_device(olens, feats.device)
        # embed: linear -> x*sqrt(D) + pe -> dropout.  The linear's epilogue gives x*sqrt(D);
        # the table is added by a residual-add pass with the dropout (embedding.py:81-94)
        x, c_emb = self.embed.fwd(feats, math.sqrt(D), 0.0, seeds, training)
        T2 = c_emb.T2
        pe = pos_table("abs", T2, D, feats.device)
        pp = self.positional_dropout_rate if training else 0.0
        sp = seeds.next()
        x3 = x.view(B, T2, D)
        xpe = torch.empty_like(x)
        for b in range(B):  # x + pe, then dropout over the whole tensor
            K.scale_dropout(pe, xpe[b * T2:(b + 1) * T2], alpha=1.0, drop_p=0.0, seed=0, r=x3[b], beta=1.0)
        if pp > 0:
            K.scale_dropout(xpe, xpe, drop_p=pp, seed=sp)
        ctxs = []
        y = xpe
        for layer in self.encoders:
            y, c = layer.fwd(y, klen, B, T2, seeds, training)
            ctxs.append(c)
        hs, c_after = self.after_norm.fwd(y)
        return hs.view(B, T2, D), olens, Ctx(emb=c_emb, layers=ctxs, after=c_after, pp=pp, sp=sp)

    def run_backward(self, saved, dhs, grad_hook=None):
        B, T2, D = dhs.shape
        d = self.after_norm.bwd_new(saved.after, dhs.view(B * T2, D))
        if grad_hook is not None:
            grad_hook(self.after_norm)
        for i in range(len(self.encoders) - 1, -1, -1):
            d = self.encoders[i].bwd(saved.layers[i], d)
            saved.layers[i] = None
            if grad_hook is not None:
                grad_hook(self.encoders[i])
        if saved.pp > 0:
            K.scale_dropout(d, d, drop_p=saved.pp, seed=saved.sp)
        self.embed.bwd(saved.emb, d)
        if grad_hook is not None:
            grad_hook(self.embed)

    def forward(self, xs_pad: torch.Tensor, ilens: torch.Tensor, prev_states: torch.Tensor = None
                ) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
        assert self.flat is not None, "call espnet_slurp_amd.flatten_model(model) before running"
        ilens_cpu = ilens.detach().cpu()
        feats = xs_pad.contiguous().float()
        olens = subsampled_lengths(ilens_cpu, feats.shape[1], self.embed.input_layer)
        hs = self.forward_prepared(feats, ilens_cpu, lengths_to_device(olens, feats.device), draw_seed())
        return hs, K.h2d(olens, xs_pad.device), None

    def forward_prepared(self, feats: torch.Tensor, ilens_cpu: torch.Tensor, klen: torch.Tensor, seed: int,
                         tvalid: torch.Tensor = None):
        """Encoder output hs (B, T', D) from device-resident inputs only (klen: int32 output
        lengths on device): no host->device traffic, so it can be captured in a HIP graph."""
        anchor = self.after_norm.weight
        hook = getattr(self, "_grad_hook", None)
        if torch.is_grad_enabled() and anchor.requires_grad:
            return EncoderFn.apply(feats, anchor, self, ilens_cpu, seed, hook, klen, tvalid)
        return self.run_forward(feats, ilens_cpu, Seeds(seed), self.training, klen=klen, tvalid=tvalid)[0]

    def output_lengths(self, ilens_cpu: torch.Tensor, T: int) -> torch.Tensor:
        """Valid output frames per utterance (host, no device round trip)."""
        return subsampled_lengths(ilens_cpu, T, self.embed.input_layer)
