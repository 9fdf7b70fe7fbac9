"""AbsEncoder (espnet2/asr/encoder/abs_encoder.py:7-19) and shared encoder plumbing."""
from __future__ import annotations

import math
from abc import ABC, abstractmethod
from typing import Dict, Optional, Tuple

import torch

from ... import kernels as K
from ...blocks import Seeds


class AbsEncoder(torch.nn.Module, ABC):
    @abstractmethod
    def output_size(self) -> int:
        raise NotImplementedError

    @abstractmethod
    def forward(self, xs_pad: torch.Tensor, ilens: torch.Tensor, prev_states: torch.Tensor = None
                ) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
        raise NotImplementedError


class TooShortUttError(Exception):
    """subsampling.py:14-29."""

    def __init__(self, message, actual_size, limit):
        super().__init__(message)
        self.actual_size = actual_size
        self.limit = limit


# second-stage (cut, stride) of the mask slicing per input_layer: conv2d `[:, :, :-2:2]` (subsampling.py:87),
# conv2d6 `[:, :, :-4:3]` (subsampling.py:146); the first stage is `[:, :, :-2:2]` for both
_MASK_STAGE2 = {"conv2d": (2, 2), "conv2d6": (4, 3)}


def subsampled_lengths(ilens_cpu: torch.Tensor, T: int, input_layer: str = "conv2d") -> torch.Tensor:
    """Valid-frame counts of `mask[:, :, :-2:2][:, :, :-c:s]` (subsampling.py:87 / :146): frame i
    survives the first stage iff i even, i < T-2, i < len; the second iff j % s == 0, j < T1 - c,
    j < len1.  Not the conv output-size formula."""
    cut, st = _MASK_STAGE2[input_layer]
    lens = ilens_cpu.long().clamp(max=T)
    T1 = len(range(0, T - 2, 2))
    l1 = torch.clamp((lens + 1) // 2, max=T1)
    l2 = torch.clamp((l1 + st - 1) // st, max=len(range(0, T1 - cut, st)))
    return l2


# ------------------------------------------------------------------ positional tables
_PE_CACHE: Dict[tuple, torch.Tensor] = {}


def _pe_rows(positions: torch.Tensor, d: int) -> torch.Tensor:
    """sin/cos rows computed exactly as embedding.py:66-80 (fp32, CPU)."""
    pe = torch.zeros(positions.numel(), d)
    position = positions.to(torch.float32).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe


def pos_table(kind: str, T: int, d: int, device, max_len: int = 5000) -> torch.Tensor:
    """Constant positional tables, host-built once per (kind, T, d) and kept resident in HBM.

    abs    : PositionalEncoding pe[:T]                         (embedding.py:35-94)
    latest : RelPositionalEncoding, rows k = PE(T-1-k), 2T-1    (embedding.py:173-244)
    legacy : LegacyRelPositionalEncoding, rows k = PE(max-1-k)  (embedding.py:133-170)
    """
    key = (kind, T, d, str(device), max_len)
    t = _PE_CACHE.get(key)
    if t is not None:
        return t
    n = max(max_len, T)
    if kind == "abs":
        tab = _pe_rows(torch.arange(0, n, dtype=torch.float32), d)[:T]
    elif kind == "legacy":
        tab = _pe_rows(torch.arange(n - 1, -1, -1.0, dtype=torch.float32), d)[:T]
    elif kind == "latest":
        position = torch.arange(0, n, dtype=torch.float32)
        pos = _pe_rows(position, d)
        neg = torch.zeros(n, d)
        div_term = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
        neg[:, 0::2] = torch.sin(-1 * position.unsqueeze(1) * div_term)
        neg[:, 1::2] = torch.cos(-1 * position.unsqueeze(1) * div_term)
        full = torch.cat([torch.flip(pos, [0]), neg[1:]], dim=0)
        c = full.size(0) // 2
        tab = full[c - T + 1: c + T]
    else:
        raise ValueError(kind)
    t = tab.contiguous().to(device)
    _PE_CACHE[key] = t
    return t


def draw_seed() -> int:
    """64-bit dropout key from torch's CPU generator (reproducible under torch.manual_seed)."""
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def lengths_to_device(lens: torch.Tensor, device) -> torch.Tensor:
    return K.h2d(lens.to(torch.int32), device)


class EncoderFn(torch.autograd.Function):
    """Runs an encoder's explicit forward; its backward writes parameter gradients into the
    flat gradient buffer (flat.py) and returns no input gradient (fbank needs none)."""

    @staticmethod
    def forward(ctx, feats, anchor, enc, ilens_cpu, seed, grad_hook, klen=None, tvalid=None, inter=None):
        kw = {} if inter is None else {"inter": inter}
        hs, olens, saved = enc.run_forward(feats, ilens_cpu, Seeds(seed), enc.training, klen=klen, tvalid=tvalid, **kw)
        ctx.enc = enc
        ctx.saved = saved
        ctx.grad_hook = grad_hook
        ctx.olens = olens
        return hs

    @staticmethod
    def backward(ctx, dhs):
        ctx.enc.run_backward(ctx.saved, dhs.contiguous(), ctx.grad_hook)
        ctx.saved = None
        return None, None, None, None, None, None, None, None, None
