"""UtteranceMVN — drop-in for espnet2/layers/utterance_mvn.py:10-88 (norm_means=True,
norm_vars=False, the espnet2 ASR default): one HIP kernel (per-utterance mean over the
valid frames, subtracted from every frame; padded frames become -mean as in the reference)."""
from __future__ import annotations

from typing import Tuple

import torch

from .. import kernels as K


class AbsNormalize(torch.nn.Module):
    def forward(self, input, input_lengths=None):
        raise NotImplementedError


class UtteranceMVN(AbsNormalize):
    def __init__(self, norm_means: bool = True, norm_vars: bool = False, eps: float = 1.0e-20):
        super().__init__()
        if not norm_means or norm_vars:
            raise NotImplementedError("UtteranceMVN: only norm_means=True, norm_vars=False is on the hot path")
        self.norm_means = norm_means
        self.norm_vars = norm_vars
        self.eps = eps

    def forward(self, x: torch.Tensor, ilens: torch.Tensor = None) -> Tuple[torch.Tensor, torch.Tensor]:
        B, T, F = x.shape
        if ilens is None:
            ilens = torch.full((B,), T, dtype=torch.long)
        return self.apply_prepared(x, K.h2d(ilens.to(torch.int32), x.device)), ilens

    @staticmethod
    def apply_prepared(x: torch.Tensor, lens_i32: torch.Tensor) -> torch.Tensor:
        y = x.contiguous().clone() if x.requires_grad else x.contiguous()
        K.utterance_mvn(y, lens_i32)
        return y
