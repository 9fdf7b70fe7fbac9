"""GlobalMVN — drop-in for espnet2/layers/global_mvn.py:11-90: statistics from the
`stats_file` (.npy matrix form or .npz dict form, loaded without pickle), buffers `mean` /
`std` (state_dict keys as the reference), forward = one in-place HIP kernel (esp_global_mvn)."""
from __future__ import annotations

from pathlib import Path
from typing import Tuple, Union

import numpy as np
import torch

from .. import kernels as K
from .utterance_mvn import AbsNormalize


class GlobalMVN(AbsNormalize):
    def __init__(self, stats_file: Union[Path, str], norm_means: bool = True, norm_vars: bool = True,
                 eps: float = 1.0e-20):
        super().__init__()
        self.norm_means, self.norm_vars, self.eps = norm_means, norm_vars, eps
        self.stats_file = Path(stats_file)
        stats = np.load(self.stats_file)  # allow_pickle=False (numpy default)
        if isinstance(stats, np.ndarray):  # global_mvn.py:42-45
            count = stats[0].flatten()[-1]
            mean = stats[0, :-1] / count
            var = stats[1, :-1] / count - mean * mean
        else:  # global_mvn.py:46-51
            count = stats["count"]
            mean = stats["sum"] / count
            var = stats["sum_square"] / count - mean * mean
        std = np.sqrt(np.maximum(var, eps))
        self.register_buffer("mean", torch.from_numpy(np.asarray(mean)))
        self.register_buffer("std", torch.from_numpy(np.asarray(std)))

    def _f32(self, device):
        return self.mean.to(device, torch.float32).contiguous(), self.std.to(device, torch.float32).contiguous()

    def apply_prepared(self, x: torch.Tensor, lens_i32: torch.Tensor) -> torch.Tensor:
        y = x.contiguous().clone() if x.requires_grad else x.contiguous()
        m, s = self._f32(y.device)
        K.global_mvn(y, lens_i32, m, s, self.norm_means, self.norm_vars)
        return y

    def forward(self, x: torch.Tensor, ilens: torch.Tensor = None) -> Tuple[torch.Tensor, torch.Tensor]:
        B, T, _ = x.shape
        if ilens is None:
            ilens = torch.full((B,), T, dtype=torch.long)
        return self.apply_prepared(x, K.h2d(ilens.to(torch.int32), x.device)), ilens
