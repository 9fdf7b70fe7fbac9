"""SpecAug — drop-in for espnet2/asr/specaug/specaug.py:13-96 (TimeWarp + freq/time masks).

The random draws follow the reference's calls (time_warp.py:25-27, mask_along_axis.py:32-44)
on torch's CPU generator; the warp + masking itself is one HIP kernel over the batch
(bicubic resampling identical to upsample_bicubic2d, align_corners=False).  `draws` can be
injected for parity tests (the reference draws from the CPU and the device generators).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple, Union

import torch

from ... import kernels as K


class AbsSpecAug(torch.nn.Module):
    def forward(self, x, x_lengths=None):
        raise NotImplementedError


class SpecAug(AbsSpecAug):
    def __init__(self, apply_time_warp: bool = True, time_warp_window: int = 5, time_warp_mode: str = "bicubic",
                 apply_freq_mask: bool = True, freq_mask_width_range: Union[int, Sequence[int]] = (0, 20),
                 num_freq_mask: int = 2, apply_time_mask: bool = True,
                 time_mask_width_range: Optional[Union[int, Sequence[int]]] = None,
                 time_mask_width_ratio_range: Optional[Union[float, Sequence[float]]] = None,
                 num_time_mask: int = 2):
        if not apply_time_warp and not apply_time_mask and not apply_freq_mask:
            raise ValueError("Either one of time_warp, time_mask, or freq_mask should be applied")
        if apply_time_mask and (time_mask_width_range is not None) and (time_mask_width_ratio_range is not None):
            raise ValueError('Either one of "time_mask_width_range" or "time_mask_width_ratio_range" can be used')
        if apply_time_mask and time_mask_width_range is None and time_mask_width_ratio_range is None:
            raise ValueError('Either one of "time_mask_width_range" or "time_mask_width_ratio_range" should be used.')
        if apply_time_warp and time_warp_mode != "bicubic":
            raise NotImplementedError("time_warp_mode other than bicubic")
        super().__init__()
        self.apply_time_warp = apply_time_warp
        self.window = time_warp_window
        self.apply_freq_mask = apply_freq_mask
        self.apply_time_mask = apply_time_mask
        if isinstance(freq_mask_width_range, int):
            freq_mask_width_range = (0, freq_mask_width_range)
        if isinstance(time_mask_width_range, int):
            time_mask_width_range = (0, time_mask_width_range)
        if isinstance(time_mask_width_ratio_range, float):
            time_mask_width_ratio_range = (0.0, time_mask_width_ratio_range)
        self.freq_range = tuple(freq_mask_width_range) if apply_freq_mask else None
        self.num_freq_mask = num_freq_mask
        self.time_range = tuple(time_mask_width_range) if time_mask_width_range is not None else None
        self.time_ratio = tuple(time_mask_width_ratio_range) if time_mask_width_ratio_range is not None else None
        self.num_time_mask = num_time_mask

    # ---------------------------------------------------------------- draws
    def _draw_warp(self, T: int, lens):
        """time_warp.py:25-27 + TimeWarp.forward :73-86 (shared warp when lengths are equal)."""
        w = self.window
        B = len(lens)
        warp = torch.zeros(B, 2, dtype=torch.int32)
        equal = all(int(l) == int(lens[0]) for l in lens)
        if equal:
            t = T
            if t - w > w:
                center = torch.randint(w, t - w, (1,))[0]
                warped = torch.randint(center - w, center + w, (1,))[0] + 1
                warp[:, 0] = int(center)
                warp[:, 1] = int(warped)
        else:
            for i in range(B):
                t = int(lens[i])
                if t - w > w:
                    center = torch.randint(w, t - w, (1,))[0]
                    warped = torch.randint(center - w, center + w, (1,))[0] + 1
                    warp[i, 0] = int(center)
                    warp[i, 1] = int(warped)
        return warp

    @staticmethod
    def _draw_mask(B, D, rng, num_mask):
        """mask_along_axis.py:32-44: widths U[lo,hi), positions U[0, max(1, D - max width))."""
        ml = torch.randint(rng[0], rng[1], (B, num_mask))
        mp = torch.randint(0, max(1, D - int(ml.max())), (B, num_mask))
        return torch.stack([mp, ml], dim=-1).to(torch.int32)

    def draw(self, B: int, T: int, F: int, lens) -> dict:
        d = {}
        if self.apply_time_warp:
            d["warp"] = self._draw_warp(T, lens)
        if self.apply_freq_mask:
            d["fmask"] = self._draw_mask(B, F, self.freq_range, self.num_freq_mask)
        if self.apply_time_mask:
            rng = self.time_range
            if rng is None:
                lo = max(0, math.floor(T * self.time_ratio[0]))
                hi = min(T, math.floor(T * self.time_ratio[1]))
                rng = (lo, hi) if hi > lo else None
            if rng is not None:
                d["tmask"] = self._draw_mask(B, T, rng, self.num_time_mask)
        return d

    def forward(self, x: torch.Tensor, x_lengths: torch.Tensor = None, draws: Optional[dict] = None
                ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        B, T, F = x.shape
        lens = x_lengths.detach().cpu() if x_lengths is not None else torch.full((B,), T)
        if draws is None:
            draws = self.draw(B, T, F, lens.tolist())
        dev = x.device
        ddev = {k: K.h2d(v, dev) for k, v in draws.items()}
        return self.apply_prepared(x, K.h2d(lens.to(torch.int32), dev), ddev), x_lengths

    @staticmethod
    def apply_prepared(x: torch.Tensor, lens_i32: torch.Tensor, draws_dev: dict) -> torch.Tensor:
        """Warp + masks from device-resident lengths and draws (one kernel, graph-capturable)."""
        y = torch.empty_like(x)
        K.specaug(x.contiguous(), y, lens_i32, draws_dev.get("warp"), draws_dev.get("fmask"), draws_dev.get("tmask"))
        return y
