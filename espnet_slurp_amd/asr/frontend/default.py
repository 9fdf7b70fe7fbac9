"""DefaultFrontend — drop-in for espnet2/asr/frontend/default.py:17-131 (single-channel,
`frontend_conf` enhancement off: the default Frontend is the identity for (B, T, F) input,
espnet/nets/pytorch_backend/frontends/frontend.py:88-128).

Same constructor kwargs, `output_size()`, `forward(input, input_lengths) -> (feats, lens)` and
the same state_dict buffer (`logmel.melmat`, (n_fft/2+1, n_mels), log_mel.py:53).  The whole
Stft -> power -> LogMel chain is ONE HIP kernel (esp_fbank_fwd, csrc/frontend.hip): one wave per
frame, FFT in LDS, HBM touched by the raw samples and the features only.  The mel matrix is
librosa.filters.mel's Slaney filterbank (log_mel.py:51), restated in `mel_filters` below (librosa
is not a dependency here).  No parameters, no backward (the reference's front end has none either).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np
import torch

from ... import kernels as K


def _hz_to_mel(f: float, htk: bool) -> float:
    if htk:
        return 2595.0 * math.log10(1.0 + f / 700.0)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    if f < min_log_hz:
        return f / f_sp
    return min_log_hz / f_sp + math.log(f / min_log_hz) / (math.log(6.4) / 27.0)


def _mel_to_hz(m: np.ndarray, htk: bool) -> np.ndarray:
    if htk:
        return 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel = min_log_hz / f_sp
    hz = f_sp * m
    t = m >= min_log_mel
    hz[t] = min_log_hz * np.exp(math.log(6.4) / 27.0 * (m[t] - min_log_mel))
    return hz


def mel_filters(fs: float, n_fft: int, n_mels: int, fmin: float, fmax: float, htk: bool) -> np.ndarray:
    """Slaney-normalised triangular mel filterbank, (n_mels, n_fft//2 + 1) float32 — the
    published algorithm of librosa.filters.mel(norm='slaney') that log_mel.py:51 calls."""
    nb = n_fft // 2 + 1
    fft_hz = np.linspace(0.0, fs / 2.0, nb)
    mel_hz = _mel_to_hz(np.linspace(_hz_to_mel(fmin, htk), _hz_to_mel(fmax, htk), n_mels + 2), htk)
    width = np.diff(mel_hz)
    rise = mel_hz[:, None] - fft_hz[None, :]
    w = np.zeros((n_mels, nb), dtype=np.float32)
    for m in range(n_mels):
        w[m] = np.maximum(0.0, np.minimum(-rise[m] / width[m], rise[m + 2] / width[m + 1]))
    w *= (2.0 / (mel_hz[2:] - mel_hz[:n_mels]))[:, None]
    return w


class LogMel(torch.nn.Module):
    """Holds the `melmat` buffer of log_mel.py:24-55 (state_dict key frontend.logmel.melmat)."""

    def __init__(self, fs: int = 16000, n_fft: int = 512, n_mels: int = 80, fmin: float = None,
                 fmax: float = None, htk: bool = False, log_base: float = None):
        super().__init__()
        if log_base is not None:
            raise NotImplementedError("LogMel: only the natural log (log_base=None) is on the hot path")
        fmin = 0 if fmin is None else fmin
        fmax = fs / 2 if fmax is None else fmax
        self.mel_options = dict(sr=fs, n_fft=n_fft, n_mels=n_mels, fmin=fmin, fmax=fmax, htk=htk)
        self.log_base = log_base
        self.register_buffer("melmat", torch.from_numpy(mel_filters(fs, n_fft, n_mels, fmin, fmax, htk).T.copy()))


class DefaultFrontend(torch.nn.Module):
    def __init__(self, fs=16000, n_fft: int = 512, win_length: int = None, hop_length: int = 128,
                 window: Optional[str] = "hann", center: bool = True, normalized: bool = False,
                 onesided: bool = True, n_mels: int = 80, fmin: int = None, fmax: int = None, htk: bool = False,
                 frontend_conf: Optional[dict] = None, apply_stft: bool = True):
        super().__init__()
        if isinstance(fs, str):  # humanfriendly.parse_size("16k") (default.py:44-45)
            s = fs.strip().lower()
            fs = int(float(s[:-1]) * 1000) if s.endswith("k") else int(s)
        if not (apply_stft and center and onesided and not normalized):
            raise NotImplementedError("DefaultFrontend: only apply_stft, center, onesided, not normalized")
        if frontend_conf and (frontend_conf.get("use_wpe") or frontend_conf.get("use_beamformer")):
            raise NotImplementedError("DefaultFrontend: WPE / beamformer (multi-channel) are not on the path")
        if window not in ("hann", None):
            raise NotImplementedError(f"DefaultFrontend: window {window}")
        self.n_fft, self.hop_length = n_fft, hop_length
        self.win_length = win_length or n_fft
        self.fs = fs
        self.logmel = LogMel(fs=fs, n_fft=n_fft, n_mels=n_mels, fmin=fmin, fmax=fmax, htk=htk)
        self.n_mels = n_mels
        self.frontend_type = "default"
        # window (periodic hann of win_length, centred in n_fft as torch.stft pads it), FFT twiddles
        wl = self.win_length
        win = torch.hann_window(wl, dtype=torch.float64) if window == "hann" else torch.ones(wl, dtype=torch.float64)
        full = torch.zeros(n_fft, dtype=torch.float64)
        left = (n_fft - wl) // 2
        full[left:left + wl] = win
        j = torch.arange(n_fft, dtype=torch.float64)  # full circle: the direct-DFT path indexes (f*k) mod n
        tw = torch.stack([torch.cos(2 * math.pi * j / n_fft), -torch.sin(2 * math.pi * j / n_fft)], -1)
        mel = self.logmel.melmat.numpy()
        nz = mel != 0
        lo = np.array([int(np.argmax(nz[:, m])) if nz[:, m].any() else 0 for m in range(n_mels)], dtype=np.int32)
        hi = np.array([int(nz.shape[0] - np.argmax(nz[::-1, m])) if nz[:, m].any() else 0 for m in range(n_mels)],
                      dtype=np.int32)
        self._tables = dict(window=full.float(), twiddle=tw.float().reshape(-1), lo=torch.from_numpy(lo),
                            hi=torch.from_numpy(hi))
        self._dev = {}

    def output_size(self) -> int:
        return self.n_mels

    def num_frames(self, n_samples: int) -> int:
        return n_samples // self.hop_length + 1  # center=True: (N + 2*(n_fft//2) - n_fft)//hop + 1

    def samples_for_frames(self, frames: int) -> int:
        """The sample count a length bucket of `frames` frames pads a batch to: the largest N with
        num_frames(N) == frames, so every batch whose frame count fits the bucket fits its samples."""
        return frames * self.hop_length - 1

    def output_lengths(self, speech_lengths: torch.Tensor) -> torch.Tensor:
        return speech_lengths // self.hop_length + 1  # stft.py:150-155

    def _device_tables(self, device):
        key = str(device)
        if key not in self._dev:
            t = {k: v.to(device) for k, v in self._tables.items()}
            t["melw"] = self.logmel.melmat.to(device).float().contiguous()
            self._dev[key] = t
        return self._dev[key]

    def apply_prepared(self, speech: torch.Tensor, wav_lens_i32: torch.Tensor, n_samples: int,
                       nvalid: torch.Tensor = None) -> torch.Tensor:
        """speech (B, >= n_samples) on device, wav_lens device int32 -> (B, T, n_mels) log-mel.
        nvalid (length buckets): device int32, the batch's own sample count (reflection point)."""
        B = speech.shape[0]
        x = speech if speech.dtype == torch.float32 else speech.float()
        if x.stride(1) != 1:
            x = x.contiguous()
        T = self.num_frames(n_samples)
        out = torch.empty(B, T, self.n_mels, dtype=torch.float32, device=x.device)
        t = self._device_tables(x.device)
        K.fbank_fwd(x, wav_lens_i32, B, n_samples, self.n_fft, self.hop_length, t["window"], t["twiddle"], t["melw"],
                    t["lo"], t["hi"], self.n_mels, out, T, nvalid=nvalid)
        return out

    def forward(self, input: torch.Tensor, input_lengths: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        lens = input_lengths.detach().cpu()
        n = int(lens.max())  # espnet_model._extract_feats: speech[:, :max(lengths)]
        feats = self.apply_prepared(input, K.h2d(lens.to(torch.int32), input.device), n)
        return feats, self.output_lengths(lens)
