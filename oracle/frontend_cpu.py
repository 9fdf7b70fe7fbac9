"""CPU oracle for the feature front end: DefaultFrontend
(STFT -> power -> LogMel) and GlobalMVN.

TEST INFRASTRUCTURE ONLY (same rules as oracle/espnet_cpu.py: only `tests/`, `smoke()` and
`bench.py`'s CPU leg may import it, as the checker).

Restates, over plain tensors:
  * espnet2/asr/frontend/default.py:82-131  (DefaultFrontend.forward, single channel; the
    default `frontend_conf` Frontend is the identity for 3-D input,
    espnet/nets/pytorch_backend/frontends/frontend.py:88-128)
  * espnet2/layers/stft.py:63-160           (Stft.forward, torch.stft branch: center,
    reflect padding, periodic window, onesided; frames >= olens zeroed, :150-158)
  * espnet2/layers/log_mel.py:24-81         (LogMel: power @ melmat, clamp 1e-10, log, mask)
  * espnet2/layers/global_mvn.py:20-90      (stats -> mean / std, (x - mean) masked / std)
  * espnet2/asr/espnet_model.py _extract_feats (speech[:, :max(lengths)] before the front end)
The mel matrix comes from `librosa.filters.mel` (log_mel.py:51), a third-party dependency that
is absent here (setup.py:18 pins only `librosa>=0.8.0`).  `mel_filters` restates librosa's
published Slaney algorithm (mel_frequencies with the Slaney scale, triangular weights from
`subtract.outer(mel_f, fftfreqs)`, 'slaney' area normalisation, float32 output); the reference
holds no numeric mel fixture (test/espnet2/layers/test_log_mel.py checks shapes only), so the
mel matrix itself is PARITY UNPINNED.  The STFT, the LogMel forward (given a mel matrix) and
GlobalMVN are pinned by golden vectors from the reference modules themselves
(tests/golden/make_golden.py -> tests/golden/frontend.npz).
"""
from __future__ import annotations

import math
from typing import Tuple

import numpy as np
import torch


def hz_to_mel(f, htk: bool = False):
    """librosa.core.convert.hz_to_mel (Slaney: linear below 1 kHz, log above)."""
    f = np.asanyarray(f, dtype=np.float64)
    if htk:
        return 2595.0 * np.log10(1.0 + f / 700.0)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if mels.ndim:
        log_t = f >= min_log_hz
        mels[log_t] = min_log_mel + np.log(f[log_t] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def mel_to_hz(m, htk: bool = False):
    """librosa.core.convert.mel_to_hz."""
    m = np.asanyarray(m, dtype=np.float64)
    if htk:
        return 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    log_t = m >= min_log_mel
    freqs[log_t] = min_log_hz * np.exp(logstep * (m[log_t] - min_log_mel))
    return freqs


def mel_filters(sr: float, n_fft: int, n_mels: int = 80, fmin: float = 0.0, fmax: float = None,
                htk: bool = False) -> np.ndarray:
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk, norm='slaney', dtype=float32)
    -> (n_mels, 1 + n_fft // 2) float32."""
    if fmax is None:
        fmax = float(sr) / 2
    weights = np.zeros((n_mels, int(1 + n_fft // 2)), dtype=np.float32)
    fftfreqs = np.linspace(0, float(sr) / 2, int(1 + n_fft // 2), endpoint=True)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin, htk=htk), hz_to_mel(fmax, htk=htk), n_mels + 2), htk=htk)
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


def frame_lengths(ilens: torch.Tensor, n_fft: int, hop: int, center: bool = True) -> torch.Tensor:
    """stft.py:150-155: olens = (ilens + 2*(n_fft//2) - n_fft) // hop + 1 (center)."""
    if center:
        ilens = ilens + 2 * (n_fft // 2)
    return (ilens - n_fft) // hop + 1


def stft(x: torch.Tensor, ilens: torch.Tensor, n_fft: int = 512, hop: int = 128, win_length: int = None,
         center: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """stft.py:63-160 (single channel, hann window, onesided, not normalized):
    x (B, N) -> (B, frames, n_fft//2 + 1, 2), olens; frames >= olens zeroed."""
    win_length = win_length or n_fft
    window = torch.hann_window(win_length, dtype=x.dtype)
    out = torch.stft(x, n_fft=n_fft, win_length=win_length, hop_length=hop, center=center, window=window,
                     normalized=False, onesided=True, return_complex=False)
    out = out.transpose(1, 2)
    olens = frame_lengths(ilens, n_fft, hop, center)
    t = torch.arange(out.shape[1])
    mask = t[None, :] >= olens[:, None]
    out = out.masked_fill(mask[:, :, None, None], 0.0)
    return out, olens


def log_mel(power: torch.Tensor, olens: torch.Tensor, melmat: torch.Tensor) -> torch.Tensor:
    """log_mel.py:57-81 (log_base None): matmul, clamp(1e-10), log, zero the padded frames.
    melmat: (n_fft//2 + 1, n_mels) as registered by LogMel (melmat.T)."""
    mel = torch.clamp(torch.matmul(power, melmat), min=1e-10)
    out = mel.log()
    t = torch.arange(out.shape[1])
    return out.masked_fill((t[None, :] >= olens[:, None])[:, :, None], 0.0)


def default_frontend(speech: torch.Tensor, speech_lengths: torch.Tensor, fs: int = 16000, n_fft: int = 512,
                     hop: int = 128, n_mels: int = 80, fmin: float = None, fmax: float = None,
                     htk: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """espnet_model._extract_feats + default.py:82-131 for single-channel input."""
    speech = speech[:, : int(speech_lengths.max())]
    spec, olens = stft(speech, speech_lengths, n_fft, hop)
    power = spec[..., 0] ** 2 + spec[..., 1] ** 2
    fmin = 0 if fmin is None else fmin
    fmax = fs / 2 if fmax is None else fmax
    melmat = torch.from_numpy(mel_filters(fs, n_fft, n_mels, fmin, fmax, htk).T).float()
    return log_mel(power, olens, melmat), olens


def global_mvn_stats(stats: dict, eps: float = 1.0e-20) -> Tuple[np.ndarray, np.ndarray]:
    """global_mvn.py:40-58 for the dict (npz) form: mean, std (float64)."""
    count = stats["count"]
    mean = stats["sum"] / count
    var = stats["sum_square"] / count - mean * mean
    return mean, np.sqrt(np.maximum(var, eps))


def global_mvn(x: torch.Tensor, ilens: torch.Tensor, mean: np.ndarray, std: np.ndarray,
               norm_means: bool = True, norm_vars: bool = True) -> torch.Tensor:
    """global_mvn.py:67-90: (x - mean), padded frames zeroed, / std (mean/std cast to x.dtype)."""
    m = torch.from_numpy(np.asarray(mean)).to(x.dtype)
    s = torch.from_numpy(np.asarray(std)).to(x.dtype)
    t = torch.arange(x.shape[1])
    mask = (t[None, :] >= ilens[:, None])[:, :, None]
    if norm_means:
        x = x - m
    x = x.masked_fill(mask, 0.0)
    if norm_vars:
        x = x / s
    return x
