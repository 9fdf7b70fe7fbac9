"""`sound` loader: "key /path/x.wav" scp -> (rate, samples) (espnet2/fileio/sound_scp.py:8-66).

The reference reads through libsndfile (`soundfile`, absent from this image); this reader
parses RIFF/WAVE PCM itself (8/16/24/32-bit integer and 32/64-bit float data chunks).  With
normalize=True (what ESPnetDataset's "sound" type uses, dataset.py:202-209) integer PCM is
scaled like libsndfile's float read: int16 / 2^15, int32 / 2^31, 24-bit / 2^23, uint8
(x - 128) / 2^7, returned as float64; otherwise the raw integers (dtype kwarg, default int16).
always_2d keeps a (samples, channels) array for mono files too.  Compressed formats (FLAC,
MP3) raise NotImplementedError: convert them to PCM WAV in data preparation.
"""
import collections.abc
import struct
from pathlib import Path
from typing import Tuple, Union

import numpy as np

from .read_text import read_2column_text


def read_wav(path: Union[str, Path], normalize: bool = True, dtype=np.int16,
             always_2d: bool = False) -> Tuple[np.ndarray, int]:
    with open(path, "rb") as f:
        blob = f.read()
    if blob[:4] == b"fLaC":
        # the SLURP recipe dumps FLAC by default (asr.sh --audio_format flac); no FLAC decoder is
        # available here (soundfile / libFLAC are absent): dump the corpus as WAV instead
        raise NotImplementedError(f"{path}: FLAC audio is not supported; re-run the recipe's data dump with "
                                  "--audio_format wav (asr.sh stage 3) or convert the files to PCM WAV")
    if len(blob) < 12 or blob[:4] != b"RIFF" or blob[8:12] != b"WAVE":
        raise NotImplementedError(f"{path}: not a RIFF/WAVE file (only PCM WAV is supported)")
    pos, fmt, data = 12, None, None
    while pos + 8 <= len(blob):
        cid, size = blob[pos:pos + 4], struct.unpack_from("<I", blob, pos + 4)[0]
        body = blob[pos + 8: pos + 8 + size]
        if cid == b"fmt ":
            tag, nch, rate, _, _, bits = struct.unpack_from("<HHIIHH", body, 0)
            if tag == 0xFFFE and len(body) >= 26:  # WAVE_FORMAT_EXTENSIBLE: sub-format GUID
                tag = struct.unpack_from("<H", body, 24)[0]
            fmt = (tag, nch, rate, bits)
        elif cid == b"data":
            data = body
        pos += 8 + size + (size & 1)
    if fmt is None or data is None:
        raise RuntimeError(f"{path}: missing fmt or data chunk")
    tag, nch, rate, bits = fmt
    if tag == 1:  # integer PCM
        width = bits // 8
        n = len(data) // width
        if width == 1:
            raw = np.frombuffer(data, np.uint8, n)
            x = (raw.astype(np.float64) - 128.0) / 128.0 if normalize else raw.astype(np.int16) - 128
        elif width == 3:
            b = np.frombuffer(data, np.uint8, n * 3).reshape(n, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = v / float(1 << 23) if normalize else v
        elif width in (2, 4):
            raw = np.frombuffer(data, np.int16 if width == 2 else np.int32, n)
            x = raw / float(1 << (8 * width - 1)) if normalize else raw
        else:
            raise NotImplementedError(f"{path}: {bits}-bit PCM")
    elif tag == 3:  # IEEE float
        x = np.frombuffer(data, np.float32 if bits == 32 else np.float64).astype(np.float64)
    else:
        raise NotImplementedError(f"{path}: WAVE format tag {tag} (only PCM / IEEE float)")
    x = np.asarray(x)
    if not normalize and tag == 1:
        x = x.astype(dtype)
    x = x.reshape(-1, nch)
    if nch == 1 and not always_2d:
        x = x[:, 0]
    return np.ascontiguousarray(x), rate


class SoundScpReader(collections.abc.Mapping):
    def __init__(self, fname, dtype=np.int16, always_2d: bool = False, normalize: bool = False):
        self.fname = fname
        self.dtype = dtype
        self.always_2d = always_2d
        self.normalize = normalize
        self.data = read_2column_text(fname)

    def __getitem__(self, key):
        array, rate = read_wav(self.data[key], self.normalize, self.dtype, self.always_2d)
        return rate, array

    def get_path(self, key):
        return self.data[key]

    def __contains__(self, item):
        return item in self.data

    def __len__(self):
        return len(self.data)

    def __iter__(self):
        return iter(self.data)

    def keys(self):
        return self.data.keys()


def write_wav(path, x: np.ndarray, rate: int):
    """16-bit PCM writer (tests / data preparation)."""
    x = np.asarray(x)
    if x.dtype.kind == "f":
        x = np.clip(np.round(x * 32768.0), -32768, 32767).astype("<i2")
    x = x.astype("<i2")
    nch = 1 if x.ndim == 1 else x.shape[1]
    data = x.tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 1, nch, rate, rate * nch * 2, nch * 2, 16)
    hdr += b"data" + struct.pack("<I", len(data))
    with open(path, "wb") as f:
        f.write(hdr + data)
