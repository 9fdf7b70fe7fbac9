"""`kaldi_ark` loader: feats.scp ("key /path/x.ark:offset") -> np.ndarray
(espnet2/train/dataset.py:231-238, where the reference calls kaldiio.load_scp; kaldiio is
absent from this image, so this module reads Kaldi's binary holder format itself).

Binary holders supported: float / double matrices ("FM " / "DM ") and vectors ("FV " /
"DV "): "\\0B" marker, type token, then "\\4"<int32 rows>["\\4"<int32 cols>] and the raw
little-endian data.  Compressed matrices ("CM", "CM2", "CM3") and text-mode arks raise
NotImplementedError.  The offset in an scp line points at the "\\0B" marker (as Kaldi's
ark,scp writers emit).  Files stay open per path (one handle per worker process).
"""
import collections.abc
import struct
from typing import Dict, Iterator, Tuple

import numpy as np

from .read_text import read_2column_text

_TYPES = {b"FM ": (np.float32, 2), b"DM ": (np.float64, 2), b"FV ": (np.float32, 1), b"DV ": (np.float64, 1)}


def _read_holder(f, where: str) -> np.ndarray:
    if f.read(2) != b"\0B":
        raise NotImplementedError(f"{where}: only binary Kaldi holders are supported")
    tok = f.read(3)
    if tok not in _TYPES:
        raise NotImplementedError(f"{where}: holder type {tok!r} (compressed matrices are not supported)")
    dtype, ndim = _TYPES[tok]
    dims = []
    for _ in range(ndim):
        size_byte, n = struct.unpack("<bi", f.read(5))
        if size_byte != 4:
            raise RuntimeError(f"{where}: bad dimension header")
        dims.append(n)
    count = int(np.prod(dims))
    buf = f.read(count * np.dtype(dtype).itemsize)
    return np.frombuffer(buf, dtype=dtype, count=count).reshape(dims).copy()


def read_ark(path: str) -> Iterator[Tuple[str, np.ndarray]]:
    """Iterate (key, array) over a whole binary ark."""
    with open(path, "rb") as f:
        while True:
            key = bytearray()
            c = f.read(1)
            if not c:
                return
            while c not in (b" ", b""):
                key += c
                c = f.read(1)
            yield key.decode(), _read_holder(f, f"{path}:{key.decode()}")


def write_ark(path: str, items: Dict[str, np.ndarray]) -> Dict[str, str]:
    """Write float32/float64 matrices / vectors; returns the scp table {key: path:offset}."""
    scp = {}
    with open(path, "wb") as f:
        for key, a in items.items():
            a = np.asarray(a)
            tok = {(np.dtype(np.float32), 2): b"FM ", (np.dtype(np.float64), 2): b"DM ",
                   (np.dtype(np.float32), 1): b"FV ", (np.dtype(np.float64), 1): b"DV "}[(a.dtype, a.ndim)]
            f.write(key.encode() + b" ")
            scp[key] = f"{path}:{f.tell()}"
            f.write(b"\0B" + tok)
            for d in a.shape:
                f.write(struct.pack("<bi", 4, d))
            f.write(np.ascontiguousarray(a).astype(a.dtype.newbyteorder("<")).tobytes())
    return scp


class KaldiArkScpReader(collections.abc.Mapping):
    def __init__(self, fname):
        self.fname = fname
        self.data = read_2column_text(fname)
        self._files = {}

    def _open(self, path):
        f = self._files.get(path)
        if f is None:
            f = self._files[path] = open(path, "rb")
        return f

    def __getitem__(self, key) -> np.ndarray:
        spec = self.data[key]
        path, sep, off = spec.rpartition(":")
        if not sep or not off.isdigit():
            raise NotImplementedError(f"{spec}: expected 'path.ark:offset'")
        f = self._open(path)
        f.seek(int(off))
        return _read_holder(f, spec)

    def __getstate__(self):  # picklable for DataLoader workers: handles are reopened lazily
        d = dict(self.__dict__)
        d["_files"] = {}
        return d

    def __contains__(self, item):
        return item in self.data

    def __len__(self):
        return len(self.data)

    def __iter__(self):
        return iter(self.data)

    def keys(self):
        return self.data.keys()
