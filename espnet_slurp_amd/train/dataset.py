"""ESPnetDataset (espnet2/train/dataset.py:355-540): {name: (path, type)} -> uid -> {name: ndarray}.

Loader types (dataset.py:201-300): sound (PCM WAV, fileio/sound_scp.py), kaldi_ark
(fileio/kaldi_ark.py), npy, text_int / csv_int / text_float / csv_float (numeric text
tables), text (raw strings; a preprocess callable must turn them into arrays).  score,
duration, rand_float / rand_int and hdf5 are outside this build's scope and raise ValueError
like any unknown type.  After the optional preprocess every value is cast: floating -> float_dtype,
integer -> int_dtype (dataset.py:517-528); other kinds raise NotImplementedError.
"""
import collections.abc
import numbers
from typing import Callable, Collection, Dict, Mapping, Optional, Tuple, Union

import numpy as np
import torch

from ..fileio.kaldi_ark import KaldiArkScpReader
from ..fileio.npy_scp import NpyScpReader
from ..fileio.read_text import load_num_sequence_text, read_2column_text
from ..fileio.sound_scp import SoundScpReader


class AdapterForSoundScpReader(collections.abc.Mapping):
    """(rate, array) -> array with a consistent sampling rate (dataset.py:26-84)."""

    def __init__(self, loader, dtype=None):
        self.loader, self.dtype, self.rate = loader, dtype, None

    def keys(self):
        return self.loader.keys()

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        return iter(self.loader)

    def __getitem__(self, key) -> np.ndarray:
        v = self.loader[key]
        if isinstance(v, tuple):
            assert len(v) == 2, len(v)
            if isinstance(v[0], int) and isinstance(v[1], np.ndarray):
                rate, arr = v
            elif isinstance(v[1], int) and isinstance(v[0], np.ndarray):
                arr, rate = v
            else:
                raise RuntimeError(f"Unexpected type: {type(v[0])}, {type(v[1])}")
            if self.rate is not None and self.rate != rate:
                raise RuntimeError(f"Sampling rates are mismatched: {self.rate} != {rate}")
            self.rate = rate
        else:
            arr = v
        assert isinstance(arr, np.ndarray), type(arr)
        return arr.astype(self.dtype) if self.dtype is not None else arr


def _make_loader(path: str, loader_type: str, float_dtype: str):
    if loader_type == "sound":
        return AdapterForSoundScpReader(SoundScpReader(path, always_2d=False, normalize=True), float_dtype)
    if loader_type == "kaldi_ark":
        return AdapterForSoundScpReader(KaldiArkScpReader(path), float_dtype)
    if loader_type == "npy":
        return NpyScpReader(path)
    if loader_type in ("text_int", "csv_int", "text_float", "csv_float"):
        return load_num_sequence_text(path, loader_type)
    if loader_type == "text":
        return read_2column_text(path)
    raise ValueError(f"Not supported: loader_type={loader_type}")


DATA_TYPES = ("sound", "kaldi_ark", "npy", "text_int", "csv_int", "text_float", "csv_float", "text")


class ESPnetDataset(torch.utils.data.Dataset):
    def __init__(self, path_name_type_list: Collection[Tuple[str, str, str]],
                 preprocess: Optional[Callable[[str, Dict[str, np.ndarray]], Dict[str, np.ndarray]]] = None,
                 float_dtype: str = "float32", int_dtype: str = "long", max_cache_size: Union[float, int] = 0.0,
                 max_cache_fd: int = 0):
        if len(path_name_type_list) == 0:
            raise ValueError('1 or more elements are required for "path_name_type_list"')
        self.preprocess = preprocess
        self.float_dtype = float_dtype
        self.int_dtype = "int64" if int_dtype == "long" else int_dtype
        self.loader_dict: Dict[str, Mapping] = {}
        self.debug_info: Dict[str, Tuple[str, str]] = {}
        for path, name, _type in path_name_type_list:
            if name in self.loader_dict:
                raise RuntimeError(f'"{name}" is duplicated for data-key')
            loader = _make_loader(path, _type, float_dtype)
            self.loader_dict[name] = loader
            self.debug_info[name] = path, _type
            if len(loader) == 0:
                raise RuntimeError(f"{path} has no samples")
        self.cache = {} if max_cache_size > 0 else None

    def has_name(self, name) -> bool:
        return name in self.loader_dict

    def names(self) -> Tuple[str, ...]:
        return tuple(self.loader_dict)

    def __iter__(self):
        return iter(next(iter(self.loader_dict.values())))

    def __repr__(self):
        body = "".join(f'\n  {n}: {{"path": "{p}", "type": "{t}"}}' for n, (p, t) in self.debug_info.items())
        return f"{self.__class__.__name__}({body}\n  preprocess: {self.preprocess})"

    def __getitem__(self, uid: Union[str, int]) -> Tuple[str, Dict[str, np.ndarray]]:
        if isinstance(uid, int):
            uid = list(next(iter(self.loader_dict.values())))[uid]
        if self.cache is not None and uid in self.cache:
            return uid, self.cache[uid]
        data = {}
        for name, loader in self.loader_dict.items():
            v = loader[uid]
            if isinstance(v, list):
                v = np.array(v)
            if isinstance(v, torch.Tensor):
                v = v.numpy()
            elif isinstance(v, numbers.Number):
                v = np.array([v])
            elif not isinstance(v, (np.ndarray, str, tuple)):
                raise TypeError(f"Must be ndarray, torch.Tensor, str,  Number or tuple: {type(v)}")
            data[name] = v
        if self.preprocess is not None:
            data = self.preprocess(uid, data)
        for name, v in list(data.items()):
            if not isinstance(v, np.ndarray):
                raise RuntimeError(f"All values must be converted to np.ndarray object by preprocessing, "
                                   f'but "{name}" is still {type(v)}.')
            if v.dtype.kind == "f":
                data[name] = v.astype(self.float_dtype)
            elif v.dtype.kind == "i":
                data[name] = v.astype(self.int_dtype)
            else:
                raise NotImplementedError(f"Not supported dtype: {v.dtype}")
        if self.cache is not None:
            self.cache[uid] = data
        return uid, data
