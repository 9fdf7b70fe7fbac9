"""`npy` loader: "key /path/x.npy" scp -> np.load (espnet2/fileio/npy_scp.py:60-97).
Files are opened with allow_pickle=False (no object arrays execute anything)."""
import collections.abc
from pathlib import Path
from typing import Union

import numpy as np

from .read_text import read_2column_text


class NpyScpReader(collections.abc.Mapping):
    def __init__(self, fname: Union[Path, str]):
        self.fname = Path(fname)
        self.data = read_2column_text(fname)

    def get_path(self, key):
        return self.data[key]

    def __getitem__(self, key) -> np.ndarray:
        return np.load(self.data[key], allow_pickle=False)

    def __contains__(self, item):
        return item in self.data

    def __len__(self):
        return len(self.data)

    def __iter__(self):
        return iter(self.data)

    def keys(self):
        return self.data.keys()
