"""CommonCollateFn (espnet2/train/collate_fn.py:10-99): list of (utt_id, {name: ndarray}) ->
(utt_ids, {name: padded tensor, name_lengths: int64 lengths}).

Integer arrays are padded with int_pad_value (the ASR task passes -1, asr.py:365), floats with
float_pad_value; the first axis is the sequence axis; names in not_sequence get no *_lengths.
The padded batch is assembled in ONE preallocated buffer per name (optionally page-locked, so
the host->device copy of the batch is a single asynchronous DMA: see DevicePrefetcher in
iterators/sequence_iter_factory.py) instead of a per-utterance tensor list.
"""
from typing import Collection, Dict, List, Tuple, Union

import numpy as np
import torch


def common_collate_fn(data: Collection[Tuple[str, Dict[str, np.ndarray]]], float_pad_value: Union[float, int] = 0.0,
                      int_pad_value: int = -32768, not_sequence: Collection[str] = (),
                      pin_memory: bool = False) -> Tuple[List[str], Dict[str, torch.Tensor]]:
    ids = [u for u, _ in data]
    items = [d for _, d in data]
    names = list(items[0])
    assert all(set(names) == set(d) for d in items), "dict-keys mismatching"
    assert all(not k.endswith("_lengths") for k in names), f"*_lengths is reserved: {names}"
    out: Dict[str, torch.Tensor] = {}
    for name in names:
        arrs = [np.asarray(d[name]) for d in items]
        pad = int_pad_value if arrs[0].dtype.kind == "i" else float_pad_value
        lens = [a.shape[0] for a in arrs]
        tail = arrs[0].shape[1:]
        dtype = torch.from_numpy(arrs[0][:0]).dtype
        buf = torch.empty((len(arrs), max(lens)) + tuple(tail), dtype=dtype, pin_memory=pin_memory)
        buf.fill_(pad)
        view = buf.numpy()
        for i, a in enumerate(arrs):
            view[i, : a.shape[0]] = a
        out[name] = buf
        if name not in not_sequence:
            out[name + "_lengths"] = torch.tensor(lens, dtype=torch.long)
    return ids, out


class CommonCollateFn:
    """Functor of common_collate_fn (collate_fn.py:10-37)."""

    def __init__(self, float_pad_value: Union[float, int] = 0.0, int_pad_value: int = -32768,
                 not_sequence: Collection[str] = (), pin_memory: bool = False):
        self.float_pad_value = float_pad_value
        self.int_pad_value = int_pad_value
        self.not_sequence = set(not_sequence)
        self.pin_memory = pin_memory

    def __repr__(self):
        return f"{self.__class__}(float_pad_value={self.float_pad_value}, int_pad_value={self.float_pad_value})"

    def __call__(self, data):
        return common_collate_fn(data, float_pad_value=self.float_pad_value, int_pad_value=self.int_pad_value,
                                 not_sequence=self.not_sequence, pin_memory=self.pin_memory)
