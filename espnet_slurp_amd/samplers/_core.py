"""Batch samplers of the espnet2 data feed, restated.

Every sampler turns shape files ("utt L,D,..." per line) into a fixed list of key tuples; the
iterator factory shuffles that list per epoch.  Batch compositions are identical to the
reference's for the same files (tests/test_data_feed.py against golden lists generated from
the reference samplers).  Shared rules (num_elements_batch_sampler.py:57-157,
folded_batch_sampler.py:48-151, length_batch_sampler.py:45-140):
  * keys are ordered by the first shape file's leading length, ascending, stable;
  * a batch is closed as soon as its cost exceeds the budget and it holds >= min_batch_size
    keys (the key that crossed the budget stays in the batch);
  * a last batch smaller than min_batch_size is dealt out one key at a time to the earlier
    batches, from the back (numel / length: starting with the last remaining batch; folded:
    starting one before it — the reference's index offsets differ, reproduced here);
  * sort_in_batch "descending" reverses each batch, sort_batch "descending" reverses the list.
"""
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from ..fileio.read_text import load_num_sequence_text, read_2column_text


def _check_orders(sort_in_batch, sort_batch):
    if sort_batch not in ("ascending", "descending"):
        raise ValueError(f"sort_batch must be ascending or descending: {sort_batch}")
    if sort_in_batch not in ("ascending", "descending"):
        raise ValueError(f"sort_in_batch must be ascending or descending: {sort_in_batch}")


def _load_shapes(shape_files) -> Tuple[List[Dict[str, list]], List[str]]:
    tables = [load_num_sequence_text(s, loader_type="csv_int") for s in shape_files]
    ref = set(tables[0])
    for path, t in zip(shape_files, tables):
        if set(t) != ref:
            raise RuntimeError(f"keys are mismatched between {path} != {shape_files[0]}")
    keys = sorted(tables[0], key=lambda k: tables[0][k][0])
    if not keys:
        raise RuntimeError(f"0 lines found: {shape_files[0]}")
    return tables, keys


def _fold_small_tail(sizes: List[int], min_batch_size: int, back: int):
    if len(sizes) > 1 and sizes[-1] < min_batch_size:
        tail = sizes.pop()
        for i in range(tail):
            sizes[-(i % len(sizes)) - back] += 1


def _cut(keys: Sequence[str], sizes: Sequence[int], sort_in_batch: str) -> List[Tuple[str, ...]]:
    out, start = [], 0
    for n in sizes:
        chunk = list(keys[start:start + n])
        start += n
        if len(chunk) < n:
            break
        if sort_in_batch == "descending":
            chunk.reverse()
        out.append(tuple(chunk))
    return out


class AbsSampler:
    batch_list: List[Tuple[str, ...]]

    def __len__(self):
        return len(self.batch_list)

    def __iter__(self) -> Iterator[Tuple[str, ...]]:
        return iter(self.batch_list)

    def generate(self, seed):
        return list(self)


def _budget_sizes(costs_fn, n_keys: int, budget: int, min_batch_size: int, drop_last: bool) -> List[int]:
    """Greedy batch sizes: costs_fn(first, last) is the cost of keys[first..last]."""
    sizes, first = [], 0
    for last in range(n_keys):
        if costs_fn(first, last) > budget and last - first + 1 >= min_batch_size:
            sizes.append(last - first + 1)
            first = last + 1
    if first < n_keys and (not drop_last or not sizes):
        sizes.append(n_keys - first)
    if not sizes:
        raise RuntimeError("0 batches")
    return sizes


class NumElementsBatchSampler(AbsSampler):
    """Budget on elements: padded (batch x longest x feat dims) summed over the shape files,
    or, with padding=False, the sum of every key's element count."""

    def __init__(self, batch_bins: int, shape_files, min_batch_size: int = 1, sort_in_batch: str = "descending",
                 sort_batch: str = "ascending", drop_last: bool = False, padding: bool = True):
        assert batch_bins > 0
        _check_orders(sort_in_batch, sort_batch)
        self.batch_bins, self.shape_files = batch_bins, shape_files
        self.sort_in_batch, self.sort_batch, self.drop_last = sort_in_batch, sort_batch, drop_last
        tables, keys = _load_shapes(shape_files)
        if padding:
            for path, t in zip(shape_files, tables):
                dims0 = tuple(t[keys[0]][1:])
                if any(tuple(t[k][1:]) != dims0 for k in keys):
                    raise RuntimeError(f"If padding=True, the feature dimension must be unified: {path}")
            per = np.zeros(len(keys), dtype=np.int64)  # sum_files len(key) * prod(feat dims)
            for t in tables:
                fd = int(np.prod(t[keys[0]][1:]))
                per += np.array([t[k][0] for k in keys], dtype=np.int64) * fd
            cost = lambda a, b: (b - a + 1) * int(per[b])  # noqa: E731 (keys ascending: b is longest)
        else:
            tot = np.zeros(len(keys) + 1, dtype=np.int64)
            tot[1:] = np.cumsum([sum(int(np.prod(t[k])) for t in tables) for k in keys])
            cost = lambda a, b: int(tot[b + 1] - tot[a])  # noqa: E731
        sizes = _budget_sizes(cost, len(keys), batch_bins, min_batch_size, drop_last)
        _fold_small_tail(sizes, min_batch_size, back=1)
        if not drop_last:
            assert sum(sizes) == len(keys), f"{sum(sizes)} != {len(keys)}"
        self.batch_list = _cut(keys, sizes, sort_in_batch)
        if sort_batch == "descending":
            self.batch_list.reverse()

    def __repr__(self):
        return (f"{self.__class__.__name__}(N-batch={len(self)}, batch_bins={self.batch_bins}, "
                f"sort_in_batch={self.sort_in_batch}, sort_batch={self.sort_batch})")


class LengthBatchSampler(AbsSampler):
    """Budget on lengths only: batch x longest (padding) or the sum of lengths, over files."""

    def __init__(self, batch_bins: int, shape_files, min_batch_size: int = 1, sort_in_batch: str = "descending",
                 sort_batch: str = "ascending", drop_last: bool = False, padding: bool = True):
        assert batch_bins > 0
        _check_orders(sort_in_batch, sort_batch)
        self.batch_bins, self.shape_files = batch_bins, shape_files
        self.sort_in_batch, self.sort_batch, self.drop_last = sort_in_batch, sort_batch, drop_last
        tables, keys = _load_shapes(shape_files)
        lens = np.zeros(len(keys), dtype=np.int64)
        for t in tables:
            lens += np.array([t[k][0] for k in keys], dtype=np.int64)
        if padding:
            cost = lambda a, b: (b - a + 1) * int(lens[b])  # noqa: E731
        else:
            tot = np.concatenate([[0], np.cumsum(lens)])
            cost = lambda a, b: int(tot[b + 1] - tot[a])  # noqa: E731
        sizes = _budget_sizes(cost, len(keys), batch_bins, min_batch_size, drop_last)
        _fold_small_tail(sizes, min_batch_size, back=1)
        if not drop_last:
            assert sum(sizes) == len(keys), f"{sum(sizes)} != {len(keys)}"
        self.batch_list = _cut(keys, sizes, sort_in_batch)
        if sort_batch == "descending":
            self.batch_list.reverse()

    def __repr__(self):
        return (f"{self.__class__.__name__}(N-batch={len(self)}, batch_bins={self.batch_bins}, "
                f"sort_in_batch={self.sort_in_batch}, sort_batch={self.sort_batch})")


class FoldedBatchSampler(AbsSampler):
    """batch_size shrunk by 1 + max_i floor(len_i / fold_length_i) of each batch's FIRST
    (shortest) key, per category of utt2category (folded_batch_sampler.py:81-111)."""

    def __init__(self, batch_size: int, shape_files, fold_lengths: Sequence[int], min_batch_size: int = 1,
                 sort_in_batch: str = "descending", sort_batch: str = "ascending", drop_last: bool = False,
                 utt2category_file: Optional[str] = None):
        assert batch_size > 0
        _check_orders(sort_in_batch, sort_batch)
        self.batch_size, self.shape_files = batch_size, shape_files
        self.sort_in_batch, self.sort_batch, self.drop_last = sort_in_batch, sort_batch, drop_last
        tables, keys = _load_shapes(shape_files)
        groups: Dict[str, List[str]] = {}
        if utt2category_file is not None:
            cat = read_2column_text(utt2category_file)
            if set(cat) != set(tables[0]):
                raise RuntimeError(f"keys are mismatched between {utt2category_file} != {shape_files[0]}")
            for k in keys:
                groups.setdefault(cat[k], []).append(k)
        else:
            groups["default_category"] = keys
        self.batch_list = []
        for gkeys in groups.values():
            sizes, start = [], 0
            while True:
                k = gkeys[start]
                factor = max(int(t[k][0] / m) for t, m in zip(tables, fold_lengths))
                bs = max(min_batch_size, int(batch_size / (1 + factor)))
                if drop_last and start + bs > len(gkeys) and self.batch_list:
                    break
                bs = min(len(gkeys) - start, bs)
                sizes.append(bs)
                start += bs
                if start >= len(gkeys):
                    break
            if not sizes:
                raise RuntimeError("0 batches")
            _fold_small_tail(sizes, min_batch_size, back=2)
            if not drop_last:
                assert sum(sizes) == len(gkeys), f"{sum(sizes)} != {len(gkeys)}"
            part = _cut(gkeys, sizes, sort_in_batch)
            if sort_batch == "descending":
                part.reverse()
            self.batch_list.extend(part)

    def __repr__(self):
        return (f"{self.__class__.__name__}(N-batch={len(self)}, batch_size={self.batch_size}, "
                f"shape_files={self.shape_files}, sort_in_batch={self.sort_in_batch}, "
                f"sort_batch={self.sort_batch})")


class SortedBatchSampler(AbsSampler):
    """Keys sorted by length (sort_in_batch order), split into max(N // bs, 1) near-equal
    batches (sorted_batch_sampler.py:30-80); batches are tuples here (the reference yields
    lists when drop_last is False)."""

    def __init__(self, batch_size: int, shape_file: str, sort_in_batch: str = "descending",
                 sort_batch: str = "ascending", drop_last: bool = False):
        assert batch_size > 0
        self.batch_size, self.shape_file = batch_size, shape_file
        self.sort_in_batch, self.sort_batch, self.drop_last = sort_in_batch, sort_batch, drop_last
        shapes = load_num_sequence_text(shape_file, loader_type="csv_int")
        if sort_in_batch == "descending":
            keys = sorted(shapes, key=lambda k: -shapes[k][0])
        elif sort_in_batch == "ascending":
            keys = sorted(shapes, key=lambda k: shapes[k][0])
        else:
            raise ValueError(f"sort_in_batch must be either one of ascending, descending, or None: {sort_in_batch}")
        if not keys:
            raise RuntimeError(f"0 lines found: {shape_file}")
        n = max(len(keys) // batch_size, 1)
        if drop_last:
            self.batch_list = [tuple(keys[i * batch_size:(i + 1) * batch_size]) for i in range(n)]
        else:
            self.batch_list = [tuple(keys[i * len(keys) // n:(i + 1) * len(keys) // n]) for i in range(n)]
        if sort_in_batch != sort_batch:
            if sort_batch not in ("ascending", "descending"):
                raise ValueError(f"sort_batch must be ascending or descending: {sort_batch}")
            self.batch_list.reverse()

    def __repr__(self):
        return (f"{self.__class__.__name__}(N-batch={len(self)}, batch_size={self.batch_size}, "
                f"shape_file={self.shape_file}, sort_in_batch={self.sort_in_batch}, sort_batch={self.sort_batch})")


class UnsortedBatchSampler(AbsSampler):
    """File order, max(N // bs, 1) near-equal batches per category (unsorted_batch_sampler.py).
    As in the reference, the split points of a category use the TOTAL key count."""

    def __init__(self, batch_size: int, key_file: str, drop_last: bool = False,
                 utt2category_file: Optional[str] = None):
        assert batch_size > 0
        self.batch_size, self.key_file, self.drop_last = batch_size, key_file, drop_last
        keys = list(read_2column_text(key_file))
        if not keys:
            raise RuntimeError(f"0 lines found: {key_file}")
        groups: Dict[str, List[str]] = {}
        if utt2category_file is not None:
            cat = read_2column_text(utt2category_file)
            if set(cat) != set(keys):
                raise RuntimeError(f"keys are mismatched between {utt2category_file} != {key_file}")
            for k, v in cat.items():
                groups.setdefault(v, []).append(k)
        else:
            groups["default_category"] = keys
        self.batch_list = []
        for g in groups.values():
            n = max(len(g) // batch_size, 1)
            if drop_last:
                self.batch_list += [tuple(g[i * batch_size:(i + 1) * batch_size]) for i in range(n)]
            else:
                self.batch_list += [tuple(g[i * len(keys) // n:(i + 1) * len(keys) // n]) for i in range(n)]

    def __repr__(self):
        return f"{self.__class__.__name__}(N-batch={len(self)}, batch_size={self.batch_size}, key_file={self.key_file}, "


BATCH_TYPES = ("unsorted", "sorted", "folded", "numel", "length")


def build_batch_sampler(type: str, batch_size: int, batch_bins: int, shape_files, sort_in_batch: str = "descending",
                        sort_batch: str = "ascending", drop_last: bool = False, min_batch_size: int = 1,
                        fold_lengths: Sequence[int] = (), padding: bool = True,
                        utt2category_file: Optional[str] = None) -> AbsSampler:
    """espnet2/samplers/build_batch_sampler.py:78-162 (same argument names and errors)."""
    if len(shape_files) == 0:
        raise ValueError("No shape file are given")
    if type == "unsorted":
        return UnsortedBatchSampler(batch_size=batch_size, key_file=shape_files[0], drop_last=drop_last)
    if type == "sorted":
        return SortedBatchSampler(batch_size=batch_size, shape_file=shape_files[0], sort_in_batch=sort_in_batch,
                                  sort_batch=sort_batch, drop_last=drop_last)
    if type == "folded":
        if len(fold_lengths) != len(shape_files):
            raise ValueError(f"The number of fold_lengths must be equal to the number of shape_files: "
                             f"{len(fold_lengths)} != {len(shape_files)}")
        return FoldedBatchSampler(batch_size=batch_size, shape_files=shape_files, fold_lengths=fold_lengths,
                                  sort_in_batch=sort_in_batch, sort_batch=sort_batch, drop_last=drop_last,
                                  min_batch_size=min_batch_size, utt2category_file=utt2category_file)
    if type == "numel":
        return NumElementsBatchSampler(batch_bins=batch_bins, shape_files=shape_files, sort_in_batch=sort_in_batch,
                                       sort_batch=sort_batch, drop_last=drop_last, padding=padding,
                                       min_batch_size=min_batch_size)
    if type == "length":
        return LengthBatchSampler(batch_bins=batch_bins, shape_files=shape_files, sort_in_batch=sort_in_batch,
                                  sort_batch=sort_batch, drop_last=drop_last, padding=padding,
                                  min_batch_size=min_batch_size)
    raise ValueError(f"Not supported: {type}")
