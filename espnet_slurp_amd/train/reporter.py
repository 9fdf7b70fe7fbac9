"""Reporter — the per-epoch statistics store of espnet2/train/reporter.py:24-580, restated for
the checkpoint interop row: `Reporter.state_dict()` is what the
reference writes into checkpoint.pth ({"stats": {epoch: {key: {key2: value}}}, "epoch": e},
reporter.py:575-580) and what its best-model selection / n-best averaging read
(sort_epochs_and_values, reporter.py:364-395).

Difference from the reference (by design): `SubReporter.register` accepts device tensors and
keeps them as they are; they are read back once, when the epoch is aggregated
(`finish_epoch`), instead of one host sync per registered value.  Aggregation semantics are the
reference's: plain values -> nanmean (Average), weighted -> weighted mean over finite
(value, weight) pairs (WeightedAverage, reporter.py:44-85); keys missing from a step are
nan-filled (reporter.py:137-151).  TensorBoard / wandb / matplotlib output is out of scope.
"""
from __future__ import annotations

import dataclasses
import datetime
import time
import warnings
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List, Optional, Tuple, Union

import numpy as np
import torch

Num = Union[float, int, complex, torch.Tensor, np.ndarray]
_reserved = {"time", "total_count"}


class ReportedValue:
    pass


@dataclasses.dataclass
class Average(ReportedValue):
    value: Num


@dataclasses.dataclass
class WeightedAverage(ReportedValue):
    value: Num
    weight: Num


def _scalar(v) -> float:
    if isinstance(v, (torch.Tensor, np.ndarray)):
        if int(np.prod(v.shape)) != 1:
            raise ValueError(f"v must be 0 or 1 dimension: {len(v.shape)}")
        return v.item()
    return v


def to_reported_value(v: Num, weight: Num = None):
    """reporter.py:24-41 (tensor values stay unresolved until aggregation)."""
    if isinstance(v, (torch.Tensor, np.ndarray)) and int(np.prod(v.shape)) != 1:
        raise ValueError(f"v must be 0 or 1 dimension: {len(v.shape)}")
    if isinstance(weight, (torch.Tensor, np.ndarray)) and int(np.prod(weight.shape)) != 1:
        raise ValueError(f"weight must be 0 or 1 dimension: {len(weight.shape)}")
    if weight is not None:
        return WeightedAverage(v, weight)
    return Average(v)


def _resolve(values):
    """Read every device tensor of a stats list back in ONE transfer."""
    dev = [x for r in values for x in ((r.value, r.weight) if isinstance(r, WeightedAverage) else (r.value,))
           if isinstance(x, torch.Tensor)]
    if dev:
        host = torch.stack([t.detach().reshape(()).double() for t in dev]).cpu().tolist()
        it = iter(host)
        out = []
        for r in values:
            if isinstance(r, WeightedAverage):
                v = next(it) if isinstance(r.value, torch.Tensor) else r.value
                w = next(it) if isinstance(r.weight, torch.Tensor) else r.weight
                out.append(WeightedAverage(_scalar(v), _scalar(w)))
            else:
                out.append(Average(_scalar(next(it) if isinstance(r.value, torch.Tensor) else r.value)))
        return out
    return [WeightedAverage(_scalar(r.value), _scalar(r.weight)) if isinstance(r, WeightedAverage)
            else Average(_scalar(r.value)) for r in values]


def aggregate(values) -> float:
    """reporter.py:44-85."""
    for v in values:
        if not isinstance(v, type(values[0])):
            raise ValueError(f"Can't use different Reported type together: {type(v)} != {type(values[0])}")
    if len(values) == 0:
        warnings.warn("No stats found")
        return np.nan
    if not isinstance(values[0], (Average, WeightedAverage)):
        raise NotImplementedError(f"type={type(values[0])}")
    values = _resolve(values)
    if isinstance(values[0], Average):
        return np.nanmean([v.value for v in values])
    values = [v for v in values if np.isfinite(v.value) and np.isfinite(v.weight)]
    if len(values) == 0:
        warnings.warn("No valid stats found")
        return np.nan
    sum_weights = sum(v.weight for v in values)
    sum_value = sum(v.value * v.weight for v in values)
    if sum_weights == 0:
        warnings.warn("weight is zero")
        return np.nan
    return sum_value / sum_weights


class SubReporter:
    """reporter.py:113-285 (register / next / finished)."""

    def __init__(self, key: str, epoch: int, total_count: int):
        self.key = key
        self.epoch = epoch
        self.start_time = time.perf_counter()
        self.stats = defaultdict(list)
        self._finished = False
        self.total_count = total_count
        self.count = 0
        self._seen_keys_in_the_step = set()

    def get_total_count(self) -> int:
        return self.total_count

    def get_epoch(self) -> int:
        return self.epoch

    def next(self):
        for key, stats_list in self.stats.items():
            if key not in self._seen_keys_in_the_step:
                if isinstance(stats_list[0], WeightedAverage):
                    stats_list.append(to_reported_value(np.nan, 0))
                else:
                    stats_list.append(to_reported_value(np.nan))
            assert len(stats_list) == self.count, (len(stats_list), self.count)
        self._seen_keys_in_the_step = set()

    def register(self, stats: Dict[str, Optional[Num]], weight: Num = None) -> None:
        if self._finished:
            raise RuntimeError("Already finished")
        if len(self._seen_keys_in_the_step) == 0:
            self.total_count += 1
            self.count += 1
        for key2, v in stats.items():
            if key2 in _reserved:
                raise RuntimeError(f"{key2} is reserved.")
            if key2 in self._seen_keys_in_the_step:
                raise RuntimeError(f"{key2} is registered twice.")
            if v is None:
                v = np.nan
            r = to_reported_value(v, weight)
            if key2 not in self.stats:
                nan = to_reported_value(np.nan, None if weight is None else 0)
                self.stats[key2].extend(r if i == self.count - 1 else nan for i in range(self.count))
            else:
                self.stats[key2].append(r)
            self._seen_keys_in_the_step.add(key2)

    def log_message(self, start: int = None, end: int = None) -> str:
        if self._finished:
            raise RuntimeError("Already finished")
        start = 0 if start is None else (start + self.count if start < 0 else start)
        end = self.count if end is None else end
        if self.count == 0 or start == end:
            return ""
        parts = [f"{self.epoch}epoch:{self.key}:{start + 1}-{end}batch: "]
        for key2, stats_list in self.stats.items():
            vals = stats_list[start:end]
            if len(vals) == 0:
                continue
            v = aggregate(vals)
            parts.append(f"{key2}={v:.3e}, " if abs(v) > 1.0e3 else f"{key2}={v:.3f}, ")
        return "".join(parts).rstrip(", ")

    def finished(self) -> None:
        self._finished = True

    @contextmanager
    def measure_time(self, name: str):
        start = time.perf_counter()
        yield start
        self.register({name: time.perf_counter() - start})

    def measure_iter_time(self, iterable, name: str):
        iterator = iter(iterable)
        while True:
            try:
                start = time.perf_counter()
                retval = next(iterator)
                self.register({name: time.perf_counter() - start})
                yield retval
            except StopIteration:
                break


class Reporter:
    """reporter.py:286-580.  stats[epoch][key][key2] -> aggregated value."""

    def __init__(self, epoch: int = 0):
        if epoch < 0:
            raise ValueError(f"epoch must be 0 or more: {epoch}")
        self.epoch = epoch
        self.stats = {}

    def get_epoch(self) -> int:
        return self.epoch

    def set_epoch(self, epoch: int) -> None:
        if epoch < 0:
            raise ValueError(f"epoch must be 0 or more: {epoch}")
        self.epoch = epoch

    @contextmanager
    def observe(self, key: str, epoch: int = None):
        sub_reporter = self.start_epoch(key, epoch)
        yield sub_reporter
        self.finish_epoch(sub_reporter)

    def start_epoch(self, key: str, epoch: int = None) -> SubReporter:
        if epoch is not None:
            if epoch < 0:
                raise ValueError(f"epoch must be 0 or more: {epoch}")
            self.epoch = epoch
        if self.epoch - 1 not in self.stats or key not in self.stats[self.epoch - 1]:
            if self.epoch - 1 != 0:
                warnings.warn(f"The stats of the previous epoch={self.epoch - 1}doesn't exist.")
            total_count = 0
        else:
            total_count = self.stats[self.epoch - 1][key]["total_count"]
        sub_reporter = SubReporter(key, self.epoch, total_count)
        self.stats.pop(epoch, None)
        return sub_reporter

    def finish_epoch(self, sub_reporter: SubReporter) -> None:
        if self.epoch != sub_reporter.epoch:
            raise RuntimeError(f"Don't change epoch during observation: {self.epoch} != {sub_reporter.epoch}")
        stats = {key2: aggregate(values) for key2, values in sub_reporter.stats.items()}
        stats["time"] = datetime.timedelta(seconds=time.perf_counter() - sub_reporter.start_time)
        stats["total_count"] = sub_reporter.total_count
        if torch.cuda.is_initialized():
            stats["gpu_max_cached_mem_GB"] = torch.cuda.max_memory_reserved() / 2 ** 30
        self.stats.setdefault(self.epoch, {})[sub_reporter.key] = stats
        sub_reporter.finished()

    def sort_epochs_and_values(self, key: str, key2: str, mode: str) -> List[Tuple[int, float]]:
        if mode not in ("min", "max"):
            raise ValueError(f"mode must min or max: {mode}")
        if not self.has(key, key2):
            raise KeyError(f"{key}.{key2} is not found: {self.get_all_keys()}")
        values = [(e, self.stats[e][key][key2]) for e in self.stats]
        if mode == "min":
            return sorted(values, key=lambda x: x[1])
        return sorted(values, key=lambda x: -x[1])

    def sort_epochs(self, key: str, key2: str, mode: str) -> List[int]:
        return [e for e, v in self.sort_epochs_and_values(key, key2, mode)]

    def sort_values(self, key: str, key2: str, mode: str) -> List[float]:
        return [v for e, v in self.sort_epochs_and_values(key, key2, mode)]

    def get_best_epoch(self, key: str, key2: str, mode: str, nbest: int = 0) -> int:
        return self.sort_epochs(key, key2, mode)[nbest]

    def check_early_stopping(self, patience: int, key1: str, key2: str, mode: str, epoch: int = None,
                             logger=None) -> bool:
        """reporter.py:397-420."""
        if epoch is None:
            epoch = self.get_epoch()
        best_epoch = self.get_best_epoch(key1, key2, mode)
        if epoch - best_epoch > patience:
            if logger is None:
                import logging as logger
            logger.info(f"[Early stopping] {key1}.{key2} has not been improved "
                        f"{epoch - best_epoch} epochs continuously. The training was stopped at {epoch}epoch")
            return True
        return False

    def has(self, key: str, key2: str, epoch: int = None) -> bool:
        if epoch is None:
            epoch = self.get_epoch()
        return epoch in self.stats and key in self.stats[epoch] and key2 in self.stats[epoch][key]

    def log_message(self, epoch: int = None) -> str:
        """reporter.py:431-460 (timedelta printed with str() instead of humanfriendly)."""
        if epoch is None:
            epoch = self.get_epoch()
        message = ""
        for key, d in self.stats[epoch].items():
            _message = ""
            for key2, v in d.items():
                if v is not None:
                    if len(_message) != 0:
                        _message += ", "
                    if isinstance(v, float):
                        if abs(v) > 1.0e3:
                            _message += f"{key2}={v:.3e}"
                        elif abs(v) > 1.0e-3:
                            _message += f"{key2}={v:.3f}"
                        else:
                            _message += f"{key2}={v:.3e}"
                    else:
                        _message += f"{key2}={v}"
            if len(_message) != 0:
                message += f"{epoch}epoch results: " if len(message) == 0 else ", "
                message += f"[{key}] {_message}"
        return message

    def get_value(self, key: str, key2: str, epoch: int = None):
        if not self.has(key, key2):
            raise KeyError(f"{key}.{key2} is not found in stats: {self.get_all_keys()}")
        if epoch is None:
            epoch = self.get_epoch()
        return self.stats[epoch][key][key2]

    def get_keys(self, epoch: int = None) -> Tuple[str, ...]:
        if epoch is None:
            epoch = self.get_epoch()
        return tuple(self.stats[epoch])

    def get_keys2(self, key: str, epoch: int = None) -> Tuple[str, ...]:
        if epoch is None:
            epoch = self.get_epoch()
        d = self.stats[epoch][key]
        return tuple(k for k in d if k not in ("time", "total_count"))

    def get_all_keys(self, epoch: int = None) -> Tuple[Tuple[str, str], ...]:
        if epoch is None:
            epoch = self.get_epoch()
        return tuple((k, k2) for k in self.stats[epoch] for k2 in self.stats[epoch][k])

    def state_dict(self):
        return {"stats": self.stats, "epoch": self.epoch}

    def load_state_dict(self, state_dict: dict):
        self.epoch = state_dict["epoch"]
        self.stats = state_dict["stats"]
