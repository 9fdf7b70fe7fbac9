"""Checkpoint interop: the reference's checkpoint files, written and
read with the same layout so that checkpoints move both ways between the reference and this
framework.

  * `save_checkpoint` / `resume`     trainer.py:340-352 (checkpoint.pth = {"model", "reporter",
                                      "optimizers", "schedulers", "scaler"}) and
                                      Trainer.resume, trainer.py:124-151
  * `save_epoch`                      trainer.py:354-420: {iepoch}epoch.pth, latest.pth link,
                                      {phase}.{key}.best.pth links, n-best pruning
  * `average_nbest_models`            main_funcs/average_nbest_models.py:13-117
  * `load_pretrained_model`           torch_utils/load_pretrained_model.py:9-116
                                      (<file>:<src_key>:<dst_key>:<excludes>)

Formats: "model" is `model.state_dict()` (same keys as the reference's modules, per-tensor
storage — the flat parameter buffer is never written as such); "optimizers" holds
torch.optim.Adam state dicts (FusedAdam.state_dict converts from its flat moment buffers);
"schedulers" the torch _LRScheduler dict of WarmupLR; "reporter" Reporter.state_dict().

Loading never unpickles arbitrary objects: `safe_load` is torch.load(weights_only=True) with
the few non-tensor types a reference checkpoint holds (the reporter's datetime.timedelta and
numpy float64 statistics) allow-listed.
"""
from __future__ import annotations

import datetime
import logging
from pathlib import Path
from typing import Any, Collection, Dict, Optional, Sequence, Union

import numpy as np
import torch


def _safe_globals():
    g = [datetime.timedelta, np.dtype, np.float64, np.float32, np.int64]
    try:  # numpy >= 1.25: scalar reconstruction helper + per-dtype classes
        g.append(np._core.multiarray.scalar)  # type: ignore[attr-defined]
    except AttributeError:
        g.append(np.core.multiarray.scalar)
    for name in ("Float64DType", "Float32DType", "Int64DType"):
        if hasattr(np, "dtypes") and hasattr(np.dtypes, name):
            g.append(getattr(np.dtypes, name))
    return g


def safe_load(path: Union[str, Path], map_location="cpu") -> Any:
    """torch.load(..., weights_only=True) with the reporter's stat types allow-listed."""
    with torch.serialization.safe_globals(_safe_globals()):
        return torch.load(path, map_location=map_location, weights_only=True)


def _model_state(model: torch.nn.Module) -> Dict[str, torch.Tensor]:
    """state_dict with every tensor in its own storage (the parameters are views of the flat
    buffer: saved as such, every file would carry the whole buffer's storage)."""
    return {k: v.detach().clone() for k, v in model.state_dict().items()}


def save_checkpoint(path: Union[str, Path], model, reporter, optimizers: Sequence, schedulers: Sequence,
                    scaler=None, trainer=None) -> None:
    """trainer.py:340-352.  `trainer` (optional): its host counters are synchronised from the
    device first (HIP-graph mode keeps the Adam / scheduler step counts on device)."""
    if trainer is not None:
        trainer.resolve_pending()
        trainer.sync_host_state()
    torch.save({
        "model": _model_state(model),
        "reporter": reporter.state_dict(),
        "optimizers": [o.state_dict() for o in optimizers],
        "schedulers": [s.state_dict() if s is not None else None for s in schedulers],
        "scaler": scaler.state_dict() if scaler is not None else None,
    }, path)


def resume(checkpoint: Union[str, Path], model, reporter, optimizers: Sequence, schedulers: Sequence,
           scaler=None, ngpu: int = 0) -> None:
    """Trainer.resume (trainer.py:124-151): model, reporter, optimizers, schedulers, scaler
    from checkpoint.pth (the reference's or ours).  Device-side optimizer counters (graph mode)
    are refreshed from the loaded host state."""
    states = safe_load(checkpoint, map_location=f"cuda:{torch.cuda.current_device()}" if ngpu > 0 else "cpu")
    model.load_state_dict(states["model"])
    reporter.load_state_dict(states["reporter"])
    for optimizer, state in zip(optimizers, states["optimizers"]):
        optimizer.load_state_dict(state)
    for scheduler, state in zip(schedulers, states["schedulers"]):
        if scheduler is not None:
            scheduler.load_state_dict(state)
    for optimizer, scheduler in zip(optimizers, list(schedulers) + [None] * len(optimizers)):
        if hasattr(optimizer, "refresh_device_state"):
            optimizer.refresh_device_state(scheduler)
    if scaler is not None:
        if states["scaler"] is None:
            logging.warning("scaler state is not found")
        else:
            scaler.load_state_dict(states["scaler"])
    logging.info(f"The training was resumed using {checkpoint}")


def _relink(p: Path, target: str) -> None:
    if p.is_symlink() or p.exists():
        p.unlink()
    p.symlink_to(target)


def save_epoch(output_dir: Union[str, Path], iepoch: int, model, reporter,
               best_model_criterion: Sequence[Sequence[str]], keep_nbest_models: Union[int, Sequence[int]] = 10,
               nbest_averaging_interval: int = 0) -> list:
    """End-of-epoch model files, trainer.py:354-420: {iepoch}epoch.pth, latest.pth ->
    {iepoch}epoch.pth, {phase}.{key}.best.pth for every improved criterion, the n-best
    average every `nbest_averaging_interval` epochs, and removal of epoch files outside the
    union of the n-best sets.  Returns the improved criteria."""
    output_dir = Path(output_dir)
    keep = [keep_nbest_models] if isinstance(keep_nbest_models, int) else list(keep_nbest_models) or [1]
    torch.save(_model_state(model), output_dir / f"{iepoch}epoch.pth")
    _relink(output_dir / "latest.pth", f"{iepoch}epoch.pth")
    improved = []
    for phase, k, mode in best_model_criterion:
        if reporter.has(phase, k):
            if reporter.get_best_epoch(phase, k, mode) == iepoch:
                _relink(output_dir / f"{phase}.{k}.best.pth", f"{iepoch}epoch.pth")
                improved.append(f"{phase}.{k}")
    if len(improved) == 0:
        logging.info("There are no improvements in this epoch")
    else:
        logging.info("The best model has been updated: " + ", ".join(improved))
    nbests = set().union(*[set(reporter.sort_epochs(ph, k, m)[: max(keep)])
                           for ph, k, m in best_model_criterion if reporter.has(ph, k)])
    if nbest_averaging_interval > 0 and iepoch % nbest_averaging_interval == 0:
        average_nbest_models(output_dir=output_dir, reporter=reporter, best_model_criterion=best_model_criterion,
                             nbest=keep, suffix=f"till{iepoch}epoch")
    removed = []
    for e in range(1, iepoch):
        p = output_dir / f"{e}epoch.pth"
        if p.exists() and e not in nbests:
            p.unlink()
            removed.append(str(p))
    if removed:
        logging.info("The model files were removed: " + ", ".join(removed))
    return improved


@torch.no_grad()
def average_nbest_models(output_dir: Union[str, Path], reporter, best_model_criterion: Sequence[Sequence[str]],
                         nbest: Union[Collection[int], int], suffix: Optional[str] = None) -> None:
    """average_nbest_models.py:13-117: for every criterion, {ph}.{k}.ave_{n}best[.suffix].pth
    = mean of the n best epochs' model files (integer tensors such as BatchNorm's
    num_batches_tracked are summed, not averaged), ave_1best as a link to the best epoch file,
    and {ph}.{k}.ave[.suffix].pth linking the largest n."""
    output_dir = Path(output_dir)
    nbests = [nbest] if isinstance(nbest, int) else list(nbest)
    if len(nbests) == 0:
        logging.warning("At least 1 nbest values are required")
        nbests = [1]
    suffix = suffix + "." if suffix is not None else ""
    nbest_epochs = [(ph, k, reporter.sort_epochs_and_values(ph, k, m)[: max(nbests)])
                    for ph, k, m in best_model_criterion if reporter.has(ph, k)]
    loaded = {}
    for ph, cr, epoch_and_values in nbest_epochs:
        _nbests = [i for i in nbests if i <= len(epoch_and_values)] or [1]
        for n in _nbests:
            if n == 0:
                continue
            if n == 1:
                e, _ = epoch_and_values[0]
                _relink(output_dir / f"{ph}.{cr}.ave_1best.{suffix}pth", f"{e}epoch.pth")
                continue
            op = output_dir / f"{ph}.{cr}.ave_{n}best.{suffix}pth"
            logging.info(f'Averaging {n}best models: criterion="{ph}.{cr}": {op}')
            avg = None
            for e, _ in epoch_and_values[:n]:
                if e not in loaded:
                    loaded[e] = safe_load(output_dir / f"{e}epoch.pth", map_location="cpu")
                states = loaded[e]
                if avg is None:
                    avg = dict(states)
                else:
                    for k in avg:
                        avg[k] = avg[k] + states[k]
            for k in avg:
                if not str(avg[k].dtype).startswith("torch.int"):
                    avg[k] = avg[k] / n
            torch.save(avg, op)
        _relink(output_dir / f"{ph}.{cr}.ave.{suffix}pth", f"{ph}.{cr}.ave_{max(_nbests)}best.{suffix}pth")


def filter_state_dict(dst_state: Dict[str, torch.Tensor], src_state: Dict[str, torch.Tensor]) -> dict:
    """load_pretrained_model.py:9-36: keep the entries whose name and size match."""
    match = {}
    for key, value in src_state.items():
        if key in dst_state and dst_state[key].size() == src_state[key].size():
            match[key] = value
        elif key not in dst_state:
            logging.warning(f"Filter out {key} from pretrained dict because of name not found in target dict")
        else:
            logging.warning(f"Filter out {key} from pretrained dict because of size mismatch"
                            f"({dst_state[key].size()}-{src_state[key].size()})")
    return match


def load_pretrained_model(init_param: str, model: torch.nn.Module, ignore_init_mismatch: bool,
                          map_location: str = "cpu") -> None:
    """load_pretrained_model.py:39-116: init_param = <file>[:<src_key>[:<dst_key>[:<excludes>]]];
    src_key selects (and strips) a prefix of the file's keys, dst_key the target submodule,
    excludes a comma list of key prefixes to drop."""
    sps = init_param.split(":", 4)
    if len(sps) == 4:
        path, src_key, dst_key, excludes = sps
    elif len(sps) == 3:
        (path, src_key, dst_key), excludes = sps, None
    elif len(sps) == 2:
        (path, src_key), dst_key, excludes = sps, None, None
    else:
        (path,), src_key, dst_key, excludes = sps, None, None, None
    src_key = src_key or None
    dst_key = dst_key or None
    obj = model
    if dst_key is not None and dst_key.strip() != "":
        for k in dst_key.split("."):
            obj = getattr(obj, k)
    src_state = safe_load(path, map_location=map_location)
    if excludes is not None:
        for e in excludes.split(","):
            src_state = {k: v for k, v in src_state.items() if not k.startswith(e)}
    if src_key is not None:
        src_state = {k[len(src_key) + 1:]: v for k, v in src_state.items() if k.startswith(src_key)}
    dst_state = obj.state_dict()
    if ignore_init_mismatch:
        src_state = filter_state_dict(dst_state, src_state)
    dst_state.update(src_state)
    obj.load_state_dict(dst_state)
