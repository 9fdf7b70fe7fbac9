"""Fused Adam over the flat parameter buffer — the `adam` choice of espnet2
(abs_task.py:78-79 -> torch.optim.Adam) as one HIP kernel per step, applied after the
device-side clip_grad_norm_ (trainer.py:642-686).  Non-finite gradient norm => the kernel
skips the update (trainer.py:651-667) without a host round trip."""
from __future__ import annotations

import torch

from .. import kernels as K
from ..flat import FlatParams


def clip_grad_norm_(flat: FlatParams, max_norm: float, out: torch.Tensor = None) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ on the flat gradient, on device.  Returns a 3-vector
    (total L2 norm, clip coefficient min(1, max_norm/(norm+1e-6)), finite flag); the
    coefficient is applied inside the Adam kernel."""
    if out is None:
        out = torch.empty(3, dtype=torch.float32, device=flat.grad.device)
    K.grad_norm(flat.grad, max_norm, out)
    return out


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam over the flat parameter buffer.  One param group (the espnet2 default,
    abs_task.py:856-880 builds Adam(model.parameters(), **optim_conf)) is one launch over the whole
    buffer; several groups (each its own lr / betas / eps / weight_decay / amsgrad, as torch) are one
    launch per run of a group's parameters that lie next to each other in the flat buffer.
    amsgrad=True keeps max_exp_avg_sq in a third flat buffer."""

    def __init__(self, params, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad))
        self.flat = flat
        self.exp_avg = torch.zeros_like(flat.flat)
        self.exp_avg_sq = torch.zeros_like(flat.flat)
        self.max_exp_avg_sq = (torch.zeros_like(flat.flat) if any(g["amsgrad"] for g in self.param_groups)
                               else None)
        self.n_steps = 0
        self._ones = torch.tensor([1.0, 1.0, 1.0], device=flat.flat.device)
        self._ranges = self.group_ranges()

    def group_ranges(self):
        """Per param group, the (offset, length) runs of the flat buffer its launches cover: the whole
        buffer for a single group holding every flat parameter, else the group's parameters in flat
        order, merged while no parameter of another group lies between them (alignment padding inside
        a run holds zeros, which Adam leaves at zero)."""
        slots = self.flat.slots
        for g in self.param_groups:
            for p in g["params"]:
                if id(p) not in slots:
                    raise ValueError("FusedAdam: a parameter outside the flat buffer")
        if len(self.param_groups) == 1 and len(self.param_groups[0]["params"]) == len(slots):
            return [[(0, self.flat.flat.numel())]]
        owner = {id(p): gi for gi, g in enumerate(self.param_groups) for p in g["params"]}
        order = sorted(slots.items(), key=lambda kv: kv[1][0])  # every flat parameter, by offset
        out = [[] for _ in self.param_groups]
        prev = None  # (group, run start) of the run being extended
        for pid, (o, k) in order:
            gi = owner.get(pid)
            if gi is None:
                prev = None
                continue
            if prev is not None and prev[0] == gi:
                start = out[gi][-1][0]
                out[gi][-1] = (start, o + k - start)
            else:
                out[gi].append((o, k))
            prev = (gi, o)
        return out

    def _bufs(self, o, k):
        f = self.flat
        vm = self.max_exp_avg_sq[o:o + k] if self.max_exp_avg_sq is not None else None
        return f.flat[o:o + k], f.grad[o:o + k], self.exp_avg[o:o + k], self.exp_avg_sq[o:o + k], vm

    @torch.no_grad()
    def step(self, closure=None, clip: torch.Tensor = None):
        """clip: the 3-vector of clip_grad_norm_ (coefficient + finite flag); None = no clipping."""
        self.n_steps += 1
        c = clip if clip is not None else self._ones
        for g, runs in zip(self.param_groups, self._ranges):
            b1, b2 = g["betas"]
            for o, k in runs:
                p, gr, m, v, vm = self._bufs(o, k)
                if g["amsgrad"]:
                    K.adam_amsgrad(p, gr, m, v, vm, c, g["lr"], b1, b2, g["eps"], g["weight_decay"], self.n_steps)
                else:
                    K.adam(p, gr, m, v, c, g["lr"], b1, b2, g["eps"], g["weight_decay"], self.n_steps)
        return None

    # ---------------------------------------------------------- device-resident bookkeeping
    def device_state(self, scheduler=None) -> torch.Tensor:
        """{Adam steps applied, scheduler steps taken} as a device float64 pair, initialised from
        the host counters (graph mode keeps counting on device, esp_opt_advance)."""
        if getattr(self, "_dstate", None) is None:
            dev = self.flat.flat.device
            last = float(scheduler.last_epoch) if scheduler is not None else 0.0
            self._dstate = torch.tensor([float(self.n_steps), last], dtype=torch.float64, device=dev)
            self._hyper = torch.empty(3, dtype=torch.float32, device=dev)
            self._hyper_g = [self._hyper] + [torch.empty(3, dtype=torch.float32, device=dev)
                                             for _ in self.param_groups[1:]]
        return self._dstate

    def step_device(self, clip: torch.Tensor, scheduler=None):
        """Adam step whose lr / bias corrections come from the device state (WarmupLR formula
        on device): capturable in a HIP graph.  Counts the step (and the scheduler step) on
        device only when the gradient norm was finite."""
        st = self.device_state(scheduler)
        warmup = float(getattr(scheduler, "warmup_steps", 0.0) or 0.0)
        for gi, (g, runs) in enumerate(zip(self.param_groups, self._ranges)):
            b1, b2 = g["betas"]
            base = scheduler.base_lrs[gi] if scheduler is not None else g["lr"]
            hyper = self._hyper if gi == 0 else self._hyper_g[gi]
            K.opt_hyper(st, base, warmup, b1, b2, hyper)
            for o, k in runs:
                p, gr, m, v, vm = self._bufs(o, k)
                if g["amsgrad"]:
                    K.adam_dev_amsgrad(p, gr, m, v, vm, clip, hyper, b1, b2, g["eps"], g["weight_decay"])
                else:
                    K.adam_dev(p, gr, m, v, clip, hyper, b1, b2, g["eps"], g["weight_decay"])
        K.opt_advance(st, clip)

    def sync_from_device(self, scheduler=None):
        """Copy the device counters back to the host objects (after graph replays)."""
        if getattr(self, "_dstate", None) is None:
            return
        n, s = (int(x) for x in self._dstate.tolist())
        self.n_steps = n
        if scheduler is not None and s != scheduler.last_epoch:
            scheduler.last_epoch = s
            for grp, lr in zip(self.param_groups, scheduler.get_lr()):
                grp["lr"] = lr

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    # ---------------------------------------------------------- checkpoint interop
    @staticmethod
    def _adam_group(g) -> dict:
        """A param group as torch.optim.Adam would hold it (every Adam default key of this torch
        version, with the group's hyper-parameters)."""
        ref = torch.optim.Adam([torch.nn.Parameter(torch.zeros(1))], lr=g["lr"], betas=g["betas"], eps=g["eps"],
                               weight_decay=g["weight_decay"], amsgrad=g["amsgrad"])
        return dict(ref.param_groups[0])

    def state_dict(self):
        """torch.optim.Adam.state_dict() format — what the reference's checkpoint.pth holds under
        "optimizers" (trainer.py:340-352, abs_task.py:78-79): per parameter (keyed by its index,
        numbered across the param groups in order) {"step": float32 scalar, "exp_avg", "exp_avg_sq"
        (+ "max_exp_avg_sq" in an amsgrad group)} with the parameter's shape, copied out of the flat
        moment buffers.  Graph mode keeps the step count on device: it is read from there.  The
        groups' lr are the host values — call Trainer.sync_host_state() first (train_one_epoch does)."""
        n = int(self._dstate[0].item()) if getattr(self, "_dstate", None) is not None else self.n_steps
        state, groups, idx = {}, [], 0
        for g in self.param_groups:
            ids = []
            for p in g["params"]:
                if n > 0:
                    o, k = self.flat.slots[id(p)]
                    st = {"step": torch.tensor(float(n), dtype=torch.float32),
                          "exp_avg": self.exp_avg[o:o + k].view(p.shape).clone(),
                          "exp_avg_sq": self.exp_avg_sq[o:o + k].view(p.shape).clone()}
                    if g["amsgrad"]:
                        st["max_exp_avg_sq"] = self.max_exp_avg_sq[o:o + k].view(p.shape).clone()
                    state[idx] = st
                ids.append(idx)
                idx += 1
            group = self._adam_group(g)
            group["params"] = ids
            if "initial_lr" in g:  # added by the LR scheduler (torch _LRScheduler.__init__)
                group["initial_lr"] = g["initial_lr"]
            groups.append(group)
        return {"state": state, "param_groups": groups}

    @torch.no_grad()
    def load_state_dict(self, state_dict):
        """Load a torch.optim.Adam state_dict (the reference's checkpoint, or ours): the moments
        are copied into the flat buffers in place (a captured HIP graph keeps pointing at them),
        the step count into the host and device counters.  The groups must match this optimizer's
        in number and size (torch's rule); a group's amsgrad setting is taken from the checkpoint.
        FusedAdam keeps ONE step count: a checkpoint whose parameters have different Adam step
        counts is refused."""
        saved_groups = state_dict["param_groups"]
        if len(saved_groups) != len(self.param_groups) or any(
                len(sg["params"]) != len(g["params"]) for sg, g in zip(saved_groups, self.param_groups)):
            raise ValueError("loaded state dict has a different number of parameter groups / parameters")
        index = {}
        for sg, g in zip(saved_groups, self.param_groups):
            for key in ("lr", "betas", "eps", "weight_decay"):
                g[key] = tuple(sg[key]) if key == "betas" else sg[key]
            g["amsgrad"] = bool(sg.get("amsgrad", False))
            if "initial_lr" in sg:  # set by the LR scheduler at construction
                g["initial_lr"] = sg["initial_lr"]
            index.update(zip(sg["params"], g["params"]))
        if any(g["amsgrad"] for g in self.param_groups) and self.max_exp_avg_sq is None:
            self.max_exp_avg_sq = torch.zeros_like(self.flat.flat)
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        if self.max_exp_avg_sq is not None:
            self.max_exp_avg_sq.zero_()
        steps = set()
        for i, st in state_dict["state"].items():
            p = index[int(i)]
            o, k = self.flat.slots[id(p)]
            if st["exp_avg"].numel() != k:
                raise ValueError(f"state of parameter {i}: {tuple(st['exp_avg'].shape)} != {tuple(p.shape)}")
            self.exp_avg[o:o + k].copy_(st["exp_avg"].reshape(-1))
            self.exp_avg_sq[o:o + k].copy_(st["exp_avg_sq"].reshape(-1))
            if "max_exp_avg_sq" in st:
                self.max_exp_avg_sq[o:o + k].copy_(st["max_exp_avg_sq"].reshape(-1))
            steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError(f"parameters have different Adam step counts {sorted(steps)}")
        self.n_steps = steps.pop() if steps else 0
        if getattr(self, "_dstate", None) is not None:
            self._dstate[0].fill_(float(self.n_steps))

    def refresh_device_state(self, scheduler=None):
        """After loading optimizer / scheduler state: write the host counters into the device
        state in place (graph mode reads the lr schedule position from there)."""
        if getattr(self, "_dstate", None) is None:
            return
        last = float(scheduler.last_epoch) if scheduler is not None else 0.0
        self._dstate.copy_(torch.tensor([float(self.n_steps), last], dtype=torch.float64))
