"""Flat parameter / gradient storage.

All trainable parameters of a model live as views into ONE contiguous fp32 device buffer,
and their `.grad` tensors as views into ONE flat gradient buffer.  The kernels accumulate
gradients straight into those views, the fused Adam / clip-norm kernels sweep the flat
buffers in a single launch each, and the data-parallel all-reduce works on large
contiguous buckets of the flat gradient (train/distributed.py).  The parameter objects
themselves are the reference's (same names, shapes and state_dict keys).

Each slot starts at a multiple of 8 floats (32 B): float4 accesses stay aligned, and a slot's
element offset is a multiple of 8, so the per-step bf16 copy / bf16 split planes of the WHOLE flat
buffer (kernels.flat_cast: one launch per step) hold every weight's copy at a 16-B aligned address.
Attention projections are laid out q|k|v consecutively (weights, then biases) so that
the fused QKV (and decoder KV) GEMMs read one (3D, D) weight view.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch

from . import kernels as K
from torch import nn


def _align4(n: int) -> int:
    return (n + 3) // 4 * 4


def _align8(n: int) -> int:
    return (n + 7) // 8 * 8


def ordered_parameters(model: nn.Module) -> List[Tuple[str, nn.Parameter]]:
    """named_parameters() order, except that the q/k/v projections of every attention module
    are emitted as one group (q.w, k.w, v.w, q.b, k.b, v.b) at the position of the first."""
    groups = {}
    for _, mod in model.named_modules():
        if all(hasattr(mod, a) for a in ("linear_q", "linear_k", "linear_v")):
            g = [getattr(getattr(mod, a), attr) for attr in ("weight", "bias")
                 for a in ("linear_q", "linear_k", "linear_v")]
            for p in g:
                groups[id(p)] = g
    names = {id(p): n for n, p in model.named_parameters()}
    seen = set()
    out: List[Tuple[str, nn.Parameter]] = []
    for n, p in model.named_parameters():
        for q in groups.get(id(p), [p]):
            if id(q) not in seen:
                seen.add(id(q))
                out.append((names[id(q)], q))
    return out


class FlatParams:
    def __init__(self, model: nn.Module, device):
        self.params = ordered_parameters(model)
        self.slots: Dict[int, Tuple[int, int]] = {}
        off = 0
        for _, p in self.params:
            self.slots[id(p)] = (off, p.numel())
            off += _align8(p.numel())
        self.numel = off
        self.flat = torch.zeros(off, dtype=torch.float32, device=device)
        K.register_param_storage(self.flat)  # bf16 weight copies cached per training step (kernels)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        with torch.no_grad():
            for _, p in self.params:
                o, n = self.slots[id(p)]
                self.flat[o:o + n].copy_(p.detach().reshape(-1).to(device=device, dtype=torch.float32))
                p.data = self.flat[o:o + n].view(p.shape)
        # floating buffers (BatchNorm running statistics) as views into one more flat buffer:
        # DDP's per-forward buffer broadcast (X7) is then ONE collective with no packing
        self.buffers = [b for _, b in model.named_buffers() if b.dtype == torch.float32]
        self.other_buffers = [b for _, b in model.named_buffers() if b.is_floating_point() and b.dtype != torch.float32]
        nb = sum(_align4(b.numel()) for b in self.buffers)
        self.buf_flat = torch.zeros(max(nb, 4), dtype=torch.float32, device=device)
        off = 0
        with torch.no_grad():
            for b in self.buffers:
                n = b.numel()
                self.buf_flat[off:off + n].copy_(b.detach().reshape(-1).to(device=device, dtype=torch.float32))
                b.data = self.buf_flat[off:off + n].view(b.shape)
                off += _align4(n)
        self.link_grads(zero=True)

    def view(self, p: nn.Parameter) -> torch.Tensor:
        o, n = self.slots[id(p)]
        return self.flat[o:o + n].view(p.shape)

    def gview(self, p: nn.Parameter) -> torch.Tensor:
        o, n = self.slots[id(p)]
        return self.grad[o:o + n].view(p.shape)

    def span(self, plist) -> Tuple[int, int]:
        """(offset, numel) of consecutive params (checks adjacency)."""
        o0, n0 = self.slots[id(plist[0])]
        end = o0 + n0
        for p in plist[1:]:
            o, n = self.slots[id(p)]
            assert o == _align8(end) and _align8(end) == end, "parameters are not adjacent"
            end = o + n
        return o0, end - o0

    def fused(self, plist, shape, grad=False) -> torch.Tensor:
        o, n = self.span(plist)
        buf = self.grad if grad else self.flat
        return buf[o:o + n].view(shape)

    def link_grads(self, zero: bool = False):
        """Re-attach p.grad to the flat-gradient views (after zero_grad(set_to_none))."""
        any_none = any(p.grad is None for _, p in self.params)
        if zero or any_none:
            with torch.no_grad():
                if zero:
                    self.grad.zero_()
                else:
                    for _, p in self.params:
                        if p.grad is None:
                            self.gview(p).zero_()
        for _, p in self.params:
            g = self.gview(p)
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                if p.grad is not None:
                    with torch.no_grad():
                        g.copy_(p.grad)
                p.grad = g

    def ensure_grads(self):
        """Cheap per-step check: a caller's optimizer.zero_grad() (set_to_none=True, the torch
        default) leaves p.grad None; re-attach the flat views (zeroed) before the backward."""
        for _, p in self.params:
            if p.grad is None:
                self.link_grads()
                return

    def zero_grad(self):
        self.grad.zero_()
        self.link_grads()
