"""initialize(model, init) — espnet2/torch_utils/initialize.py:12-139 for this model's modules.

`--init` (ASRTask.build_model, asr.py:556-557): "chainer" (LeCun-normal weights, zero
biases, N(0, 1) embeddings) or a torch.nn.init scheme for every >1-D parameter followed by
zero biases and the default re-initialisation of Embedding / LayerNorm modules.  Runs in
place on the parameters (before or after flattening: the flat buffer holds views)."""
from __future__ import annotations

import math

import torch

from ..blocks import LayerNorm


def _reset_default(m):
    if isinstance(m, torch.nn.Embedding):
        torch.nn.init.normal_(m.weight)
        if m.padding_idx is not None:
            with torch.no_grad():
                m.weight[m.padding_idx].fill_(0)
    elif isinstance(m, (LayerNorm, torch.nn.LayerNorm, torch.nn.GroupNorm)):
        with torch.no_grad():
            m.weight.fill_(1.0)
            m.bias.zero_()


def initialize(model: torch.nn.Module, init: str):
    if init == "chainer":
        for name, p in model.named_parameters():
            data = p.data
            if ".bias" in name and data.dim() == 1:
                data.zero_()
            elif data.dim() in (1, 2):
                data.normal_(0, 1.0 / math.sqrt(data.size(-1)))
            elif data.dim() in (3, 4):
                n = data.size(1)
                for k in data.size()[2:]:
                    n *= k
                data.normal_(0, 1.0 / math.sqrt(n))
            else:
                raise NotImplementedError
        for m in model.modules():
            if isinstance(m, torch.nn.Embedding):
                m.weight.data.normal_(0, 1)
            if hasattr(m, "espnet_initialization_fn"):
                m.espnet_initialization_fn()
        return
    schemes = {
        "xavier_uniform": torch.nn.init.xavier_uniform_,
        "xavier_normal": torch.nn.init.xavier_normal_,
        "kaiming_uniform": lambda t: torch.nn.init.kaiming_uniform_(t, nonlinearity="relu"),
        "kaiming_normal": lambda t: torch.nn.init.kaiming_normal_(t, nonlinearity="relu"),
    }
    for p in model.parameters():
        if p.dim() > 1:
            if init not in schemes:
                raise ValueError("Unknown initialization: " + init)
            schemes[init](p.data)
    for name, p in model.named_parameters():
        if ".bias" in name and p.dim() == 1:
            p.data.zero_()
    for m in model.modules():
        _reset_default(m)
        if hasattr(m, "espnet_initialization_fn"):
            m.espnet_initialization_fn()
