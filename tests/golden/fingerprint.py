"""Whole-tensor gradient fingerprints for the full-size fixtures (test infrastructure only).

The full-size gates compare every parameter gradient with the fp64 reference through its L2 norm and
16 fixed elements (make_golden.slice_indices).  A localised error inside a large tensor -- one 128 x 128
tile of a 262k-element weight gradient, one column counted twice -- can keep the norm and miss the
slice.  So each fixture also stores, per tensor (VERDICT r5 'next' 1c):

  fp_<tag>/<n>   the 8 fp64 projections of the flattened gradient onto fixed +-1 vectors (`signs`);
  rn_f64/<n>     for tensors of rank >= 2, the fp64 L2 norm of every row of g.view(shape[0], -1)
                 (rn_eref/<n>: the reference fp32 run's max row error relative to the largest row).

The +-1 vectors are a counter hash of (crc32(name), projection, element), so the generator (CPU) and the
GPU test make the same vectors in torch on their own device without storing them.  Gate: the error
relative to the fp64 norm (projections) or to the largest fp64 row norm (rows) within max(1e-4, 2 e_ref),
the rule of every other full-size gate (tests/helpers.grad_gate).  A block of n of the N elements off by
a relative eps moves a projection by ~eps sqrt(n / N) of the norm: a 1/16 tile with eps = 4e-4 fails it.
"""
import zlib

import torch

N_PROJ = 8
_M32 = 0xFFFFFFFF


def signs(name: str, numel: int, device="cpu") -> torch.Tensor:
    """[N_PROJ, numel] float64 of +-1: bit 0 of a 32-bit mix of (crc32(name), j, element index).  Every
    product is masked to 32 bits, so the int64 arithmetic is exact (or wraps identically) on any device."""
    seed = zlib.crc32(name.encode())
    e = torch.arange(numel, dtype=torch.int64, device=device)
    out = torch.empty(N_PROJ, numel, dtype=torch.float64, device=device)
    for j in range(N_PROJ):
        x = (e * 0x9E3779B1 + ((seed ^ (j * 0x7F4A7C15)) & _M32)) & _M32
        x = x ^ (x >> 16)
        x = (x * 0x85EBCA6B) & _M32
        x = x ^ (x >> 13)
        x = (x * 0xC2B2AE35) & _M32
        x = x ^ (x >> 16)
        out[j] = 1.0 - 2.0 * (x & 1).to(torch.float64)
    return out


def projections(name: str, g: torch.Tensor) -> torch.Tensor:
    """The N_PROJ fp64 projections of g (any shape, any device) -> float64 [N_PROJ] on g's device."""
    gf = g.detach().reshape(-1).to(torch.float64)
    return signs(name, gf.numel(), gf.device) @ gf


def row_norms(g: torch.Tensor):
    """fp64 L2 norms of the rows of g.view(shape[0], -1) (None for a vector)."""
    if g.dim() < 2:
        return None
    return g.detach().reshape(g.shape[0], -1).to(torch.float64).norm(dim=1)


def summarize(name: str, g: torch.Tensor, tag: str, out: dict, rows: dict):
    """One run's (tag "f32" / "f64") fingerprint of one tensor: fp_<tag>/<name> into out, its row norms
    into rows (finish_rows turns the two runs' row norms into rn_f64 / rn_eref)."""
    out[f"fp_{tag}/{name}"] = projections(name, g).cpu().numpy()
    r = row_norms(g)
    if r is not None:
        rows[(tag, name)] = r.cpu()


def finish_rows(out: dict, rows: dict):
    import numpy as np
    for (tag, name), r64 in list(rows.items()):
        if tag != "f64":
            continue
        r32 = rows[("f32", name)]
        out[f"rn_f64/{name}"] = r64.numpy()
        out[f"rn_eref/{name}"] = np.float64(float((r32 - r64).abs().max()) / max(float(r64.max()), 1e-300))
