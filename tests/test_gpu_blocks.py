"""Block-level parity (GPU vs the oracle restatement in fp64 with autograd): the relative-
position MHA (latest and legacy), the convolution module and the subsampling stack, each
forward + explicit backward, with padding masks."""
import math

import numpy as np
import pytest
import torch

from espnet_slurp_amd.blocks import ConvolutionModule, Conv2dSubsampling, RelPositionMultiHeadedAttention, Seeds
from espnet_slurp_amd.asr.encoder.abs_encoder import pos_table
from espnet_slurp_amd.flat import FlatParams
from oracle import espnet_cpu as O
from tests.helpers import rel_err

pytestmark = pytest.mark.gpu


def _check_grads(mod, P, prefix, tol=2e-5):
    """Per-tensor relative error; tensors whose exact gradient is 0 (softmax-invariant key
    bias, BN-fed conv bias) are compared against the block's gradient scale instead."""
    scale = max(float(P[prefix + "." + n].grad.abs().max()) for n, _ in mod.named_parameters())
    errs = {}
    for n, p in mod.named_parameters():
        ref = P[prefix + "." + n].grad
        if float(ref.abs().max()) < 1e-6 * scale:
            assert float(p.grad.abs().max()) < 1e-5 * scale, n
            continue
        errs[n] = rel_err(p.grad.cpu(), ref)
    print(sorted(errs.items(), key=lambda kv: kv[1])[-4:])
    bad = {n: e for n, e in errs.items() if e >= tol}
    assert not bad, bad


def _params64(mod, prefix):
    return {prefix + "." + k: v.detach().cpu().double().clone().requires_grad_(True) for k, v in mod.named_parameters()}


@pytest.mark.parametrize("legacy", [False, True])
def test_relpos_mha_block(dev, legacy):
    torch.manual_seed(0)
    B, T, D, H = 3, 29, 64, 4
    klen = torch.tensor([29, 23, 15])
    mod = RelPositionMultiHeadedAttention(H, D, 0.0, legacy).to(dev)
    with torch.no_grad():
        for p in mod.parameters():
            p.normal_(0, 0.2)
    flat = FlatParams(mod, dev)
    mod.flat = flat
    x = torch.randn(B * T, D)
    res = torch.randn(B * T, D)
    dout = torch.randn(B * T, D)
    pos = pos_table("legacy" if legacy else "latest", T, D, dev)
    out, c = mod.fwd(x.to(dev), res.to(dev), pos, klen.int().to(dev), B, T, 0.0, Seeds(1), True)
    dx = mod.bwd(c, dout.to(dev))
    P = _params64(mod, "a")
    xt = x.double().view(B, T, D).requires_grad_(True)
    mask = (~O.make_pad_mask(klen, T))[:, None, :]
    ref = O.rel_mha(P, "a", xt, pos.cpu().double()[None], mask, H, legacy) + res.double().view(B, T, D)
    ref.backward(dout.double().view(B, T, D))
    assert rel_err(out.cpu(), ref.detach().reshape(B * T, D)) < 1e-5
    assert rel_err(dx.cpu(), xt.grad.reshape(B * T, D)) < 1e-5
    _check_grads(mod, P, "a")


@pytest.mark.parametrize("fwd,legacy,bwd", [("wave16", False, "dscores"), ("wave16", True, "dscores"),
                                            ("wave16", False, "rowpass"), ("wave16", True, "rowpass"),
                                            ("wave16", False, "fused"), ("block32", False, "dscores"),
                                            ("block32", False, "fused")])
@pytest.mark.parametrize("T,klens", [(29, [29, 23, 15]), (77, [77, 40, 9]), (130, [130, 129, 64])])
def test_relpos_mha_fused_dk64(dev, T, klens, fwd, legacy, bwd, monkeypatch):
    """d_k = 64 rel-pos attention through the fused score kernels — the 16-row-wave kernel
    (esp_relpos_attn_probs, latest and legacy rel_shift) and the 32-row-block kernel
    (esp_relpos_attn_fwd, latest) — several row groups incl. a partial last one, and the three
    score-gradient paths (dscores: the softmax / rel_shift adjoints in the dP GEMM epilogue;
    rowpass: dP GEMM + row-wise adjoint pass; fused: esp_relpos_attn_bwd), against the fp64
    oracle."""
    from espnet_slurp_amd import kernels as K
    monkeypatch.setattr(K, "FUSED_ATTN_BWD", bwd == "fused")
    monkeypatch.setattr(K, "ATTN_DSCORES", bwd == "dscores")
    monkeypatch.setattr(K, "FLASH_ATTN", False)  # the materialised paths (flash: tests/test_gpu_flash.py)
    monkeypatch.setattr(K, "ATTN_FWD32", fwd == "block32")
    torch.manual_seed(3)
    B, D, H = 3, 256, 4
    assert K.relpos_fused_ok(T, D // H) and K.relpos_probs_ok(T, D // H)
    klen = torch.tensor(klens)
    mod = RelPositionMultiHeadedAttention(H, D, 0.0, legacy).to(dev)
    with torch.no_grad():
        for p in mod.parameters():
            p.normal_(0, 0.1)
    mod.flat = FlatParams(mod, dev)
    x = torch.randn(B * T, D)
    res = torch.randn(B * T, D)
    dout = torch.randn(B * T, D)
    pos = pos_table("legacy" if legacy else "latest", T, D, dev)
    out, c = mod.fwd(x.to(dev), res.to(dev), pos, klen.int().to(dev), B, T, 0.0, Seeds(1), True)
    dx = mod.bwd(c, dout.to(dev))
    P = _params64(mod, "a")
    xt = x.double().view(B, T, D).requires_grad_(True)
    mask = (~O.make_pad_mask(klen, T))[:, None, :]
    ref = O.rel_mha(P, "a", xt, pos.cpu().double()[None], mask, H, legacy) + res.double().view(B, T, D)
    ref.backward(dout.double().view(B, T, D))
    assert rel_err(out.cpu(), ref.detach().reshape(B * T, D)) < 1e-5
    assert rel_err(dx.cpu(), xt.grad.reshape(B * T, D)) < 1e-5
    _check_grads(mod, P, "a")


def _unfused(K, monkeypatch):
    monkeypatch.setattr(K, "relpos_fused_ok", lambda T, dk: False)
    monkeypatch.setattr(K, "relpos_probs_ok", lambda T, dk: False)


@pytest.mark.parametrize("fwd,legacy,T,bwd", [("block32", False, 100, "fused"), ("wave16", False, 100, "fused"),
                                              ("wave16", False, 100, "dscores"), ("wave16", True, 100, "dscores"),
                                              ("wave16", False, 374, "dscores"), ("wave16", True, 374, "dscores"),
                                              ("wave16", False, 374, "fused")])
def test_relpos_fused_matches_unfused_with_dropout(dev, monkeypatch, fwd, legacy, T, bwd):
    """Same seeds -> the fused kernels reproduce the unfused path's (ac GEMM, bd GEMM, rel_shift +
    softmax pass; dP GEMM + row-wise adjoint pass) attention probabilities and dropout masks (mask
    index row*T + j), the same block output and the same gradients; T = 374 is the C2/C4/C5
    subsampled length (score rows of pitch 376)."""
    from espnet_slurp_amd import kernels as K
    monkeypatch.setattr(K, "FLASH_ATTN", False)  # the materialised paths (flash: tests/test_gpu_flash.py)
    monkeypatch.setattr(K, "ATTN_FWD32", fwd == "block32")
    monkeypatch.setattr(K, "ATTN_DSCORES", bwd == "dscores")
    torch.manual_seed(4)
    B, D, H = 2, 256, 4
    klen = torch.tensor([T, (T * 3) // 5]).int().to(dev)
    mod = RelPositionMultiHeadedAttention(H, D, 0.1, legacy).to(dev)
    mod.flat = FlatParams(mod, dev)
    x = torch.randn(B * T, D, device=dev)
    res = torch.randn(B * T, D, device=dev)
    pos = pos_table("legacy" if legacy else "latest", T, D, dev)
    dout = torch.randn(B * T, D, device=dev)
    monkeypatch.setattr(K, "FUSED_ATTN_BWD", bwd == "fused")
    out_f, c_f = mod.fwd(x, res, pos, klen, B, T, 0.0, Seeds(7), True)
    dx_f = mod.bwd(c_f, dout)
    g_f = mod.flat.grad.clone()
    mod.flat.grad.zero_()
    _unfused(K, monkeypatch)
    monkeypatch.setattr(K, "FUSED_ATTN_BWD", False)
    monkeypatch.setattr(K, "ATTN_DSCORES", False)
    out_u, c_u = mod.fwd(x, res, pos, klen, B, T, 0.0, Seeds(7), True)
    dx_u = mod.bwd(c_u, dout)
    Tp = K.pitch(T)
    rows = lambda t: t.view(-1, Tp)[:, :T]  # noqa: E731  (the pitch columns are never written)
    assert float((rows(c_f.attn) - rows(c_u.attn)).abs().max()) < 1e-6
    assert bool(((rows(c_f.pv) == 0) == (rows(c_u.pv) == 0)).all())
    assert float((out_f - out_u).abs().max()) < 1e-4
    # backward: the fused dP / dropout / softmax / rel_shift adjoint kernel regenerates the same masks
    assert rel_err(dx_f.cpu(), dx_u.cpu()) < 1e-5
    assert rel_err(g_f.cpu(), mod.flat.grad.cpu()) < 1e-5


def test_conv_module_block(dev):
    torch.manual_seed(1)
    B, T, D = 3, 29, 64
    mod = ConvolutionModule(D, 31).to(dev)
    with torch.no_grad():
        for p in mod.parameters():
            p.normal_(0, 0.2)
    flat = FlatParams(mod, dev)
    x = torch.randn(B * T, D)
    res = torch.randn(B * T, D)
    dout = torch.randn(B * T, D)
    out, c = mod.fwd(x.to(dev), res.to(dev), B, T, 0.0, Seeds(2), True)
    dx = mod.bwd(c, dout.to(dev))
    P = _params64(mod, "m")
    P["m.norm.running_mean"] = torch.zeros(D, dtype=torch.double)
    P["m.norm.running_var"] = torch.ones(D, dtype=torch.double)
    xt = x.double().view(B, T, D).requires_grad_(True)
    ref = O.conv_module(P, "m", xt, 31) + res.double().view(B, T, D)
    ref.backward(dout.double().view(B, T, D))
    assert rel_err(out.cpu(), ref.detach().reshape(B * T, D)) < 1e-5
    assert rel_err(dx.cpu(), xt.grad.reshape(B * T, D)) < 1e-5
    _check_grads(mod, P, "m")


@pytest.mark.parametrize("implicit", [False, True])
@pytest.mark.parametrize("T,F,D", [(64, 80, 32), (65, 81, 64)])  # odd / even conv1 grid (parity classes)
def test_subsampling_block(dev, T, F, D, implicit, monkeypatch):
    from espnet_slurp_amd import kernels as K
    monkeypatch.setattr(K, "CONV2_IMPLICIT_DGRAD", implicit)
    torch.manual_seed(2)
    B = 2
    mod = Conv2dSubsampling(F, D).to(dev)
    with torch.no_grad():
        for p in mod.parameters():
            p.normal_(0, 0.1)
    flat = FlatParams(mod, dev)
    x = torch.randn(B, T, F)
    out, c = mod.fwd(x.to(dev), math.sqrt(D), 0.0, Seeds(3), True)
    T2 = c.T2
    dout = torch.randn(B * T2, D)
    mod.bwd(c, dout.to(dev))
    P = _params64(mod, "e")
    y, _ = O.conv2d_subsampling(P, "e", x.double(), torch.ones(B, 1, T, dtype=torch.bool))
    y = y * math.sqrt(D)
    y.backward(dout.double().reshape(B, T2, D))
    assert rel_err(out.cpu(), y.detach().reshape(B * T2, D)) < 1e-5
    _check_grads(mod, P, "e")


@pytest.mark.parametrize("T", [29, 77, 130, 256, 300, 374, 384])
@pytest.mark.parametrize("legacy", [False, True])
@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_probs_lds_slot_schedule(dev, T, legacy, mode):
    """relpos_probs_lds_kernel's LDS slot schedule (attention.hip, the audit above the kernel): every NTA
    instantiation (8 / 16 / 24 key tiles), latest and legacy, the fp32 (six products) and bf16 forms, ragged
    key lengths, dropout on.  In the slot-check build (ESP_LIB_VARIANT=_slotchk: per-wave generation words
    checked before and after every fragment read) no read may overlap a write of its slot; in every build
    the probabilities are finite and each row with keys sums to 1."""
    from espnet_slurp_amd import _native
    from espnet_slurp_amd import kernels as K
    lib = _native.load()
    lib.esp_attn_slot_check_errors()  # reset
    B, H, dk = 3, 4, 64
    D, Z = H * dk, 3 * H
    P = T if legacy else 2 * T - 1
    g = torch.Generator().manual_seed(T)
    qkv = (torch.randn(B * T, 3 * D, generator=g) * 0.5).to(dev)
    p = (torch.randn(P, D, generator=g) * 0.5).to(dev)
    q_u = (torch.randn(Z * T * dk, generator=g) * 0.5).to(dev)
    q_v = (torch.randn(Z * T * dk, generator=g) * 0.5).to(dev)
    klen = torch.tensor([T, max(1, T - 7), max(1, T // 3)], dtype=torch.int32, device=dev)
    Tp = K.pitch(T)
    ac = torch.empty(Z * T * Tp, device=dev)
    pdrop = torch.empty(Z * T * Tp, device=dev)
    with K.gemm_compute(mode):
        K.relpos_attn_probs(q_u, q_v, qkv, 3 * D, p, D, 2 if legacy else 1, B, H, math.sqrt(dk), klen, ac, pdrop,
                            0.1, 1234, T, Tp, k_off=D)
    torch.cuda.synchronize()
    n = lib.esp_attn_slot_check_errors()
    assert n in (-1, 0), f"{n} LDS slot-schedule violations"
    a = ac.view(Z, T, Tp)[:, :, :T]
    assert torch.isfinite(a).all()
    assert torch.allclose(a.sum(-1), torch.ones(Z, T, device=dev), atol=1e-5)
