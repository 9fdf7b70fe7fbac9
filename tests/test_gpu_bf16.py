"""bf16-input MFMA GEMM path (esp_set_gemm_compute(1); TrainerOptions.use_amp).

Kernel level: with operands rounded to bf16 (round-to-nearest-even, as the kernel's LDS staging
does) every product is exact in fp32, so the kernel must match an fp64 GEMM of the ROUNDED
operands up to fp32 accumulation order: |err| <= 4e-6 * sqrt(K) * max|a||b| scale.  Against the
unrounded fp32 GEMM the error is the bf16 input rounding (relative 2^-8 per operand).
Model level: the reference offers only fp16 autocast here (trainer.py:181-195), so parity of the
bf16 step is statistical: the bf16 loss within 1 % of the fp32 loss of the same weights and
batch, and the gradient direction (cosine) within 1e-3 of the fp32 gradient.
"""
import math

import pytest
import torch

from espnet_slurp_amd import kernels as K
from oracle import espnet_cpu as O
from tests.helpers import build_model, load_seeded, small_cfg

pytestmark = pytest.mark.gpu


def _r(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g)


def _bf(x):
    return x.to(torch.bfloat16).double()


def _ref(A, B, ma, mb):
    a = _bf(A) if ma == K.KC else _bf(A).t()
    b = _bf(B).t() if mb == K.KC else _bf(B)
    return a @ b


@pytest.fixture
def bf16_mode():
    prev = K.set_gemm_compute("bf16")
    yield
    K.set_gemm_compute(prev)


@pytest.mark.parametrize("shape", [(1, 1, 1), (37, 53, 19), (128, 128, 32), (300, 260, 129), (1000, 96, 512),
                                   (130, 7, 3), (64, 33, 3000), (384, 256, 2048)])
@pytest.mark.parametrize("modes", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_bf16_gemm_modes(dev, bf16_mode, shape, modes):
    M, N, Kk = shape
    ma, mb = modes
    A = _r(M, Kk, seed=1) if ma == K.KC else _r(Kk, M, seed=1)
    B = _r(N, Kk, seed=2) if mb == K.KC else _r(Kk, N, seed=2)
    Ad, Bd = A.to(dev), B.to(dev)
    C = torch.empty(M, N, device=dev)
    K.gemm(M, N, Kk, Ad, Bd, C, mode_a=ma, lda=Ad.stride(0), mode_b=mb, ldb=Bd.stride(0), ldc=N)
    torch.cuda.synchronize()
    ref = _ref(A, B, ma, mb)
    err = (C.cpu().double() - ref).abs().max().item()
    assert err <= 4e-6 * max(1.0, math.sqrt(Kk)) * 4, err
    # and it is NOT the fp32 GEMM (the mode switch took effect)
    if Kk >= 19:
        a = A.double() if ma == K.KC else A.double().t()
        b = B.double().t() if mb == K.KC else B.double()
        assert (C.cpu().double() - a @ b).abs().max().item() > 1e-4


def test_bf16_gemm_epilogue_and_batched(dev, bf16_mode):
    M, N, Kk = 257, 132, 96
    X, W, b, R = _r(M, Kk, seed=3), _r(N, Kk, seed=4), _r(N, seed=5), _r(M, N, seed=6)
    out = torch.empty(M, N, device=dev)
    aux = torch.empty(M, N, device=dev)
    K.linear_fwd(X.to(dev), W.to(dev), b.to(dev), out, act=K.ACT_SWISH, aux=aux, alpha=0.5, R=R.to(dev), beta=1.0)
    pre = _bf(X) @ _bf(W).t() + b.double()
    ref = 0.5 * pre * torch.sigmoid(pre) + R.double()
    torch.cuda.synchronize()
    assert (aux.cpu().double() - pre).abs().max() < 1e-4
    assert (out.cpu().double() - ref).abs().max() < 1e-4
    # batched (z = z1*nb2 + z2) attention-style product: (H*B) x (T x dk) @ (T x dk)^T
    Z, T, dk = 6, 75, 64
    q, k = _r(Z, T, dk, seed=7), _r(Z, T, dk, seed=8)
    s = torch.empty(Z, T, T, device=dev)
    qd, kd = q.to(dev), k.to(dev)
    K.gemm(T, T, dk, qd, kd, s, mode_a=K.KC, lda=dk, mode_b=K.KC, ldb=dk, ldc=T, batch=Z, nb2=1,
           sa=(T * dk, 0), sb=(T * dk, 0), sc=(T * T, 0))
    torch.cuda.synchronize()
    ref = torch.bmm(_bf(q), _bf(k).transpose(1, 2))
    assert (s.cpu().double() - ref).abs().max() < 4e-6 * 8 * 4


def test_gemm_compute_setter(dev):
    prev = K.set_gemm_compute("fp32")
    assert K.get_gemm_compute() == 0
    with K.gemm_compute("bf16"):
        assert K.get_gemm_compute() == 1
    assert K.get_gemm_compute() == 0
    with pytest.raises(RuntimeError):
        K.set_gemm_compute(7)
    K.set_gemm_compute(prev)


def _loss_and_grad(dev, use_amp, wide=False):
    if wide:  # the C5 shape (SLURP-entity Conformer: d=512, H=8, FF 2048), two blocks
        cfg = O.ModelCfg(vocab_size=64, enc=O.EncCfg(output_size=512, attention_heads=8, linear_units=2048,
                                                     num_blocks=2, rel_pos_type="latest"),
                         dec=O.DecCfg(attention_heads=8, linear_units=2048, num_blocks=1), ctc_weight=0.3,
                         lsm_weight=0.1)
    else:
        cfg = small_cfg("latest", D=128, blocks=2, V=64)
    model = build_model(cfg, dev, dropout=0.0)
    load_seeded(model, cfg, 5)
    model.train()
    speech, slen, text, tlen = O.synthetic_batch(3, 160, 80, 64, [160, 140, 120], [9, 7, 5], 3)
    with K.gemm_compute("bf16" if use_amp else "fp32"):
        loss, stats, _ = model(speech=speech.to(dev), speech_lengths=slen, text=text, text_lengths=tlen)
        loss.backward()
    torch.cuda.synchronize()
    return loss.item(), model.flat.grad.detach().double().cpu().clone()


@pytest.mark.parametrize("wide", [False, True])
def test_bf16_model_step_close_to_fp32(dev, wide):
    l32, g32 = _loss_and_grad(dev, False, wide)
    l16, g16 = _loss_and_grad(dev, True, wide)
    assert abs(l16 - l32) <= 1e-2 * abs(l32), (l16, l32)
    cos = float((g16 @ g32) / (g16.norm() * g32.norm()))
    assert cos > 0.999, cos
    assert g16.norm() > 0 and torch.isfinite(g16).all()


def test_bf16_trainer_graph_matches_eager(dev):
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions

    def make(graph):
        cfg = small_cfg("latest")
        model = build_model(cfg, dev, dropout=0.0)
        load_seeded(model, cfg, 11)
        model.train()
        opt = FusedAdam(model.parameters(), model.flat, lr=1e-3)
        return Trainer(model, opt, None, TrainerOptions(grad_clip=5.0, use_amp=True), cuda_graph=graph), model

    te, me = make(False)
    tg, mg = make(True)
    for _ in range(3):
        speech, slen, text, tlen = O.synthetic_batch(3, 96, 80, 32, [96, 80, 71], [6, 5, 4], 12)
        b = dict(speech=speech.to(dev), speech_lengths=slen, text=text, text_lengths=tlen)
        le = te.train_one_step(dict(b, speech=b["speech"].clone(), text=b["text"].clone()))["loss"].item()
        lg = tg.train_one_step(dict(b, speech=b["speech"].clone(), text=b["text"].clone()))["loss"].item()
        assert abs(le - lg) <= 1e-6 * max(1.0, abs(le)), (le, lg)
    assert K.get_gemm_compute() == 0  # the trainer restores the process-wide setting
    torch.cuda.synchronize()
    assert torch.allclose(me.flat.flat, mg.flat.flat, rtol=0, atol=1e-6)


def test_bf16_loss_curve_statistical_gate(dev):
    """SURVEY §8(d) C5 gate (statistical, the reference's AMP path is fp16 autocast,
    trainer.py:181-195,554): 50 HIP-graph Trainer steps at the C5 layer shape (d=512, H=8,
    FF 2048; 2 encoder blocks, 1 decoder block) from the same init on the same 5 cycled batches,
    bf16 GEMM operands vs the fp32 path.  Gates: every step's loss within 3 % of the fp32 step's,
    the final losses within 2 %, and both curves descend (last-5 mean < 0.8 x first-5 mean)."""
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions

    cfg = O.ModelCfg(vocab_size=64, enc=O.EncCfg(output_size=512, attention_heads=8, linear_units=2048,
                                                 num_blocks=2, rel_pos_type="latest"),
                     dec=O.DecCfg(attention_heads=8, linear_units=2048, num_blocks=1), ctc_weight=0.3,
                     lsm_weight=0.1)
    batches = [O.synthetic_batch(4, 160, 80, 64, [160, 150, 130, 120], [9, 8, 7, 5], 100 + i) for i in range(5)]

    def curve(amp):
        model = build_model(cfg, dev, dropout=0.0)
        load_seeded(model, cfg, 7)
        model.train()
        opt = FusedAdam(model.parameters(), model.flat, lr=5e-4)
        tr = Trainer(model, opt, None, TrainerOptions(grad_clip=5.0, use_amp=amp), cuda_graph=True)
        out = []
        for step in range(50):
            speech, slen, text, tlen = batches[step % 5]
            st = tr.train_one_step(dict(speech=speech.to(dev), speech_lengths=slen, text=text.clone(),
                                        text_lengths=tlen))
            out.append(st["loss"].detach().clone())  # graph-mode stats are rewritten by the next replay
        return torch.stack([x.reshape(()) for x in out]).double().cpu()

    l32, l16 = curve(False), curve(True)
    assert torch.isfinite(l16).all() and torch.isfinite(l32).all()
    rel = ((l16 - l32).abs() / l32.abs()).max().item()
    assert rel <= 0.03, rel
    assert abs(l16[-1] - l32[-1]).item() <= 0.02 * abs(l32[-1]).item(), (l16[-1], l32[-1])
    for c in (l32, l16):
        assert c[-5:].mean() < 0.8 * c[:5].mean(), c


# ------------------------------------------------------------------ bf16-operand GEMM (PREC 2)
@pytest.mark.parametrize("M,N,Kd", [(304, 200, 136), (11968, 512, 512), (64, 64, 4096), (1000, 1024, 8),
                                    (256, 136, 520), (512, 64, 23936), (296, 72, 200)])
@pytest.mark.parametrize("modes", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_bf16_operand_gemm(dev, M, N, Kd, modes):
    """esp_gemm_bf16: bf16 operands in mode KC ([rows][K]) or RC ([K][rows], transposing LDS
    reads) with fp32 accumulate == fp64 GEMM of the same bf16 values up to accumulation order
    (ragged M / N edges, a K tail inside the last 64-wide slab, split-K for the small-M x N,
    long-K cases: the weight-gradient shape RC x RC).  An RC operand's row count is a multiple of 8
    (the ABI's contract); tile edges stay ragged (304, 296 rows)."""
    ma, mb = modes
    A, B = _r(M, Kd, seed=31), _r(N, Kd, seed=32)
    A16 = (A if ma == K.KC else A.t().contiguous()).to(torch.bfloat16).to(dev)
    B16 = (B if mb == K.KC else B.t().contiguous()).to(torch.bfloat16).to(dev)
    C = torch.full((M, N), float("nan"), device=dev)
    K.gemm_bf16(M, N, Kd, A16, B16, C, lda=Kd if ma == K.KC else M, ldb=Kd if mb == K.KC else N, ldc=N,
                mode_a=ma, mode_b=mb)
    a = A.to(torch.bfloat16).double()
    b = B.to(torch.bfloat16).double()
    ref = a @ b.t()
    err = (C.cpu().double() - ref).abs().max().item()
    assert err <= 4e-6 * math.sqrt(Kd) * max(1.0, A.abs().max().item() * B.abs().max().item()), err


def test_amp_linear_paths_use_bf16_operands(dev):
    """In the reduced-precision mode an nn.Linear forward / input gradient / weight gradient (with
    the fused bias gradient) runs on bf16 operands (cast + esp_gemm_bf16) and equals the fp64 result
    of the bf16-rounded operands; the fused bias gradient is the fp32 sum of the bf16-rounded dy (as
    torch AMP sums a bf16 grad_output)."""
    M, Din, Dout = 1000, 512, 256
    x, W, dy = _r(M, Din, seed=51), _r(Dout, Din, seed=52), _r(M, Dout, seed=53)
    xd, Wd, dyd = x.to(dev), W.to(dev), dy.to(dev)
    out, dx = torch.empty(M, Dout, device=dev), torch.empty(M, Din, device=dev)
    dW, db = torch.zeros(Dout, Din, device=dev), torch.zeros(Dout, device=dev)
    with K.gemm_compute("bf16"):
        K.linear_fwd(xd, Wd, None, out)
        K.linear_bwd_data(dyd, Wd, dx)
        K.linear_bwd_weight(dyd, xd, dW, db)
    torch.cuda.synchronize()
    xb, Wb, dyb = _bf(x), _bf(W), _bf(dy)
    for got, ref, k in ((out, xb @ Wb.t(), Din), (dx, dyb @ Wb, Dout), (dW, dyb.t() @ xb, M)):
        err = (got.cpu().double() - ref).abs().max().item()
        assert err <= 4e-6 * math.sqrt(k) * 16, err
    assert (db.cpu().double() - dyb.sum(0)).abs().max().item() <= 1e-5 * math.sqrt(M) * 4


def test_bf16_operand_gemm_epilogues(dev):
    """The fused epilogues on the bf16-operand kernel: bias + Swish + dropout with the derivative
    stored (FFN w_1), bias + dropout + residual (linear_out), plain + residual; each equals the
    fp32-operand kernel applied to the same (bf16-valued) operands."""
    M, N, Kd = 517, 256, 192
    A = _r(M, Kd, seed=41).to(torch.bfloat16).float().to(dev)
    B = _r(N, Kd, seed=42).to(torch.bfloat16).float().to(dev)
    A16, B16 = A.to(torch.bfloat16), B.to(torch.bfloat16)
    b, R = _r(N, seed=43).to(dev), _r(M, N, seed=44).to(dev)
    cases = [dict(bias=b, act=K.ACT_SWISH | K.ACT_AUX_DERIV, aux=True, drop_p=0.1, seed=5),
             dict(bias=b, R=R, beta=1.0, alpha=0.5, drop_p=0.1, seed=6),
             dict(R=R, beta=1.0)]
    for kw in cases:
        outs = []
        for bf in (False, True):
            C = torch.empty(M, N, device=dev)
            aux = torch.empty(M, N, device=dev) if kw.get("aux") else None
            args = {k: v for k, v in kw.items() if k != "aux"}
            if bf:
                K.gemm_bf16(M, N, Kd, A16, B16, C, lda=Kd, ldb=Kd, ldc=N, aux=aux, **args)
            else:
                K.gemm(M, N, Kd, A, B, C, lda=Kd, ldb=Kd, ldc=N, aux=aux, **args)
            outs.append((C, aux))
        (c0, a0), (c1, a1) = outs
        assert torch.equal(c0 == 0, c1 == 0)  # same dropout masks
        assert (c0 - c1).abs().max().item() <= 1e-4 * max(1.0, c0.abs().max().item())
        if a0 is not None:
            assert (a0 - a1).abs().max().item() <= 1e-4


@pytest.mark.parametrize("rows,cols", [(1000, 520), (37, 64), (4096, 2048)])
def test_f32_to_bf16_casts(dev, rows, cols):
    """esp_f32_to_bf16: round-to-nearest-even, plain and transposed, bit-equal to torch."""
    x = (_r(rows, cols, seed=51) * 100).to(dev)
    x[0, :4] = torch.tensor([float("inf"), -float("inf"), 0.0, -0.0])
    ref = x.to(torch.bfloat16)
    y = K.to_bf16(x, rows, cols, cols)
    assert torch.equal(y.view(torch.int16), ref.view(torch.int16))
    yt = K.to_bf16(x, rows, cols, cols, transpose=True)
    assert torch.equal(yt.view(torch.int16), ref.t().contiguous().view(torch.int16))
