"""Building blocks of the hot path with explicit forward and backward passes.

Each block mirrors a reference module (same submodule/parameter names, so state_dict keys
match) and exposes `fwd(...) -> (out, ctx)` / `bwd(ctx, dout) -> dinput`.  Gradients
are accumulated straight into the flat gradient views (flat.py).  Activations are
row-major [B*T, D] device tensors.  All arithmetic is in libespnet_mi355.so (kernels.py).

Reference: espnet/nets/pytorch_backend/{conformer,transformer}/*.py (cited per class).
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
from torch import nn

from . import kernels as K


def _mix64(x: int) -> int:
    x &= 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


class Seeds:
    """Per-forward stream of dropout seeds (stateless counter RNG keys)."""

    def __init__(self, base: int):
        self.base = base & 0xFFFFFFFFFFFFFFFF
        self.i = 0

    def next(self) -> int:
        self.i += 1
        return _mix64(self.base + 0x9E3779B97F4A7C15 * self.i)


class Ctx(dict):
    __getattr__ = dict.__getitem__
    __setattr__ = dict.__setitem__


def empty(*shape, like: torch.Tensor):
    return torch.empty(*shape, dtype=torch.float32, device=like.device)


# False: the bf16 mode casts an fp32 dz2 for the conv2 gradients (an A/B constant, r04o: +0.6 % with it)
_DZ2_DIRECT = True


def grad_buf(dout):
    """The buffer of a branch gradient that only the branch's weight- and input-gradient GEMMs read:
    kernels.Planes in the fp32 mode (the GEMMs then split nothing), else fp32 like dout."""
    return K.grad_planes_like(dout) or torch.empty_like(dout)


class Linear(nn.Module):
    """Parameter container with torch.nn.Linear's names/shapes/init (weight (out,in), bias)."""

    def __init__(self, idim: int, odim: int, bias: bool = True):
        super().__init__()
        ref = nn.Linear(idim, odim, bias=bias)
        self.weight = ref.weight
        if bias:
            self.bias = ref.bias
        else:
            self.register_parameter("bias", None)

    def fwd(self, x2d, out=None, **kw):
        if out is None:
            out = empty(x2d.shape[0], self.weight.shape[0], like=x2d)
        return K.linear_fwd(x2d, self.weight, self.bias, out, **kw)

    def bwd(self, dy, x2d, dx=None, accumulate=False, need_dx=True):
        K.linear_bwd_weight(dy, x2d, self.weight.grad, self.bias.grad if self.bias is not None else None)
        if not need_dx:
            return None
        if dx is None:
            dx = empty(dy.shape[0], self.weight.shape[1], like=dy)
            accumulate = False
        return K.linear_bwd_data(dy, self.weight, dx, accumulate=accumulate)


class LayerNorm(nn.Module):
    """espnet LayerNorm (torch.nn.LayerNorm(size, eps=1e-12)), layer_norm.py:12-38."""

    def __init__(self, size: int, eps: float = 1e-12):
        super().__init__()
        ref = nn.LayerNorm(size, eps=eps)
        self.weight = ref.weight
        self.bias = ref.bias
        self.eps = eps

    def fwd(self, x2d, gemm_only: bool = False):
        """gemm_only: y feeds only GEMMs (a projection and its weight gradient) -- written as
        kernels.Planes in the current compute mode (kernels.planes_mode), else fp32."""
        M, D = x2d.shape
        mean = empty(M, like=x2d)
        rstd = empty(M, like=x2d)
        n = K.planes_mode() if gemm_only and D % 4 == 0 else 0
        if n:
            y = K.Planes(M, D, x2d.device, n)
            K.layernorm_fwd_planes(x2d, self.weight, self.bias, y, mean, rstd, self.eps)
        elif gemm_only and D % 8 == 0 and K.wgrad_xplanes_ok():
            # fp32 y for the Linear's forward beside the weight planes, and y's split planes for its weight
            # gradient (B planes: no B split in that RC x RC GEMM's k-loop)
            y = empty(M, D, like=x2d)
            K.layernorm_fwd_dual(x2d, self.weight, self.bias, y, mean, rstd, self.eps)
        else:
            y = empty(M, D, like=x2d)
            K.layernorm_fwd(x2d, self.weight, self.bias, y, mean, rstd, self.eps)
        return y, Ctx(x=x2d, mean=mean, rstd=rstd)

    def bwd(self, ctx, dy, dx_acc):
        """dx_acc += LN'(dy)  (dx_acc is the residual-stream gradient buffer)."""
        K.layernorm_bwd(dy, ctx.x, self.weight, ctx.mean, ctx.rstd, dx_acc, self.weight.grad, self.bias.grad,
                        accumulate=True)

    def bwd_new(self, ctx, dy):
        dx = torch.empty_like(dy)
        K.layernorm_bwd(dy, ctx.x, self.weight, ctx.mean, ctx.rstd, dx, self.weight.grad, self.bias.grad,
                        accumulate=False)
        return dx


class PositionwiseFeedForward(nn.Module):
    """positionwise_feed_forward.py:12-32: w_2(dropout(act(w_1(x))))."""

    def __init__(self, idim: int, hidden: int, dropout_rate: float, act: int):
        super().__init__()
        self.w_1 = Linear(idim, hidden)
        self.w_2 = Linear(hidden, idim)
        self.p = dropout_rate
        self.act = act

    def fwd(self, x2d, resid, alpha, p_res, seeds: Seeds, training: bool):
        """returns resid + alpha * drop_res(w_2(drop(act(w_1 x))))  (new buffer)."""
        M = x2d.shape[0]
        H = self.w_1.weight.shape[0]
        # the w_1 epilogue stores h = drop(act(v)) and, instead of v, the local derivative
        # dh/dv = keep * scale * act'(v): the backward epilogue is then a single multiply
        dact = empty(M, H, like=x2d)
        # h feeds only w_2 (forward and weight gradient): written as planes by the w_1 epilogue
        npl = K.planes_mode() if H % 8 == 0 else 0
        h = K.Planes(M, H, x2d.device, npl) if npl else empty(M, H, like=x2d)
        p_in = self.p if training else 0.0
        s1, s2 = seeds.next(), seeds.next()
        self.w_1.fwd(x2d, h, act=self.act | K.ACT_AUX_DERIV, aux=dact, drop_p=p_in, seed=s1)
        out = empty(M, x2d.shape[1], like=x2d)
        pr = p_res if training else 0.0
        self.w_2.fwd(h, out, alpha=alpha, drop_p=pr, seed=s2, R=resid, beta=1.0)
        return out, Ctx(x=x2d, dact=dact, h=h, s1=s1, s2=s2, p_in=p_in, pr=pr, alpha=alpha)

    def bwd(self, c, dout):
        """dout: grad w.r.t. the residual output; returns grad w.r.t. x2d (new buffer)."""
        dz = grad_buf(dout)
        K.scale_dropout(dout, dz, alpha=c.alpha, drop_p=c.pr, seed=c.s2)
        K.linear_bwd_weight(dz, c.h, self.w_2.weight.grad, self.w_2.bias.grad)
        # dh feeds only w_1's weight- and input-gradient GEMMs: planes from the multiply epilogue
        dh = grad_buf(c.dact)
        K.linear_bwd_data_act(dz, self.w_2.weight, dh, c.dact, K.ACT_MUL)
        return self.w_1.bwd(dh, c.x)


class RelPositionMultiHeadedAttention(nn.Module):
    """(Legacy)RelPositionMultiHeadedAttention, attention.py:117-308 (zero_triu=False).

    Scores are materialised per (head, utterance) in head-major order z = h*B + b."""

    def __init__(self, n_head: int, n_feat: int, dropout_rate: float, legacy: bool):
        super().__init__()
        assert n_feat % n_head == 0
        self.h, self.d_k = n_head, n_feat // n_head
        self.linear_q = Linear(n_feat, n_feat)
        self.linear_k = Linear(n_feat, n_feat)
        self.linear_v = Linear(n_feat, n_feat)
        self.linear_out = Linear(n_feat, n_feat)
        self.linear_pos = Linear(n_feat, n_feat, bias=False)
        self.pos_bias_u = nn.Parameter(torch.Tensor(self.h, self.d_k))
        self.pos_bias_v = nn.Parameter(torch.Tensor(self.h, self.d_k))
        nn.init.xavier_uniform_(self.pos_bias_u)
        nn.init.xavier_uniform_(self.pos_bias_v)
        self.p = dropout_rate
        self.legacy = legacy
        self.flat = None  # set by the model after flattening

    def _wqkv(self, grad=False):
        f = self.flat
        D = self.h * self.d_k
        w = f.fused([self.linear_q.weight, self.linear_k.weight, self.linear_v.weight], (3 * D, D), grad)
        b = f.fused([self.linear_q.bias, self.linear_k.bias, self.linear_v.bias], (3 * D,), grad)
        return w, b

    def fwd(self, x2d, resid, pos_emb, klen, B, T, p_res, seeds: Seeds, training: bool, tvalid=None):
        """tvalid (legacy only): the length-bucket T' (ConformerEncoder.run_forward); the legacy
        rel_shift is taken at T' inside esp_relpos_attn_probs / esp_attn_softmax_bwd_relpos."""
        H, dk = self.h, self.d_k
        D = H * dk
        M = B * T
        Z = H * B
        P = pos_emb.shape[0]
        relpos = 2 if self.legacy else 1
        w, b = self._wqkv()
        qkv = empty(M, 3 * D, like=x2d)
        K.linear_fwd(x2d, w, b, qkv)
        p = empty(P, D, like=x2d)
        K.linear_fwd(pos_emb, self.linear_pos.weight, None, p)
        q_u = empty(Z * T * dk, like=x2d)
        q_v = empty(Z * T * dk, like=x2d)
        K.heads_split2(qkv, 3 * D, 0, B, T, H, dk, self.pos_bias_u, q_u, self.pos_bias_v, q_v)
        pa = self.p if training else 0.0
        sa = seeds.next()
        tv = tvalid if self.legacy else None
        # a legacy length-bucketed batch (rel_shift at T' = *tvalid) takes the materialised kernels, which read
        # T' on device; the opt-in flash / score-gradient forms stay for every other batch
        if K.flash_ok(T, dk) and tv is None:
            # scores, softmax, dropout and P.V in one kernel: only ctx and 2 floats per row to HBM
            ctx_ = empty(M, D, like=x2d)
            stats = empty(Z * T * 2, like=x2d)
            K.relpos_flash_fwd(q_u, q_v, qkv, 3 * D, qkv, 3 * D, p, D, relpos, B, H, math.sqrt(dk), klen, ctx_, D,
                               stats, pa, sa, T, k_off=D, v_off=2 * D)
            out = empty(M, D, like=x2d)
            pr = p_res if training else 0.0
            so = seeds.next()
            self.linear_out.fwd(ctx_, out, drop_p=pr, seed=so, R=resid, beta=1.0)
            return out, Ctx(x=x2d, qkv=qkv, p=p, pos=pos_emb, q_u=q_u, q_v=q_v, ctx=ctx_, stats=stats, klen=klen,
                            flash=True, pa=pa, sa=sa, pr=pr, so=so, B=B, T=T, P=P)
        Tp, Pp = K.pitch(T), K.pitch(P)  # 16-B aligned score rows
        ac = empty(Z * T * Tp, like=x2d)
        pdrop = empty(Z * T * Tp, like=x2d) if pa > 0 else None
        if K.relpos_probs_ok(T, dk) and not K.ATTN_FWD32:
            # ac and the bd band on the MFMA inside the softmax kernel (latest and legacy
            # rel_shift): only attn and its dropout copy reach HBM
            K.relpos_attn_probs(q_u, q_v, qkv, 3 * D, p, D, relpos, B, H, math.sqrt(dk), klen, ac, pdrop, pa, sa, T,
                                Tp, k_off=D, tvalid=tv)
        elif not self.legacy and K.relpos_fused_ok(T, dk):
            K.relpos_attn_fwd(q_u, q_v, qkv, 3 * D, p, D, B, H, math.sqrt(dk), klen, ac, pdrop, pa, sa, T, Tp,
                              k_off=D)
        else:
            # ac[z] = q_u[z] k[b,h]^T
            K.gemm(T, T, dk, q_u, qkv, ac, mode_a=K.KC, lda=dk, mode_b=K.KC, ldb=3 * D, ldc=Tp, b_off=D,
                   batch=Z, nb2=B, sa=(B * T * dk, T * dk), sb=(dk, T * 3 * D), sc=(B * T * Tp, T * Tp))
            bd = empty(Z * T * Pp, like=x2d)
            K.gemm(T, P, dk, q_v, p, bd, mode_a=K.KC, lda=dk, mode_b=K.KC, ldb=D, ldc=Pp,
                   batch=Z, nb2=B, sa=(B * T * dk, T * dk), sb=(dk, 0), sc=(B * T * Pp, T * Pp))
            K.attn_softmax_fwd(ac, bd, relpos, P, math.sqrt(dk), klen, B, False, ac, pdrop, pa, sa, Z, T, T,
                               lds=Tp, ldp=Pp, tvalid=tv)
            del bd
        attn = ac
        pv = pdrop if pdrop is not None else attn
        # ctx feeds only linear_out (forward and weight gradient): planes from the P.V epilogue (the
        # score-gradient epilogue, ESP_ATTN_DSCORES, reads it in fp32)
        npl = K.planes_mode() if D % 8 == 0 and not K.ATTN_DSCORES else 0
        ctx_ = K.Planes(M, D, x2d.device, npl) if npl else empty(M, D, like=x2d)
        K.gemm(T, dk, T, pv, qkv, ctx_, mode_a=K.KC, lda=Tp, mode_b=K.RC, ldb=3 * D, ldc=D, b_off=2 * D,
               batch=Z, nb2=B, sa=(B * T * Tp, T * Tp), sb=(dk, T * 3 * D), sc=(dk, T * D))
        out = empty(M, D, like=x2d)
        pr = p_res if training else 0.0
        so = seeds.next()
        self.linear_out.fwd(ctx_, out, drop_p=pr, seed=so, R=resid, beta=1.0)
        return out, Ctx(x=x2d, qkv=qkv, p=p, pos=pos_emb, q_u=q_u, q_v=q_v, attn=attn, pv=pv, ctx=ctx_,
                        flash=False, pa=pa, sa=sa, pr=pr, so=so, B=B, T=T, P=P, tvalid=tv)

    def bwd(self, c, dout):
        H, dk = self.h, self.d_k
        D = H * dk
        B, T, P = c.B, c.T, c.P
        M, Z = B * T, H * B
        relpos = 2 if self.legacy else 1
        dz = grad_buf(dout)
        K.scale_dropout(dout, dz, drop_p=c.pr, seed=c.so)
        dctx = self.linear_out.bwd(dz, c.ctx)
        dqkv = empty(M, 3 * D, like=dout)
        if c.flash:
            return self._bwd_flash(c, dctx, dqkv)
        Tp, Pp = K.pitch(T), K.pitch(P)
        dS = empty(Z * T * Tp, like=dout)
        # the fused dP + softmax/rel_shift adjoint kernel measures slower than the K=64 GEMM + the
        # row-wise adjoint pass at C2 (198 vs 157 us per layer): opt-in until it is reworked
        fused = not self.legacy and K.relpos_fused_ok(T, dk) and K.FUSED_ATTN_BWD
        dscores = not fused and K.ATTN_DSCORES and c.tvalid is None  # (legacy + length bucket: the row-wise pass)
        # latest rel_shift, row-wise adjoint: dbd in the kept zeroed buffer, only its band written
        band = None if (self.legacy or fused or dscores or Tp % 4 or T > 1024) else K.relpos_band_buffer(Z, T, Pp, dout.device)
        dbd = band if band is not None else empty(Z * T * Pp, like=dout)
        if dscores:
            # dS = P (drop'(dP) - dot) / sqrt(dk) and its rel_shift adjoint in the dP GEMM's epilogue,
            # dot_i = dctx_i . ctx_i (= sum_j P_drop dP): no dP tensor, no row-wise pass
            dot = empty(Z * T, like=dout)
            K.attn_bwd_prep(dctx, D, c.ctx, D, B, H, dk, T, dot, dbd, Pp, relpos)
            K.attn_dscores(dctx, D, c.qkv, 3 * D, c.attn, dot, dS, dbd, Pp, relpos, B, H, dk, math.sqrt(dk), c.pa,
                           c.sa, T, Tp, v_off=2 * D)
        elif fused:  # dP = dctx v^T on the MFMA inside the softmax / rel_shift adjoint kernel
            K.relpos_attn_bwd(dctx, D, c.qkv, 3 * D, c.attn, dS, dbd, Pp, B, H, math.sqrt(dk), c.pa, c.sa, T, Tp,
                              v_off=2 * D)
        else:  # dP = dctx v^T  (into a (Z,T,T) buffer)
            K.gemm(T, T, dk, dctx, c.qkv, dS, mode_a=K.KC, lda=D, mode_b=K.KC, ldb=3 * D, ldc=Tp, b_off=2 * D,
                   batch=Z, nb2=B, sa=(dk, T * D), sb=(dk, T * 3 * D), sc=(B * T * Tp, T * Tp))
        # dV = pv^T dctx -> dqkv[:, 2D:3D]
        K.gemm(T, dk, T, c.pv, dctx, dqkv, mode_a=K.RC, lda=Tp, mode_b=K.RC, ldb=D, ldc=3 * D, c_off=2 * D,
               batch=Z, nb2=B, sa=(B * T * Tp, T * Tp), sb=(dk, T * D), sc=(dk, T * 3 * D))
        if fused or dscores:
            pass
        elif band is not None:
            K.attn_softmax_bwd_relpos_band(c.attn, dS, dS, dbd, Pp, c.pa, c.sa, math.sqrt(dk), Z * T, T, Tp)
        else:  # softmax + rel_shift adjoints in one pass (latest and legacy)
            K.attn_softmax_bwd_relpos(c.attn, dS, dS, dbd, Pp, c.pa, c.sa, math.sqrt(dk), Z * T, T, Tp, relpos=relpos,
                                      tvalid=c.tvalid)
        # dq_u = dS k -> dqkv[:, 0:D]
        K.gemm(T, dk, T, dS, c.qkv, dqkv, mode_a=K.KC, lda=Tp, mode_b=K.RC, ldb=3 * D, ldc=3 * D, b_off=D,
               batch=Z, nb2=B, sa=(B * T * Tp, T * Tp), sb=(dk, T * 3 * D), sc=(dk, T * 3 * D))
        # dk = dS^T q_u -> dqkv[:, D:2D]
        K.gemm(T, dk, T, dS, c.q_u, dqkv, mode_a=K.RC, lda=Tp, mode_b=K.RC, ldb=dk, ldc=3 * D, c_off=D,
               batch=Z, nb2=B, sa=(B * T * Tp, T * Tp), sb=(B * T * dk, T * dk), sc=(dk, T * 3 * D))
        K.colsum(dqkv, self.pos_bias_u.grad.view(-1), accumulate=True, M=M, N=D, ld=3 * D)
        # dq_v = dbd p -> tmp
        tmp = empty(M, D, like=dout)
        if not self.legacy and dk == 64:  # the band of each row tile only (dbd is 0 outside it)
            K.relpos_dqv(dbd, Pp, c.p, D, tmp, D, B, H, T)
        else:
            K.gemm(T, dk, P, dbd, c.p, tmp, mode_a=K.KC, lda=Pp, mode_b=K.RC, ldb=D, ldc=D,
                   batch=Z, nb2=B, sa=(B * T * Pp, T * Pp), sb=(dk, 0), sc=(dk, T * D))
        K.colsum(tmp, self.pos_bias_v.grad.view(-1), accumulate=True)
        K.add2d(tmp, D, dqkv, 3 * D, M, D)
        # dp[:, h] = sum_b dbd[h,b]^T q_v[h,b]   (K = B*T)
        dp = empty(P, D, like=dout)
        K.gemm(P, dk, B * T, dbd, c.q_v, dp, mode_a=K.RC, lda=Pp, mode_b=K.RC, ldb=dk, ldc=D,
               batch=H, nb2=1, sa=(B * T * Pp, 0), sb=(B * T * dk, 0), sc=(dk, 0))
        # linear_pos weight grad only (pos_emb is a constant table)
        K.gemm(D, D, P, dp, c.pos, self.linear_pos.weight.grad, mode_a=K.RC, lda=D, mode_b=K.RC, ldb=D, ldc=D,
               R=self.linear_pos.weight.grad, beta=1.0)
        w, _ = self._wqkv()
        gw, gb = self._wqkv(grad=True)
        K.linear_bwd_weight(dqkv, c.x, gw, gb)
        dx = empty(M, D, like=dout)
        K.linear_bwd_data(dqkv, w, dx)
        return dx


    def _bwd_flash(self, c, dctx, dqkv):
        """Flash backward: scores recomputed per (z, 32 rows); dq (q_u and q_v paths) and the
        pos_bias partials in-kernel; dK / dV as batched GEMMs over the dS / P_drop it writes;
        linear_pos gradient from dS along its diagonals (no dbd tensor)."""
        H, dk = self.h, self.d_k
        D = H * dk
        B, T, P = c.B, c.T, c.P
        M, Z = B * T, H * B
        rel = 2 if self.legacy else 1
        Tp = K.pitch(T)
        nqb = (T + 31) // 32
        dS = empty(Z * T * Tp, like=dctx)
        pd = empty(Z * T * Tp, like=dctx)
        bias_part = empty(Z * nqb * 2 * dk, like=dctx)
        carry = empty(Z * nqb * dk, like=dctx) if rel == 2 else None
        K.relpos_flash_bwd(c.q_u, c.q_v, c.qkv, 3 * D, c.qkv, 3 * D, c.p, D, rel, B, H, math.sqrt(dk), c.klen, c.ctx,
                           dctx, D, c.stats, c.pa, c.sa, T, dqkv, 3 * D, dS, pd, Tp, bias_part, carry,
                           k_off=D, v_off=2 * D)
        # dV = P_drop^T dctx -> dqkv[:, 2D:3D];  dK = dS^T q_u -> dqkv[:, D:2D]
        K.gemm(T, dk, T, pd, dctx, dqkv, mode_a=K.RC, lda=Tp, mode_b=K.RC, ldb=D, ldc=3 * D, c_off=2 * D,
               batch=Z, nb2=B, sa=(B * T * Tp, T * Tp), sb=(dk, T * D), sc=(dk, T * 3 * D))
        K.gemm(T, dk, T, dS, c.q_u, dqkv, mode_a=K.RC, lda=Tp, mode_b=K.RC, ldb=dk, ldc=3 * D, c_off=D,
               batch=Z, nb2=B, sa=(B * T * Tp, T * Tp), sb=(B * T * dk, T * dk), sc=(dk, T * 3 * D))
        dp = empty(P, D, like=dctx)
        K.relpos_dp(dS, Tp, c.q_v, rel, B, H, T, dp, D, bias_part, carry, self.pos_bias_u.grad.view(-1),
                    self.pos_bias_v.grad.view(-1), dqkv, 3 * D)
        del dS, pd
        K.gemm(D, D, P, dp, c.pos, self.linear_pos.weight.grad, mode_a=K.RC, lda=D, mode_b=K.RC, ldb=D, ldc=D,
               R=self.linear_pos.weight.grad, beta=1.0)
        w, _ = self._wqkv()
        gw, gb = self._wqkv(grad=True)
        K.linear_bwd_weight(dqkv, c.x, gw, gb)
        dx = empty(M, D, like=dctx)
        K.linear_bwd_data(dqkv, w, dx)
        return dx


class MultiHeadedAttention(nn.Module):
    """attention.py:16-114 (self- or source-attention), head-major z = h*B + b."""

    def __init__(self, n_head: int, n_feat: int, dropout_rate: float):
        super().__init__()
        self.h, self.d_k = n_head, n_feat // n_head
        self.linear_q = Linear(n_feat, n_feat)
        self.linear_k = Linear(n_feat, n_feat)
        self.linear_v = Linear(n_feat, n_feat)
        self.linear_out = Linear(n_feat, n_feat)
        self.p = dropout_rate
        self.flat = None

    def _w(self, names, grad=False):
        f = self.flat
        D = self.h * self.d_k
        mods = [getattr(self, n) for n in names]
        w = f.fused([m.weight for m in mods], (len(mods) * D, D), grad)
        b = f.fused([m.bias for m in mods], (len(mods) * D,), grad)
        return w, b

    def fwd(self, xq, resid, B, Tq, klen, causal, p_res, seeds: Seeds, training: bool, mem=None, Tk=None):
        """self-attention when mem is None (q,k,v from xq), else source attention over mem."""
        H, dk = self.h, self.d_k
        D = H * dk
        Z = H * B
        if mem is None:
            Tk = Tq
            w, b = self._w(("linear_q", "linear_k", "linear_v"))
            qkv = empty(B * Tq, 3 * D, like=xq)
            K.linear_fwd(xq, w, b, qkv)
            qb, qld, qoff = qkv, 3 * D, 0
            kvb, kvld, koff, voff = qkv, 3 * D, D, 2 * D
            kv = None
        else:
            qkv = empty(B * Tq, D, like=xq)
            self.linear_q.fwd(xq, qkv)
            w, b = self._w(("linear_k", "linear_v"))
            kv = empty(B * Tk, 2 * D, like=xq)
            K.linear_fwd(mem, w, b, kv)
            qb, qld, qoff = qkv, D, 0
            kvb, kvld, koff, voff = kv, 2 * D, 0, D
        Tkp = K.pitch(Tk)
        sc = empty(Z * Tq * Tkp, like=xq)
        K.gemm(Tq, Tk, dk, qb, kvb, sc, mode_a=K.KC, lda=qld, mode_b=K.KC, ldb=kvld, ldc=Tkp, a_off=qoff, b_off=koff,
               batch=Z, nb2=B, sa=(dk, Tq * qld), sb=(dk, Tk * kvld), sc=(B * Tq * Tkp, Tq * Tkp))
        pa = self.p if training else 0.0
        sa = seeds.next()
        pdrop = empty(Z * Tq * Tkp, like=xq) if pa > 0 else None
        K.attn_softmax_fwd(sc, None, 0, 0, math.sqrt(dk), klen, B, causal, sc, pdrop, pa, sa, Z, Tq, Tk, lds=Tkp)
        pv = pdrop if pdrop is not None else sc
        npl = K.planes_mode() if D % 8 == 0 else 0
        ctx_ = K.Planes(B * Tq, D, xq.device, npl) if npl else empty(B * Tq, D, like=xq)
        K.gemm(Tq, dk, Tk, pv, kvb, ctx_, mode_a=K.KC, lda=Tkp, mode_b=K.RC, ldb=kvld, ldc=D, b_off=voff,
               batch=Z, nb2=B, sa=(B * Tq * Tkp, Tq * Tkp), sb=(dk, Tk * kvld), sc=(dk, Tq * D))
        out = empty(B * Tq, D, like=xq)
        pr = p_res if training else 0.0
        so = seeds.next()
        self.linear_out.fwd(ctx_, out, drop_p=pr, seed=so, R=resid, beta=1.0)
        return out, Ctx(xq=xq, mem=mem, qkv=qkv, kv=kv, attn=sc, pv=pv, ctx=ctx_, pa=pa, sa=sa, pr=pr, so=so,
                        B=B, Tq=Tq, Tk=Tk)

    def bwd(self, c, dout, dmem=None):
        """returns dxq (new); accumulates the memory gradient into dmem for source attention."""
        H, dk = self.h, self.d_k
        D = H * dk
        B, Tq, Tk = c.B, c.Tq, c.Tk
        Z = H * B
        dz = grad_buf(dout)
        K.scale_dropout(dout, dz, drop_p=c.pr, seed=c.so)
        dctx = self.linear_out.bwd(dz, c.ctx)
        if c.mem is None:
            dq_buf = empty(B * Tq, 3 * D, like=dout)
            dqld, dqoff = 3 * D, 0
            dkv, dkvld, dkoff, dvoff = dq_buf, 3 * D, D, 2 * D
            kvb, kvld, koff, voff = c.qkv, 3 * D, D, 2 * D
            qb, qld, qoff = c.qkv, 3 * D, 0
        else:
            dq_buf = empty(B * Tq, D, like=dout)
            dqld, dqoff = D, 0
            dkv = empty(B * Tk, 2 * D, like=dout)
            dkvld, dkoff, dvoff = 2 * D, 0, D
            kvb, kvld, koff, voff = c.kv, 2 * D, 0, D
            qb, qld, qoff = c.qkv, D, 0
        Tkp = K.pitch(Tk)
        dS = empty(Z * Tq * Tkp, like=dout)
        K.gemm(Tq, Tk, dk, dctx, kvb, dS, mode_a=K.KC, lda=D, mode_b=K.KC, ldb=kvld, ldc=Tkp, b_off=voff,
               batch=Z, nb2=B, sa=(dk, Tq * D), sb=(dk, Tk * kvld), sc=(B * Tq * Tkp, Tq * Tkp))
        K.gemm(Tk, dk, Tq, c.pv, dctx, dkv, mode_a=K.RC, lda=Tkp, mode_b=K.RC, ldb=D, ldc=dkvld, c_off=dvoff,
               batch=Z, nb2=B, sa=(B * Tq * Tkp, Tq * Tkp), sb=(dk, Tq * D), sc=(dk, Tk * dkvld))
        K.attn_softmax_bwd(c.attn, dS, dS, c.pa, c.sa, math.sqrt(dk), Z * Tq, Tk, lds=Tkp)
        K.gemm(Tq, dk, Tk, dS, kvb, dq_buf, mode_a=K.KC, lda=Tkp, mode_b=K.RC, ldb=kvld, ldc=dqld, b_off=koff,
               c_off=dqoff, batch=Z, nb2=B, sa=(B * Tq * Tkp, Tq * Tkp), sb=(dk, Tk * kvld), sc=(dk, Tq * dqld))
        K.gemm(Tk, dk, Tq, dS, qb, dkv, mode_a=K.RC, lda=Tkp, mode_b=K.RC, ldb=qld, ldc=dkvld, a_off=0, b_off=qoff,
               c_off=dkoff, batch=Z, nb2=B, sa=(B * Tq * Tkp, Tq * Tkp), sb=(dk, Tq * qld), sc=(dk, Tk * dkvld))
        if c.mem is None:
            w, _ = self._w(("linear_q", "linear_k", "linear_v"))
            gw, gb = self._w(("linear_q", "linear_k", "linear_v"), grad=True)
            K.linear_bwd_weight(dq_buf, c.xq, gw, gb)
            dx = empty(B * Tq, D, like=dout)
            K.linear_bwd_data(dq_buf, w, dx)
            return dx
        dx = self.linear_q.bwd(dq_buf, c.xq)
        w, _ = self._w(("linear_k", "linear_v"))
        gw, gb = self._w(("linear_k", "linear_v"), grad=True)
        K.linear_bwd_weight(dkv, c.mem, gw, gb)
        K.linear_bwd_data(dkv, w, dmem, accumulate=True)
        return dx


class ConvolutionModule(nn.Module):
    """conformer/convolution.py:13-79 (GLU, depthwise k, BatchNorm1d train stats, Swish)."""

    def __init__(self, channels: int, kernel_size: int):
        super().__init__()
        assert (kernel_size - 1) % 2 == 0
        self.pointwise_conv1 = nn.Conv1d(channels, 2 * channels, 1)
        self.depthwise_conv = nn.Conv1d(channels, channels, kernel_size, padding=(kernel_size - 1) // 2,
                                        groups=channels)
        self.norm = nn.BatchNorm1d(channels)
        self.pointwise_conv2 = nn.Conv1d(channels, channels, 1)
        self.kernel_size = kernel_size

    def fwd(self, x2d, resid, B, T, p_res, seeds: Seeds, training: bool, tvalid=None):
        """tvalid: see ConformerEncoder.run_forward (length-bucketed batch)."""
        M, D = x2d.shape
        w1 = self.pointwise_conv1.weight.view(2 * D, D)
        u = empty(M, 2 * D, like=x2d)
        K.linear_fwd(x2d, w1, self.pointwise_conv1.bias, u)
        g = empty(M, D, like=x2d)
        K.glu_fwd(u, g)
        y = empty(M, D, like=x2d)
        K.dwconv1d(g, self.depthwise_conv.weight, self.depthwise_conv.bias, y, B, T, D, self.kernel_size, tvalid=tvalid)
        mean = empty(D, like=x2d)
        rstd = empty(D, like=x2d)
        bn = self.norm
        # s feeds only pointwise_conv2 (forward and weight gradient): planes in training mode
        npl = K.planes_mode() if training and D % 8 == 0 else 0
        s = K.Planes(M, D, x2d.device, npl) if npl else empty(M, D, like=x2d)
        if training:
            K.bn_swish_fwd(y, bn.weight, bn.bias, s, mean, rstd, bn.running_mean, bn.running_var,
                           momentum=bn.momentum, eps=bn.eps, T=T, tvalid=tvalid)
            bn.num_batches_tracked.add_(1)
        else:  # inference: running statistics (no backward is taken in eval mode)
            K.bn_swish_eval(y, bn.weight, bn.bias, s, bn.running_mean, bn.running_var, mean, rstd, eps=bn.eps)
        out = empty(M, D, like=x2d)
        pr = p_res if training else 0.0
        so = seeds.next()
        K.linear_fwd(s, self.pointwise_conv2.weight.view(D, D), self.pointwise_conv2.bias, out, drop_p=pr, seed=so,
                     R=resid, beta=1.0)
        return out, Ctx(x=x2d, u=u, g=g, y=y, s=s, mean=mean, rstd=rstd, pr=pr, so=so, B=B, T=T, tvalid=tvalid)

    def bwd(self, c, dout):
        M, D = dout.shape
        dz = grad_buf(dout)
        K.scale_dropout(dout, dz, drop_p=c.pr, seed=c.so)
        w2 = self.pointwise_conv2.weight
        K.linear_bwd_weight(dz, c.s, w2.grad.view(D, D), self.pointwise_conv2.bias.grad)
        ds = empty(M, D, like=dout)
        K.linear_bwd_data(dz, w2.view(D, D), ds)
        dy = empty(M, D, like=dout)
        sums = empty(2 * D, like=dout)
        bn = self.norm
        K.bn_swish_bwd(ds, c.y, c.mean, c.rstd, bn.weight, bn.bias, dy, bn.weight.grad, bn.bias.grad, sums,
                       T=c.T, tvalid=c.tvalid)
        dw = self.depthwise_conv
        K.colsum(dy, dw.bias.grad, accumulate=True)  # rows beyond tvalid hold 0
        K.dwconv1d_wgrad(dy, c.g, dw.weight.grad, c.B, c.T, D, self.kernel_size, tvalid=c.tvalid)
        dg = ds  # reuse
        K.dwconv1d(dy, dw.weight, None, dg, c.B, c.T, D, self.kernel_size, flip=True, tvalid=c.tvalid)
        # du feeds only pointwise_conv1's weight- and input-gradient GEMMs
        npl = K.planes_mode() if D % 4 == 0 else 0
        du = K.Planes(M, 2 * D, dout.device, npl) if npl else empty(M, 2 * D, like=dout)
        K.glu_bwd(c.u, dg, du)
        w1 = self.pointwise_conv1.weight
        K.linear_bwd_weight(du, c.x, w1.grad.view(2 * D, D), self.pointwise_conv1.bias.grad)
        dx = empty(M, D, like=dout)
        K.linear_bwd_data(du, w1.view(2 * D, D), dx)
        return dx


class Conv2dSubsampling(nn.Module):
    """subsampling.py:42-87 in NHWC; returns x*sqrt(D) (+ dropout), before the rel-pos table."""

    input_layer = "conv2d"
    k2, s2 = 3, 2  # the second convolution's kernel / stride
    min_frames = 7  # check_short_utt (subsampling.py:31-39)

    def __init__(self, idim: int, odim: int):
        super().__init__()
        self.conv = nn.Sequential(nn.Conv2d(1, odim, 3, 2), nn.ReLU(), nn.Conv2d(odim, odim, self.k2, self.s2),
                                  nn.ReLU())
        self.f2 = self.out_frames(idim)
        self.out = nn.Sequential(Linear(odim * self.f2, odim))
        self.odim = odim

    @classmethod
    def out_frames(cls, T: int) -> int:
        """Output length of the two convolutions for T input frames (or bins)."""
        return ((T - 3) // 2 + 1 - cls.k2) // cls.s2 + 1

    def fwd(self, feats, xscale, p_drop, seeds: Seeds, training: bool):
        B, T, F = feats.shape
        D = self.odim
        T1, F1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
        T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
        c0, c2 = self.conv[0], self.conv[2]
        # the bf16 mode: conv1 also writes z1's bf16 copy, the conv2 GEMM's operand (z1 stays fp32 for the
        # weight gradient's gather and the ReLU mask)
        b16 = K.conv2_bf16_ok(D)
        z1 = empty(B * T1 * F1 * D, like=feats)
        z1_16 = torch.empty(B * T1 * F1 * D, dtype=torch.bfloat16, device=feats.device) if b16 else None
        # training: the ReLU mask also as a packed bit map, the input gradient's mask operand (1/32 of z1's bytes)
        z1bits = (torch.empty(B * T1 * F1 * D // 32, dtype=torch.int32, device=feats.device)
                  if training and K.CONV2_DGRAD_BITS and K.CONV2_IMPLICIT_DGRAD and D % 32 == 0 else None)
        K.conv1_fwd(feats, c0.weight, c0.bias, z1, B, T, F, D, z16=z1_16, zbits=z1bits)
        w2r = empty(D * 9 * D, like=feats)
        K.permute3(c2.weight, w2r, D, D, 9)
        z2 = empty(B * T2 * F2, D, like=feats)
        ic = (T1, F1, D, T2, F2)
        if b16:
            K.conv2_fwd_bf16(z1_16, K.to_bf16(w2r, D, 9 * D, 9 * D), c2.bias, z2, B, T1, F1, D)
            if training and (B * T2 * F2) % 2:  # (the bf16 weight gradient takes an even pixel count)
                z1_16 = None
        else:
            K.gemm(B * T2 * F2, D, 9 * D, z1, w2r, z2, mode_a=K.I2C_KC, lda=0, mode_b=K.KC, ldb=9 * D, ldc=D,
                   bias=c2.bias, act=K.ACT_RELU, ic_a=ic, b_weight=True)
        lin = self.out[0]
        wor = empty(D * F2 * D, like=feats)
        K.permute3(lin.weight, wor, D, D, F2)  # (n, c, f) -> (n, f, c)
        x = empty(B * T2, D, like=feats)
        pd = p_drop if training else 0.0
        sd = seeds.next()
        K.linear_fwd(z2.view(B * T2, F2 * D), wor.view(D, F2 * D), lin.bias, x, alpha=xscale, drop_p=pd, seed=sd,
                     b_weight=True)
        return x, Ctx(feats=feats, z1=z1, z1_16=z1_16 if training else None, z1bits=z1bits, w2r=w2r, z2=z2, wor=wor,
                      pd=pd, sd=sd, xscale=xscale, B=B, T=T, F=F, T1=T1, F1=F1, T2=T2, F2=F2)

    def bwd(self, c, dx):
        D = self.odim
        B, T2, F2, T1, F1 = c.B, c.T2, c.F2, c.T1, c.F1
        c0, c2 = self.conv[0], self.conv[2]
        lin = self.out[0]
        dv = torch.empty_like(dx)
        K.scale_dropout(dx, dv, alpha=c.xscale, drop_p=c.pd, seed=c.sd)
        dwor = torch.zeros(D * F2 * D, dtype=torch.float32, device=dx.device)
        z2f = c.z2.view(B * T2, F2 * D)
        K.linear_bwd_weight(dv, z2f, dwor.view(D, F2 * D), lin.bias.grad)
        K.permute3(dwor, lin.weight.grad, D, F2, D, accumulate=True)  # (n, f, c) -> (n, c, f)
        npix2 = B * T2 * F2
        # the bf16 mode: dz2's bf16 copy is the operand of the weight- and input-gradient GEMMs; when both
        # take it (even pixel count, implicit input gradient) the input-gradient GEMM of `out` writes it
        # directly (its bf16 result plane, EPI_RMASK_PL) and dz2 never exists in fp32
        direct16 = (K.conv2_bf16_ok(D) and c.z1_16 is not None and K.CONV2_IMPLICIT_DGRAD and D % 32 == 0
                    and K.planes_mode() == 1 and (F2 * D) % 8 == 0 and _DZ2_DIRECT)
        if direct16:
            dz2 = K.Planes(B * T2, F2 * D, dx.device, 1)
            K.linear_bwd_data_act(dv, c.wor.view(D, F2 * D), dz2, z2f, K.ACT_RELU, b_weight=True)
            dz2p, dz2_16 = None, dz2.buf.view(npix2, D)
        else:
            dz2 = empty(B * T2, F2 * D, like=dx)
            K.linear_bwd_data_act(dv, c.wor.view(D, F2 * D), dz2, z2f, K.ACT_RELU, b_weight=True)  # ReLU' from its output
            dz2p = dz2.view(npix2, D)
            dz2_16 = K.to_bf16(dz2p, npix2, D, D) if K.conv2_bf16_ok(D) else None
        ic = (T1, F1, D, T2, F2)
        dw2r = empty(D, 9 * D, like=dx)
        if dz2_16 is not None and c.z1_16 is not None:
            K.conv2_wgrad_bf16(dz2_16, c.z1_16, dw2r, c2.bias.grad, B, T1, F1, D)
        else:
            K.gemm(D, 9 * D, npix2, dz2p, c.z1, dw2r, mode_a=K.RC, lda=D, mode_b=K.I2C_RC, ldb=0, ldc=9 * D, ic_b=ic,
                   rowsum=c2.bias.grad)
        K.permute3(dw2r, c2.weight.grad, D, 9, D, accumulate=True)  # (o, kk, c) -> (o, c, kk)
        z1bits = c.get("z1bits")
        if z1bits is not None and K.conv2_c1fold_ok(D):
            # conv1's weight gradient in the input gradient's epilogue: the conv1-map gradient is never stored
            K.conv2_dgrad_c1fold(dz2p, c2.weight, z1bits, c.feats, c.T, c.F, c0.weight.grad.view(D, 9), c0.bias.grad,
                                 B, T1, F1, D, dz2_16=dz2_16)
            return
        dz1 = empty(B * T1 * F1 * D, like=dx)
        # 4 implicit parity-class GEMMs with the ReLU mask in the epilogue (no 9x column buffer,
        # 8.4 GB at C2 B=128): 10.2 ms against 12.4 ms for column GEMM + col2im (kernels.py)
        if K.CONV2_IMPLICIT_DGRAD and D % 32 == 0:
            K.conv2_dgrad(dz2p, c2.weight, c.z1, dz1, B, T1, F1, D, dz2_16=dz2_16, z1bits=z1bits)
            del dz2_16
        else:
            dcol = empty(npix2, 9 * D, like=dx)
            K.gemm(npix2, 9 * D, D, dz2p, c.w2r, dcol, mode_a=K.KC, lda=D, mode_b=K.RC, ldb=9 * D, ldc=9 * D,
                   b_weight=True)
            K.col2im_relu(dcol, c.z1, dz1, B, T1, F1, D)
            del dcol
        K.conv1_wgrad(c.feats, dz1, c0.weight.grad.view(D, 9), c0.bias.grad, B, c.T, c.F, D)


class Conv2dSubsampling6(Conv2dSubsampling):
    """input_layer "conv2d6" (subsampling.py:101-146): Conv2d(1, D, 3, 2) + ReLU, Conv2d(D, D, 5, 3) + ReLU,
    Linear(D * F2, D), F2 = ((idim - 1) // 2 - 2) // 3.  conv1 and the output Linear are the conv2d kernels;
    the 5 x 5 / stride 3 convolution runs on explicit NHWC columns (esp_im2col_nhwc: 25 D per output pixel,
    kept for the weight gradient) as one KC x KC GEMM with the bias + ReLU epilogue, its weight gradient an
    RC x RC GEMM with the fused bias gradient, its input gradient a KC x RC GEMM into columns and the
    ReLU-masked column adjoint (esp_col2im_relu_nhwc).  The LibriSpeech-960 Conformer recipe
    (egs2/librispeech/asr1/conf/tuning/train_asr_conformer.yaml) uses it; the SLURP recipe does not, so this
    is not the bench path."""

    input_layer = "conv2d6"
    k2, s2 = 5, 3
    min_frames = 11

    def fwd(self, feats, xscale, p_drop, seeds: Seeds, training: bool):
        B, T, F = feats.shape
        D = self.odim
        k, st = self.k2, self.s2
        T1, F1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
        T2, F2 = (T1 - k) // st + 1, (F1 - k) // st + 1
        c0, c2 = self.conv[0], self.conv[2]
        z1 = empty(B * T1 * F1 * D, like=feats)
        K.conv1_fwd(feats, c0.weight, c0.bias, z1, B, T, F, D)
        npix2, KK = B * T2 * F2, k * k * D
        col = empty(npix2, KK, like=feats)
        K.im2col_nhwc(z1, col, B, T1, F1, D, k, st)
        w2r = empty(D * k * k * D, like=feats)
        K.permute3(c2.weight, w2r, D, D, k * k)  # (o, c, kt, kf) -> (o, kt, kf, c)
        z2 = empty(npix2, D, like=feats)
        K.gemm(npix2, D, KK, col, w2r, z2, mode_a=K.KC, lda=KK, mode_b=K.KC, ldb=KK, ldc=D, bias=c2.bias,
               act=K.ACT_RELU, b_weight=True)
        lin = self.out[0]
        wor = empty(D * F2 * D, like=feats)
        K.permute3(lin.weight, wor, D, D, F2)  # (n, c, f) -> (n, f, c)
        x = empty(B * T2, D, like=feats)
        pd = p_drop if training else 0.0
        sd = seeds.next()
        K.linear_fwd(z2.view(B * T2, F2 * D), wor.view(D, F2 * D), lin.bias, x, alpha=xscale, drop_p=pd, seed=sd,
                     b_weight=True)
        return x, Ctx(feats=feats, z1=z1, col=col if training else None, w2r=w2r, z2=z2, wor=wor, pd=pd, sd=sd,
                      xscale=xscale, B=B, T=T, F=F, T1=T1, F1=F1, T2=T2, F2=F2)

    def bwd(self, c, dx):
        D = self.odim
        k, st = self.k2, self.s2
        B, T2, F2, T1, F1 = c.B, c.T2, c.F2, c.T1, c.F1
        c0, c2 = self.conv[0], self.conv[2]
        lin = self.out[0]
        dv = torch.empty_like(dx)
        K.scale_dropout(dx, dv, alpha=c.xscale, drop_p=c.pd, seed=c.sd)
        dwor = torch.zeros(D * F2 * D, dtype=torch.float32, device=dx.device)
        z2f = c.z2.view(B * T2, F2 * D)
        K.linear_bwd_weight(dv, z2f, dwor.view(D, F2 * D), lin.bias.grad)
        K.permute3(dwor, lin.weight.grad, D, F2, D, accumulate=True)  # (n, f, c) -> (n, c, f)
        npix2, KK = B * T2 * F2, k * k * D
        dz2 = empty(B * T2, F2 * D, like=dx)
        K.linear_bwd_data_act(dv, c.wor.view(D, F2 * D), dz2, z2f, K.ACT_RELU, b_weight=True)  # ReLU' from its output
        dz2p = dz2.view(npix2, D)
        dw2r = empty(D, KK, like=dx)
        K.gemm(D, KK, npix2, dz2p, c.col, dw2r, mode_a=K.RC, lda=D, mode_b=K.RC, ldb=KK, ldc=KK,
               rowsum=c2.bias.grad)
        K.permute3(dw2r, c2.weight.grad, D, k * k, D, accumulate=True)  # (o, kk, c) -> (o, c, kk)
        c.col = None
        dcol = empty(npix2, KK, like=dx)
        K.gemm(npix2, KK, D, dz2p, c.w2r, dcol, mode_a=K.KC, lda=D, mode_b=K.RC, ldb=KK, ldc=KK, b_weight=True)
        dz1 = empty(B * T1 * F1 * D, like=dx)
        K.col2im_relu_nhwc(dcol, c.z1, dz1, B, T1, F1, D, k, st)
        del dcol
        K.conv1_wgrad(c.feats, dz1, c0.weight.grad.view(D, 9), c0.bias.grad, B, c.T, c.F, D)


def make_subsampling(input_layer: str, idim: int, odim: int) -> Conv2dSubsampling:
    """The encoders' input_layer choice (conformer_encoder.py:173-222 / transformer_encoder.py:97-140)."""
    cls = {"conv2d": Conv2dSubsampling, "conv2d6": Conv2dSubsampling6}.get(input_layer)
    if cls is None:
        raise NotImplementedError(f"input_layer={input_layer}: conv2d and conv2d6 are built")
    return cls(idim, odim)
