"""CTC — drop-in for espnet2/asr/ctc.py:6-127 (ctc_type="builtin").

ctc_lo Linear(D, V) on MFMA, row log-softmax, alpha/beta + gradient kernels that follow
PyTorch's CPU ctc_loss (reduction none, zero_infinity), sum / B.  The training path fuses the
loss gradient into the forward (HeadsFn in espnet_model.py); `forward` here is the
standalone module call (loss only).  argmax / forced_align provide the alignment outputs.
"""
from __future__ import annotations

import torch
from torch import nn

from .. import kernels as K
from ..blocks import Linear, empty


class CTC(nn.Module):
    def __init__(self, odim: int, encoder_output_size: int, dropout_rate: float = 0.0, ctc_type: str = "builtin",
                 reduce: bool = True, ignore_nan_grad: bool = None, zero_infinity: bool = True):
        super().__init__()
        if ctc_type != "builtin":
            raise NotImplementedError(f"ctc_type={ctc_type}: only the builtin CTC is on the hot path")
        if dropout_rate != 0.0:
            raise NotImplementedError("CTC dropout_rate != 0 (espnet2 default 0.0)")
        self.ctc_lo = Linear(encoder_output_size, odim)
        self.ctc_type = ctc_type
        self.reduce = reduce
        self.zero_infinity = zero_infinity if ignore_nan_grad is None else ignore_nan_grad
        self.dropout_rate = dropout_rate
        self.odim = odim

    # -------------------------------------------------------------- fused pieces
    def logits(self, hs2d):
        return self.ctc_lo.fwd(hs2d)

    def loss_and_grad(self, hs2d, B, T, hlens_i32, ys_pad, ys_lens_i32, Umax, gscale, want_grad=True):
        """returns (nll (B,), grad (B*T, V) or None, logits); grad = gscale * d(sum nll)/d logits."""
        V = self.odim
        logits = self.logits(hs2d)
        lp = empty(B * T, V, like=hs2d)
        K.log_softmax(logits, lp, B * T, V)
        nll = torch.empty(B, dtype=torch.float64, device=hs2d.device)  # fp64 per-utterance nll
        grad = empty(B * T, V, like=hs2d) if want_grad else None
        K.ctc_loss(lp, ys_pad, Umax, hlens_i32, ys_lens_i32, B, T, V, 0, gscale, self.zero_infinity, nll, grad)
        return nll, grad, lp

    def backward_from_logits(self, dlogits, hs2d, dhs):
        """ctc_lo backward: param grads accumulated, dhs written (not accumulated)."""
        self.ctc_lo.bwd(dlogits, hs2d, dx=dhs, accumulate=False)

    # -------------------------------------------------------------- module API
    def forward(self, hs_pad, hlens, ys_pad, ys_lens):
        B, T, D = hs_pad.shape
        ys = ys_pad.to(hs_pad.device).long().contiguous()
        with torch.no_grad():
            nll, _, _ = self.loss_and_grad(hs_pad.reshape(B * T, D).contiguous(), B, T,
                                           hlens.to(torch.int32).to(hs_pad.device), ys, ys_lens.to(torch.int32).to(hs_pad.device),
                                           ys.shape[1], 1.0, want_grad=False)
            if self.zero_infinity:
                nll = torch.where(torch.isinf(nll), torch.zeros_like(nll), nll)
        return (nll.sum() / B).float() if self.reduce else (nll / B).float()

    def log_softmax(self, hs_pad):
        B, T, D = hs_pad.shape
        with torch.no_grad():
            logits = self.logits(hs_pad.reshape(B * T, D).contiguous())
            lp = torch.empty_like(logits)
            K.log_softmax(logits, lp, B * T, self.odim)
        return lp.view(B, T, self.odim)

    def argmax(self, hs_pad):
        B, T, D = hs_pad.shape
        with torch.no_grad():
            logits = self.logits(hs_pad.reshape(B * T, D).contiguous())
            out = torch.empty(B * T, dtype=torch.int64, device=hs_pad.device)
            K.argmax(logits, out, B * T, self.odim)
        return out.view(B, T)

    def forced_align(self, h, y, blank_id=0):
        """espnet1 CTC.forced_align semantics (espnet/nets/pytorch_backend/ctc.py:185-249)."""
        lpz = self.log_softmax(h if h.dim() == 3 else h[None])[0].contiguous()
        return K.ctc_forced_align(lpz, y.to(lpz.device).long().contiguous(), blank_id)

    def forced_align_batch(self, hs_pad, hlens, ys_pad, ys_lens, blank_id=0):
        """forced_align of every utterance of a padded batch in one launch (each row as the per-utterance
        call on hs_pad[b, :hlens[b]] and ys_pad[b, :ys_lens[b]]); (B, T) int64, -1 past hlens[b]."""
        lpz = self.log_softmax(hs_pad)
        return K.ctc_forced_align_batch(lpz, hlens, ys_pad, ys_lens, blank_id)
