"""CPU oracle for the CTC family: numpy restatements (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.

* `ctc_loss_np` restates PyTorch's CPU `ctc_loss` (ATen LossCTC.cpp, torch 2.10.0 — the
  third-party engine behind `torch.nn.CTCLoss` used at espnet2/asr/ctc.py:39-41,55) in
  float64: alpha/beta over the blank-interleaved label, `zero_infinity` semantics, and
  the gradient w.r.t. the *logits* fed to `log_softmax` (ctc.py:53).
* `forced_align_np` restates espnet1 `CTC.forced_align`
  (espnet/nets/pytorch_backend/ctc.py:185-249) bit-for-bit, including its two quirks
  (SURVEY.md §0.5): state s=0 also reads state -1 (Python wrap to the last state), and
  every `max + lpz` is computed in fp32 then stored in a float64 table.
* `ctc_argmax_np` restates `CTC.argmax` (espnet2/asr/ctc.py:119-127): first max wins.
* `ctc_prefix_init_np` / `ctc_prefix_score_np` restate the beam-search CTC prefix scorer
  (espnet/nets/ctc_prefix_score.py:279-359, CTCPrefixScore.initial_state / __call__) in fp32
  with numpy's logaddexp, pinned by tests/golden/inference.npz.
"""
from __future__ import annotations

import numpy as np


def _lse(a, b):
    m = np.maximum(a, b)
    with np.errstate(invalid="ignore"):
        r = m + np.log(np.exp(a - m) + np.exp(b - m))
    return np.where(np.isneginf(m), -np.inf, r)


def ctc_loss_np(logits, ilens, targets, tlens, blank=0, zero_infinity=True):
    """logits (T,B,V) float; targets (B,Umax) int.  Returns (nll (B,), grad_logits (T,B,V)).

    grad is d(sum_b nll_b)/d logits with nll zeroed (and its gradient) where infinite.
    """
    logits = np.asarray(logits, dtype=np.float64)
    T, B, V = logits.shape
    mx = logits.max(-1, keepdims=True)
    lp = logits - mx - np.log(np.exp(logits - mx).sum(-1, keepdims=True))
    nll = np.zeros(B)
    grad = np.zeros_like(lp)
    for b in range(B):
        Tb, U = int(ilens[b]), int(tlens[b])
        y = np.asarray(targets[b][:U], dtype=np.int64)
        S = 2 * U + 1
        lab = np.full(S, blank, dtype=np.int64)
        lab[1::2] = y
        la = np.full((Tb, S), -np.inf)
        lb = np.full((Tb, S), -np.inf)
        if Tb == 0:
            nll[b] = np.inf
        else:
            la[0, 0] = lp[0, b, blank]
            if S > 1:
                la[0, 1] = lp[0, b, lab[1]]
            for t in range(1, Tb):
                for s in range(S):
                    v = la[t - 1, s]
                    if s >= 1:
                        v = _lse(v, la[t - 1, s - 1])
                    if s >= 2 and lab[s] != blank and lab[s] != lab[s - 2]:
                        v = _lse(v, la[t - 1, s - 2])
                    la[t, s] = v + lp[t, b, lab[s]]
            lb[Tb - 1, S - 1] = lp[Tb - 1, b, blank]
            if S > 1:
                lb[Tb - 1, S - 2] = lp[Tb - 1, b, lab[S - 2]]
            for t in range(Tb - 2, -1, -1):
                for s in range(S):
                    v = lb[t + 1, s]
                    if s + 1 < S:
                        v = _lse(v, lb[t + 1, s + 1])
                    if s + 2 < S and lab[s] != blank and lab[s] != lab[s + 2]:
                        v = _lse(v, lb[t + 1, s + 2])
                    lb[t, s] = v + lp[t, b, lab[s]]
            ll = la[Tb - 1, S - 1] if S == 1 else _lse(la[Tb - 1, S - 1], la[Tb - 1, S - 2])
            nll[b] = -ll
        if not np.isfinite(nll[b]):
            if zero_infinity:
                nll[b] = 0.0
            continue
        # d nll / d lp[t,c] = -exp(la+lb-lp - ll) summed over s with lab[s]==c
        prob = np.exp(lp[:Tb, b])
        occ = np.zeros((Tb, V))
        with np.errstate(invalid="ignore", over="ignore"):
            g = np.exp(la + lb - lp[:Tb, b][:, lab] + nll[b])
        np.add.at(occ, (slice(None), lab), 0.0)
        for s in range(S):
            occ[:, lab[s]] += g[:, s]
        glp = -occ                                  # d nll / d lp
        grad[:Tb, b] = glp - prob * glp.sum(-1, keepdims=True)   # through log_softmax
    return nll, grad


def ctc_argmax_np(logits):
    """(B,T,V) -> (B,T) first-max argmax."""
    return np.argmax(np.asarray(logits), axis=-1)


def forced_align_np(lpz, y, blank_id=0, return_states=False):
    """espnet1 CTC.forced_align (ctc.py:185-249); lpz (T,V) fp32 log-probs, y (U,) int."""
    lpz = np.asarray(lpz, dtype=np.float32)
    y = np.asarray(y, dtype=np.int64)
    lab = np.stack([np.full_like(y, blank_id), y], 1).reshape(-1)
    lab = np.append(lab, lab[0])
    T, S = lpz.shape[0], len(lab)
    logdelta = np.zeros((T, S)) - 100000000000.0
    state_path = np.zeros((T, S), dtype=np.int16) - 1
    logdelta[0, 0] = lpz[0][lab[0]]
    logdelta[0, 1] = lpz[0][lab[1]]
    for t in range(1, T):
        for s in range(S):
            if lab[s] == blank_id or s < 2 or lab[s] == lab[s - 2]:
                cands = np.array([logdelta[t - 1, s], logdelta[t - 1, s - 1]])
                prev = [s, s - 1]
            else:
                cands = np.array([logdelta[t - 1, s], logdelta[t - 1, s - 1], logdelta[t - 1, s - 2]])
                prev = [s, s - 1, s - 2]
            # reference: np.max(float64 array) + 0-dim fp32 torch tensor -> fp32 add
            logdelta[t, s] = np.float32(np.float32(np.max(cands)) + lpz[t][lab[s]])
            state_path[t, s] = prev[int(np.argmax(cands))]
    seq = -1 * np.ones(T, dtype=np.int64)
    cands = np.array([logdelta[-1, S - 1], logdelta[-1, S - 2]])
    seq[-1] = [S - 1, S - 2][int(np.argmax(cands))]
    for t in range(T - 2, -1, -1):
        seq[t] = state_path[t + 1, seq[t + 1]]
    labels = [int(lab[s]) for s in seq]
    # return_states: also the state index per frame as the reference holds it (-1 = the s = 0 wrap)
    return (labels, seq.tolist()) if return_states else labels


LOGZERO = np.float32(-10000000000.0)


def ctc_prefix_init_np(lp, blank=0):
    """initial_state (ctc_prefix_score.py:290-302): r^n = logzero, r^b = cumulative blank."""
    T = lp.shape[0]
    r = np.full((T, 2), LOGZERO, dtype=np.float32)
    r[0, 1] = lp[0, blank]
    for t in range(1, T):
        r[t, 1] = r[t - 1, 1] + lp[t, blank]
    return r


def ctc_prefix_score_np(lp, y, cs, r_prev, blank, eos):
    """__call__ (ctc_prefix_score.py:304-359) for prefix y (with <sos>), candidates cs:
    returns (log_psi (C,), r (C, T, 2)); rows before the recursion start are logzero."""
    lp = np.asarray(lp, dtype=np.float32)
    T = lp.shape[0]
    n_out = len(y) - 1
    C = len(cs)
    xs = lp[:, cs]
    r = np.full((T, 2, C), LOGZERO, dtype=np.float32)
    if n_out == 0:
        r[0, 0] = xs[0]
    r_sum = np.logaddexp(r_prev[:, 0], r_prev[:, 1])
    phi = np.repeat(r_sum[:, None], C, axis=1)
    if n_out > 0:
        for i, c in enumerate(cs):
            if c == y[-1]:
                phi[:, i] = r_prev[:, 1]
    start = max(n_out, 1)
    psi = r[start - 1, 0].copy()
    for t in range(start, T):
        r[t, 0] = np.logaddexp(r[t - 1, 0], phi[t - 1]) + xs[t]
        r[t, 1] = np.logaddexp(r[t - 1, 0], r[t - 1, 1]) + lp[t, blank]
        psi = np.logaddexp(psi, phi[t - 1] + xs[t])
    psi[np.asarray(cs) == eos] = r_sum[-1]
    psi[np.asarray(cs) == blank] = LOGZERO
    return psi, np.moveaxis(r, 2, 0)
