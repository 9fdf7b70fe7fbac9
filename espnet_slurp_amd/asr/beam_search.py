"""Joint CTC/attention beam search (espnet/nets/beam_search.py:20-512 with
espnet/nets/scorers/ctc.py, espnet/nets/scorers/length_bonus.py, e2e_asr_common.end_detect).

Same search as the reference's BeamSearch (what Speech2Text runs, as BatchBeamSearch, for an
ESPnet2 ASR model): per running hypothesis the full scorers (decoder log-softmax, length
bonus) are weighted and summed, the pre-beam keeps int(pre_beam_ratio * beam) labels by that
sum ("full" key), the CTC prefix scorer scores only those, the hypothesis score is added, the
top `beam` of every hypothesis are pooled, stably sorted and pruned to `beam`; hypotheses that
emit <eos> (or reach maxlen) end, and end_detect stops the search when maxlenratio == 0.

MI355X-side: all running hypotheses are scored together — ONE decoder pass over the stacked
prefixes (the HIP decoder kernels, encoder memory repeated per hypothesis) and ONE launch of
the CTC prefix kernel (esp_ctc_prefix_score: a thread per (hypothesis, candidate)) per output
step; the hypothesis bookkeeping (tiny) happens on the host after one device->host copy.
The decoder is re-run on the full prefix each step (the reference caches layer outputs in
forward_one_step; the last position's output is the same function of the prefix).
"""
import math
from itertools import chain
from typing import Any, Dict, List, NamedTuple, Optional

import numpy as np
import torch

from .. import kernels as K


class Hypothesis(NamedTuple):
    yseq: torch.Tensor
    score: float = 0.0
    scores: Dict[str, float] = dict()
    states: Dict[str, Any] = dict()

    def asdict(self) -> dict:
        return dict(yseq=self.yseq.tolist(), score=float(self.score), scores={k: float(v) for k, v in self.scores.items()})


def end_detect(ended_hyps, i, M=3, D_end=np.log(1 * np.exp(-10))):
    """e2e_asr_common.py:19-49: stop when, for each of the last M lengths, the best ended
    hypothesis of that length is worse than the overall best by more than |D_end|."""
    if len(ended_hyps) == 0:
        return False
    best = max(h["score"] for h in ended_hyps)
    count = 0
    for m in range(M):
        same = [h["score"] for h in ended_hyps if len(h["yseq"]) == i - m]
        if same and max(same) - best < D_end:
            count += 1
    return count == M


class DecoderScorer:
    """Full scorer: log p(. | prefix, x) of the attention decoder for all hypotheses at once."""

    def __init__(self, decoder):
        self.decoder = decoder

    def batch_score(self, yseqs: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        NH, L = yseqs.shape
        T, D = x.shape
        mem = x.unsqueeze(0).expand(NH, T, D).contiguous()
        hl = torch.full((NH,), T, dtype=torch.int64)
        yl = torch.full((NH,), L, dtype=torch.int64)
        logits, _ = self.decoder(mem, hl, yseqs, yl)
        last = logits[:, -1, :].contiguous()
        lp = torch.empty_like(last)
        K.log_softmax(last, lp, NH, last.shape[1])
        return lp


class LengthBonus:
    """Full scorer: +1 for every label (scorers/length_bonus.py:9-61), weighted by `penalty`."""

    @staticmethod
    def final_score(state) -> float:
        return 0.0


class CTCPrefixScorer:
    """Partial scorer (scorers/ctc.py:9-71 + ctc_prefix_score.py CTCPrefixScore).  State per
    hypothesis: (prefix log-prob psi of the hypothesis, its (T, 2) forward variables)."""

    def __init__(self, ctc, eos: int, blank: int = 0):
        self.ctc, self.eos, self.blank = ctc, eos, blank
        self.lp = None

    def init_state(self, x: torch.Tensor):
        self.lp = self.ctc.log_softmax(x.unsqueeze(0))[0].contiguous()
        return 0.0, K.ctc_prefix_init(self.lp, self.blank)

    def batch_score_partial(self, yseqs: torch.Tensor, ids: torch.Tensor, states: List[Any]):
        """ids (NH, C) labels per hypothesis -> (score deltas (NH, C), log_psi (NH, C), r (NH, C, T, 2))."""
        NH = yseqs.shape[0]
        dev = self.lp.device
        r_prev = torch.stack([s[1] for s in states]).contiguous()
        prev = torch.tensor([s[0] for s in states], dtype=torch.float32, device=dev)
        last = yseqs[:, -1].to(dev).contiguous()
        psi, r_new = K.ctc_prefix_score(self.lp, r_prev, last, yseqs.shape[1] - 1, ids.to(dev).contiguous(),
                                        self.blank, self.eos)
        return psi - prev[:, None], psi, r_new

    @staticmethod
    def final_score(state) -> float:
        return 0.0


class BeamSearch:
    def __init__(self, scorers: Dict[str, Any], weights: Dict[str, float], beam_size: int, vocab_size: int,
                 sos: int, eos: int, token_list: Optional[List[str]] = None, pre_beam_ratio: float = 1.5,
                 pre_beam_score_key: Optional[str] = "full"):
        self.weights = weights
        self.full_scorers, self.part_scorers = {}, {}
        for k, v in scorers.items():
            if v is None or weights.get(k, 0) == 0:
                continue
            if k == "ctc":
                self.part_scorers[k] = v
            else:
                self.full_scorers[k] = v
        self.sos, self.eos = sos, eos
        self.token_list = token_list
        self.beam_size = beam_size
        self.n_vocab = vocab_size
        self.pre_beam_size = int(pre_beam_ratio * beam_size)
        self.pre_beam_score_key = pre_beam_score_key
        self.do_pre_beam = (pre_beam_score_key is not None and self.pre_beam_size < self.n_vocab
                            and len(self.part_scorers) > 0)

    def init_hyp(self, x: torch.Tensor) -> List[Hypothesis]:
        states = {k: (d.init_state(x) if hasattr(d, "init_state") else None)
                  for k, d in chain(self.full_scorers.items(), self.part_scorers.items())}
        return [Hypothesis(yseq=torch.tensor([self.sos], dtype=torch.int64), score=0.0,
                           scores={k: 0.0 for k in chain(self.full_scorers, self.part_scorers)}, states=states)]

    def search(self, running: List[Hypothesis], x: torch.Tensor) -> List[Hypothesis]:
        NH, V, dev = len(running), self.n_vocab, x.device
        yseqs = torch.stack([h.yseq for h in running])
        full = {}
        weighted = torch.zeros(NH, V, dtype=torch.float32, device=dev)
        for k, d in self.full_scorers.items():
            full[k] = d.batch_score(yseqs.to(dev), x) if k == "decoder" else torch.ones(NH, V, device=dev)
            weighted += self.weights[k] * full[k]
        if self.do_pre_beam:
            pre = weighted if self.pre_beam_score_key == "full" else full[self.pre_beam_score_key]
            part_ids = torch.topk(pre, self.pre_beam_size, dim=1)[1]
        else:
            part_ids = torch.arange(V, device=dev).expand(NH, V)
        part, part_states = {}, {}
        for k, d in self.part_scorers.items():
            delta, psi, r_new = d.batch_score_partial(yseqs, part_ids, [h.states[k] for h in running])
            part[k] = delta
            part_states[k] = (psi, r_new)
            weighted.scatter_add_(1, part_ids, self.weights[k] * delta)
        weighted += torch.tensor([float(h.score) for h in running], dtype=torch.float32, device=dev)[:, None]
        # per hypothesis: top `beam` over the pre-beam survivors (others masked to -inf)
        if part_ids.shape[1] < V:
            masked = torch.full_like(weighted, -float("inf"))
            masked.scatter_(1, part_ids, weighted.gather(1, part_ids))
        else:
            masked = weighted
        top_ids = torch.topk(masked, self.beam_size, dim=1)[1]
        local_ids = torch.topk(masked.gather(1, part_ids), self.beam_size, dim=1)[1] \
            if part_ids.shape[1] < V else top_ids
        # one device->host copy of everything the bookkeeping needs
        h_top, h_loc = top_ids.cpu(), local_ids.cpu()
        h_w = weighted.gather(1, top_ids).cpu()
        h_full = {k: v.gather(1, top_ids).cpu() for k, v in full.items()}
        h_part = {k: v.gather(1, local_ids).cpu() for k, v in part.items()}
        best = []
        for n, hyp in enumerate(running):
            for b in range(self.beam_size):
                j, pj = int(h_top[n, b]), int(h_loc[n, b])
                scores = {k: hyp.scores[k] + float(h_full[k][n, b]) for k in self.full_scorers}
                for k in self.part_scorers:
                    scores[k] = hyp.scores[k] + float(h_part[k][n, b])
                states = dict(hyp.states)
                for k in self.part_scorers:
                    psi, r_new = part_states[k]
                    states[k] = (float(psi[n, pj]), r_new[n, pj])
                best.append(Hypothesis(score=float(h_w[n, b]), yseq=torch.cat([hyp.yseq, torch.tensor([j])]),
                                       scores=scores, states=states))
        # stable sort (the reference sorts after each hypothesis; pooled then sorted is the same set)
        return sorted(best, key=lambda h: h.score, reverse=True)[: min(len(best), self.beam_size)]

    def post_process(self, i: int, maxlen: int, running: List[Hypothesis], ended: List[Hypothesis]):
        if i == maxlen - 1:
            running = [h._replace(yseq=torch.cat([h.yseq, torch.tensor([self.eos])])) for h in running]
        remained = []
        for hyp in running:
            if int(hyp.yseq[-1]) == self.eos:
                for k, d in chain(self.full_scorers.items(), self.part_scorers.items()):
                    s = d.final_score(hyp.states[k]) if hasattr(d, "final_score") else 0.0
                    hyp.scores[k] += s
                    hyp = hyp._replace(score=hyp.score + self.weights[k] * s)
                ended.append(hyp)
            else:
                remained.append(hyp)
        return remained

    def forward(self, x: torch.Tensor, maxlenratio: float = 0.0, minlenratio: float = 0.0) -> List[Hypothesis]:
        maxlen = x.shape[0] if maxlenratio == 0 else max(1, int(maxlenratio * x.size(0)))
        running = self.init_hyp(x)
        ended: List[Hypothesis] = []
        with torch.no_grad():
            for i in range(maxlen):
                best = self.search(running, x)
                running = self.post_process(i, maxlen, best, ended)
                if maxlenratio == 0.0 and end_detect([h.asdict() for h in ended], i):
                    break
                if len(running) == 0:
                    break
        nbest = sorted(ended, key=lambda h: h.score, reverse=True)
        if not nbest:
            return [] if minlenratio < 0.1 else self.forward(x, maxlenratio, max(0.0, minlenratio - 0.1))
        return nbest
