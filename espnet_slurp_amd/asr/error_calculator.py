"""ErrorCalculator — eval-mode CER / WER of espnet/nets/e2e_asr_common.py:101-257.

ESPnetASRModel reports `cer_ctc` (greedy CTC, espnet_model.py:525-540) and `cer` / `wer`
(attention-decoder argmax, espnet_model.py:515-521) when not training.  The greedy argmaxes
run on device (esp_argmax); the string bookkeeping and edit distances are host work, as in
the reference (which calls `.cpu()` and the `editdistance` package).
"""
from __future__ import annotations

from itertools import groupby
from typing import List, Optional, Sequence

import numpy as np


def edit_distance(a: Sequence, b: Sequence) -> int:
    """Unit-cost Levenshtein distance (what `editdistance.eval` returns), one DP row at a time."""
    a, b = list(a), list(b)
    if not a:
        return len(b)
    if not b:
        return len(a)
    ids = {}
    bb = np.array([ids.setdefault(x, len(ids)) for x in b], dtype=np.int64)
    j = np.arange(len(b) + 1, dtype=np.int64)
    prev = j.copy()
    for i, x in enumerate(a, 1):
        # best[j] = min(substitute / match from prev[j-1], delete from prev[j])
        best = np.minimum(prev[:-1] + (bb != ids.get(x, -1)), prev[1:] + 1)
        # cur[j] = min(best[j], cur[j-1] + 1) with cur[0] = i: a running minimum of best[k] - k
        prev = np.minimum.accumulate(np.concatenate([[i], best - j[1:]])) + j
    return int(prev[-1])


class ErrorCalculator:
    def __init__(self, char_list: List[str], sym_space: str, sym_blank: str, report_cer: bool = False,
                 report_wer: bool = False):
        self.report_cer = report_cer
        self.report_wer = report_wer
        self.char_list = char_list
        self.space = sym_space
        self.blank = sym_blank
        self.idx_blank = self.char_list.index(self.blank)
        self.idx_space = self.char_list.index(self.space) if self.space in self.char_list else None

    def __call__(self, ys_hat, ys_pad, is_ctc: bool = False):
        if is_ctc:
            return self.calculate_cer_ctc(ys_hat, ys_pad)
        if not self.report_cer and not self.report_wer:
            return None, None
        seqs_hat, seqs_true = self.convert_to_char(ys_hat, ys_pad)
        cer = self.calculate_cer(seqs_hat, seqs_true) if self.report_cer else None
        wer = self.calculate_wer(seqs_hat, seqs_true) if self.report_wer else None
        return cer, wer

    def _keep(self, idx: int) -> bool:
        return idx != -1 and idx != self.idx_blank and idx != self.idx_space

    def calculate_cer_ctc(self, ys_hat, ys_pad) -> Optional[float]:
        """Collapse repeats, drop blank / space / padding, character edit distance (:145-178)."""
        eds, ref_lens = [], []
        for i, y in enumerate(np.asarray(ys_hat)):
            hyp = "".join(self.char_list[int(t)] for t, _ in groupby(y) if self._keep(int(t)))
            ref = "".join(self.char_list[int(t)] for t in np.asarray(ys_pad[i]) if self._keep(int(t)))
            if len(ref) > 0:
                eds.append(edit_distance(hyp, ref))
                ref_lens.append(len(ref))
        return float(sum(eds)) / sum(ref_lens) if eds else None

    def convert_to_char(self, ys_hat, ys_pad):
        """(:180-205): the hypothesis is cut at the reference's first padding position."""
        seqs_hat, seqs_true = [], []
        ys_pad = np.asarray(ys_pad)
        for i, y_hat in enumerate(np.asarray(ys_hat)):
            y_true = ys_pad[i]
            eos_true = np.where(y_true == -1)[0]
            ymax = eos_true[0] if len(eos_true) > 0 else len(y_true)
            hyp = "".join(self.char_list[int(t)] for t in y_hat[:ymax])
            ref = "".join(self.char_list[int(t)] for t in y_true if int(t) != -1)
            seqs_hat.append(hyp.replace(self.space, " ").replace(self.blank, ""))
            seqs_true.append(ref.replace(self.space, " "))
        return seqs_hat, seqs_true

    def calculate_cer(self, seqs_hat, seqs_true) -> float:
        eds = [edit_distance(h.replace(" ", ""), t.replace(" ", "")) for h, t in zip(seqs_hat, seqs_true)]
        return float(sum(eds)) / sum(len(t.replace(" ", "")) for t in seqs_true)

    def calculate_wer(self, seqs_hat, seqs_true) -> float:
        eds = [edit_distance(h.split(), t.split()) for h, t in zip(seqs_hat, seqs_true)]
        return float(sum(eds)) / sum(len(t.split()) for t in seqs_true)
