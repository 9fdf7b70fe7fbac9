"""Inference host logic on CPU: the CTC prefix-score oracle against the reference's own
CTCPrefixScore outputs (tests/golden/inference.npz, make_inference_golden.py), end_detect,
and the tokenizers.  The HIP scorer / beam search run in tests/test_gpu_inference.py."""
import numpy as np

from espnet_slurp_amd.asr.beam_search import end_detect
from espnet_slurp_amd.bin.asr_inference import CharTokenizer
from oracle import ctc_np
from tests.helpers import golden


def test_prefix_score_oracle_matches_reference():
    g = golden("inference")
    lp = g["cps_lp"]
    V = lp.shape[1]
    r = ctc_np.ctc_prefix_init_np(lp, 0)
    np.testing.assert_array_equal(r, g["cps_r0"])
    y = [V - 1]
    for step, nxt in enumerate(g["cps_steps"]):
        cs = g["cps_cands"][step]
        psi, rs = ctc_np.ctc_prefix_score_np(lp, y, cs, r, 0, V - 1)
        np.testing.assert_allclose(psi, g["cps_psi"][step], rtol=0, atol=1e-4)
        start = max(len(y) - 1, 1) - 1  # the reference leaves rows before the start uninitialised
        np.testing.assert_allclose(rs[:, start:], g["cps_r"][step][:, start:], rtol=0, atol=1e-4)
        i = int(np.where(cs == nxt)[0][0])
        r = rs[i]
        y = y + [int(nxt)]


def test_end_detect():
    D = np.log(np.exp(-10))
    ended = [dict(yseq=[1, 2, 3], score=-1.0)]
    assert not end_detect([], 5)
    # best ended hyp of lengths i, i-1, i-2 all much worse than the overall best -> stop
    hyps = [dict(yseq=[0] * 3, score=-1.0), dict(yseq=[0] * 10, score=-30.0), dict(yseq=[0] * 9, score=-40.0),
            dict(yseq=[0] * 8, score=-50.0)]
    assert end_detect(hyps, 10)
    assert not end_detect(hyps + [dict(yseq=[0] * 9, score=-2.0)], 10)
    assert not end_detect(ended, 3, D_end=D)


def test_char_tokenizer():
    assert CharTokenizer().tokens2text(["a", "b", "<space>", "c"]) == "ab c"
