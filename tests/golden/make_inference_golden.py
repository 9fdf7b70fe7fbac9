"""Golden vectors for inference, generated in THIS container with the
reference's own ESPnetASRModel.encode (eval mode), espnet CTCPrefixScore and BeamSearch /
BatchBeamSearch (imported through refshim).  Writes tests/golden/inference.npz (data only).
Run:  python tests/golden/make_inference_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.golden import refshim  # noqa: E402

refshim.install()
from tests.golden.make_golden import build_reference, load_params, small_cfg  # noqa: E402
from oracle import espnet_cpu as O  # noqa: E402


def main():
    from espnet.nets.batch_beam_search import BatchBeamSearch
    from espnet.nets.beam_search import BeamSearch
    from espnet.nets.ctc_prefix_score import CTCPrefixScore
    from espnet.nets.scorers.ctc import CTCPrefixScorer
    from espnet.nets.scorers.length_bonus import LengthBonus

    out = {}
    # 1) CTCPrefixScore known answers: random log-probs, a 3-label prefix, candidates incl. blank/eos/last
    rng = np.random.RandomState(0)
    T, V = 40, 12
    lp = torch.log_softmax(torch.tensor(rng.randn(T, V) * 2, dtype=torch.float32), -1).numpy()
    sc = CTCPrefixScore(lp, 0, V - 1, np)
    r = sc.initial_state()
    out["cps_lp"], out["cps_r0"] = lp, r
    y = [V - 1]
    cands_all, psi_all, r_all = [], [], []
    for step, nxt in enumerate([3, 3, 5]):
        cs = np.array([0, 1, 3, 5, 7, V - 1], dtype=np.int64)
        psi, rs = sc(y, cs, r)
        cands_all.append(cs)
        psi_all.append(psi)
        r_all.append(rs)
        i = int(np.where(cs == nxt)[0][0])
        r = rs[i]
        y = y + [nxt]
    out["cps_cands"], out["cps_psi"], out["cps_r"] = np.stack(cands_all), np.stack(psi_all), np.stack(r_all)
    out["cps_steps"] = np.array([3, 3, 5])

    # 2) end-to-end: small Conformer model, eval mode, encode + joint beam search
    cfg = small_cfg("latest", D=64, blocks=2, V=32)
    model = build_reference(cfg)
    load_params(model, cfg, 21)
    g = torch.Generator().manual_seed(5)
    for name, buf in model.named_buffers():
        if name.endswith("running_mean"):
            buf.copy_(0.1 * torch.randn(buf.shape, generator=g))
            out["bn." + name] = buf.numpy().copy()
        elif name.endswith("running_var"):
            buf.copy_(0.5 + torch.rand(buf.shape, generator=g))
            out["bn." + name] = buf.numpy().copy()
    model.eval()
    speech = torch.randn(1, 240, 80, generator=g)
    with torch.no_grad():
        enc, elen = model.encode(speech, torch.tensor([240]))
    out["speech"], out["enc"] = speech.numpy(), enc[0].numpy()
    V = cfg.vocab_size
    for tag, ctc_w, beam, penalty in (("a", 0.3, 4, 0.0), ("b", 0.5, 6, 0.2), ("c", 1.0, 3, 0.0)):
        scorers = dict(decoder=model.decoder, ctc=CTCPrefixScorer(ctc=model.ctc, eos=model.eos),
                       length_bonus=LengthBonus(V))
        weights = dict(decoder=1.0 - ctc_w, ctc=ctc_w, length_bonus=penalty)
        res = {}
        for kind, cls in (("plain", BeamSearch), ("batch", BatchBeamSearch)):
            bs = BeamSearch(scorers=scorers, weights=weights, beam_size=beam, vocab_size=V, sos=model.sos,
                            eos=model.eos, token_list=None, pre_beam_score_key=None if ctc_w == 1.0 else "full")
            bs.__class__ = cls
            with torch.no_grad():
                hyps = bs(x=enc[0], maxlenratio=0.0, minlenratio=0.0)
            res[kind] = hyps
        for kind in ("plain", "batch"):
            n = len(res[kind])
            L = max(len(h.yseq) for h in res[kind])
            ys = np.full((n, L), -1, dtype=np.int64)
            for i, h in enumerate(res[kind]):
                ys[i, : len(h.yseq)] = h.yseq.numpy()
            out[f"bs_{tag}_{kind}_yseq"] = ys
            out[f"bs_{tag}_{kind}_score"] = np.array([float(h.score) for h in res[kind]])
        out[f"bs_{tag}_cfg"] = np.array([ctc_w, beam, penalty])
        print(tag, "plain best", res["plain"][0].yseq.tolist(), float(res["plain"][0].score),
              "batch best", res["batch"][0].yseq.tolist())
    np.savez_compressed(os.path.join(HERE, "inference.npz"), **out)
    print("wrote inference.npz")


if __name__ == "__main__":
    main()
