"""Inference on the MI355X: eval-mode encoder (BatchNorm running stats),
the HIP CTC prefix scorer and the joint CTC/attention beam search, against the reference's
own encode / CTCPrefixScore / BeamSearch outputs (tests/golden/inference.npz).
Gates: prefix scores atol 1e-4 (fp32 recursions of ~40 frames); encoder output atol 1e-4;
beam search: identical best token sequence and n-best order, scores within 1e-3 relative."""
import numpy as np
import pytest
import torch

from espnet_slurp_amd import kernels as K
from oracle import ctc_np
from tests.helpers import build_model, golden, load_seeded, small_cfg

pytestmark = pytest.mark.gpu


def test_ctc_prefix_kernel_matches_reference(dev):
    g = golden("inference")
    lp = torch.tensor(g["cps_lp"], device=dev)
    V = lp.shape[1]
    r = K.ctc_prefix_init(lp, 0)
    np.testing.assert_allclose(r.cpu().numpy(), g["cps_r0"], rtol=0, atol=1e-4)
    y = [V - 1]
    for step, nxt in enumerate(g["cps_steps"]):
        cs = torch.tensor(g["cps_cands"][step], device=dev)[None]
        psi, rs = K.ctc_prefix_score(lp, r[None].contiguous(), torch.tensor([y[-1]], device=dev), len(y) - 1, cs, 0,
                                     V - 1)
        np.testing.assert_allclose(psi[0].cpu().numpy(), g["cps_psi"][step], rtol=0, atol=1e-4)
        start = max(len(y) - 1, 1) - 1
        np.testing.assert_allclose(rs[0, :, start:].cpu().numpy(), g["cps_r"][step][:, start:], rtol=0, atol=1e-4)
        i = int(np.where(g["cps_cands"][step] == nxt)[0][0])
        r = rs[0, i].contiguous()
        y = y + [int(nxt)]


def test_ctc_prefix_kernel_batched_vs_oracle(dev):
    rng = np.random.RandomState(3)
    T, V, NH, C = 57, 20, 5, 7
    lp = torch.log_softmax(torch.tensor(rng.randn(T, V) * 3, dtype=torch.float32), -1).numpy()
    prefixes = [[V - 1] + list(rng.randint(1, V - 1, 4)) for _ in range(NH)]
    prefixes[1][-1] = prefixes[1][-2]  # repeated label
    states = []
    for y in prefixes:  # state of each prefix by successive oracle calls
        r = ctc_np.ctc_prefix_init_np(lp, 0)
        for k in range(1, len(y)):
            psi, rs = ctc_np.ctc_prefix_score_np(lp, y[:k], np.array([y[k]]), r, 0, V - 1)
            r = rs[0]
        states.append(r)
    cands = np.stack([rng.choice(V, C, replace=False) for _ in range(NH)])
    cands[0, 0], cands[2, 1] = 0, V - 1
    cands[1, 2] = prefixes[1][-1]
    psi, rs = K.ctc_prefix_score(torch.tensor(lp, device=dev), torch.tensor(np.stack(states), device=dev),
                                 torch.tensor([y[-1] for y in prefixes], device=dev), 4, torch.tensor(cands, device=dev),
                                 0, V - 1)
    for n, y in enumerate(prefixes):
        want_psi, want_r = ctc_np.ctc_prefix_score_np(lp, y, cands[n], states[n], 0, V - 1)
        np.testing.assert_allclose(psi[n].cpu().numpy(), want_psi, rtol=0, atol=1e-4)
        np.testing.assert_allclose(rs[n, :, 3:].cpu().numpy(), want_r[:, 3:], rtol=0, atol=1e-4)


def _model(dev):
    g = golden("inference")
    cfg = small_cfg("latest", D=64, blocks=2, V=32)
    model = build_model(cfg, dev, dropout=0.0)
    load_seeded(model, cfg, 21)
    with torch.no_grad():
        for name, buf in model.named_buffers():
            if "bn." + name in g:
                buf.copy_(torch.tensor(g["bn." + name]))
    model.eval()
    return model, g


def test_eval_encoder_matches_reference(dev):
    model, g = _model(dev)
    from espnet_slurp_amd.bin.asr_inference import Speech2Text
    s2t = Speech2Text(model, beam_size=2)
    enc = s2t.encode(torch.tensor(g["speech"][0]))
    assert enc.shape == g["enc"].shape
    np.testing.assert_allclose(enc.cpu().numpy(), g["enc"], rtol=0, atol=1e-4)


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_beam_search_matches_reference(dev, tag):
    from espnet_slurp_amd.bin.asr_inference import Speech2Text
    model, g = _model(dev)
    ctc_w, beam, penalty = g[f"bs_{tag}_cfg"]
    s2t = Speech2Text(model, beam_size=int(beam), ctc_weight=float(ctc_w), penalty=float(penalty), nbest=int(beam))
    res = s2t(torch.tensor(g["speech"][0]))
    want_y, want_s = g[f"bs_{tag}_plain_yseq"], g[f"bs_{tag}_plain_score"]
    best = res[0][3]
    w0 = want_y[0][want_y[0] >= 0]
    assert best.yseq.tolist() == w0.tolist()
    assert abs(best.score - want_s[0]) <= 1e-3 * abs(want_s[0])
    assert res[0][2] == [t for t in w0[1:-1].tolist() if t != 0]
    n = min(len(res), len(want_s), 3)
    for i in range(n):
        wi = want_y[i][want_y[i] >= 0]
        assert res[i][3].yseq.tolist() == wi.tolist(), i
        assert abs(res[i][3].score - want_s[i]) <= 1e-3 * abs(want_s[i]), i


def test_slu_model_loss_equals_asr(dev):
    """Same weights and batch: the SLU model's training loss is the ASR model's (transcript ignored)."""
    from oracle import espnet_cpu as O
    from espnet_slurp_amd.slu.espnet_model import ESPnetSLUModel
    from tests.helpers import token_list
    cfg = small_cfg("latest")
    asr = build_model(cfg, dev, dropout=0.0)
    load_seeded(asr, cfg, 9)
    from tests.test_slu import _parts
    slu = ESPnetSLUModel(vocab_size=cfg.vocab_size, token_list=token_list(cfg.vocab_size), ctc_weight=cfg.ctc_weight,
                         lsm_weight=cfg.lsm_weight, **_parts(cfg)).to(dev)
    slu.flatten()
    load_seeded(slu, cfg, 9)
    speech, slen, text, tlen = O.synthetic_batch(2, 96, 80, cfg.vocab_size, [96, 70], [6, 4], 3)
    asr.train()
    slu.train()
    la = asr(speech.to(dev), slen, text.clone(), tlen)[0].item()
    ls = slu(speech.to(dev), slen, text.clone(), tlen, transcript=text.clone(), transcript_lengths=tlen)[0].item()
    assert abs(la - ls) <= 1e-6 * max(1.0, abs(la)), (la, ls)
