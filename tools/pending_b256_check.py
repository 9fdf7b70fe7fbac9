"""Pending check for the B=256 bench batch (tools/b256_default.patch): the
duplicated-batch property test, run explicitly (`pytest tools/pending_b256_check.py`) until it has
passed on hardware and moves into tests/test_gpu_bench_shape.py with the bench default."""
import pytest
import torch

from tests.helpers import FlipProbe, build_model, golden, load_seeded
from tests.test_gpu_bench_shape import _batch, _cfg


@pytest.fixture
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda:0")


def test_bench_shape_b256_duplicated_batch_matches_b128(dev):
    """B=256 (bench.py's default batch since round 4): the fixture's 128 utterances twice over give
    the B=128 step's loss and gradients (utterance-mean normalisation, BatchNorm statistics of a
    duplicated batch equal the original's) -- a size-independent property at the shape the bench
    runs, where the conv1 output holds 1.91e9 elements (int32 index range) and every grid is twice
    the fixture's.  Gates: loss within 1e-5 relative, each parameter's gradient within 5e-4 of its
    norm (GEMM tilings and split-K counts differ with M), 2e-3 for a decoder layer's w_1 / norm3 when
    one of its near-zero ReLU decisions flips between the two (counted, at most 1e-5 of them), exactly-zero
    gradients (the fixture's fp64 ones) within grad_gate's absolute bound."""
    g = golden("bench_c2_b128")
    cfg = _cfg()
    model = build_model(cfg, dev)
    load_seeded(model, cfg, int(g["seed"]))
    model.train()
    speech, slen, text, tlen = _batch(g, dev)
    res, acts = [], []
    for rep in (1, 2):
        model.flat.grad.zero_()
        with FlipProbe(model) as fp:
            loss, stats, _ = model(speech.repeat(rep, 1, 1), slen.repeat(rep), text.clone().repeat(rep, 1),
                                   tlen.repeat(rep))
        loss.backward()
        torch.cuda.synchronize()
        assert torch.isfinite(loss).item()
        res.append((loss.item(), stats["loss_ctc"].item(),
                    {n: p.grad.detach().double().clone() for n, p in model.named_parameters()}))
        # the decoder FFNs' ReLU decisions (dact = keep * scale * (v > 0); dropout 0)
        acts.append([fp.ctx[id(layer.feed_forward)].dact > 0 for layer in model.decoder.decoders])
    (l1, c1, g1), (l2, c2, g2) = res
    # ReLU decisions within rounding of 0 that the two tilings take differently: each changes its
    # layer's w_1 and norm3 gradients by one row's contribution (as against fp64, grad_gate's flip
    # correction); those tensors are held to 2e-3 where their layer has a flip
    flips = []
    for a1, a2 in zip(*acts):
        n1 = a1.shape[0]
        flips.append(int((a2[:n1] != a1).sum().item() + (a2[n1:] != a1).sum().item()))
        assert flips[-1] <= 1e-5 * a1.numel(), flips  # a handful, not a defect
    relu_adj = {f"decoder.decoders.{l}.{t}" for l, f in enumerate(flips) if f
                for t in ("feed_forward.w_1.weight", "feed_forward.w_1.bias", "norm3.weight", "norm3.bias")}
    assert abs(l2 - l1) <= 1e-5 * abs(l1), (l1, l2)
    assert abs(c2 - c1) <= 1e-5 * abs(c1), (c1, c2)
    # tensors whose exact gradient is zero (the key bias under the row softmax, the depthwise bias
    # before BatchNorm): fp32 noise on both sides, held to grad_gate's absolute bound instead
    scale = max(float(g["gmax_f64/" + n]) for n in g1)
    bad = []
    for n, a in g1.items():
        if float(g["gmax_f64/" + n]) < 1e-6 * scale:
            m = max(a.abs().max().item(), g2[n].abs().max().item())
            if m > 1e-5 * scale:
                bad.append((n, "nonzero", m))
            continue
        na = a.norm().item()
        d = (g2[n] - a).norm().item()
        if d > (2e-3 if n in relu_adj else 5e-4) * na + 1e-9:
            bad.append((n, d / max(na, 1e-30)))
    assert not bad, (bad[:10], flips)
