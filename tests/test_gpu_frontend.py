"""Front end on the GPU: the fused STFT -> power -> log-mel kernel and
GlobalMVN against the reference's own outputs (tests/golden/frontend.npz, produced by the
reference Stft / LogMel / GlobalMVN modules) and against the CPU oracle on ragged batches; a
training step of a model whose features come from raw samples, against the oracle; and the
same model replayed as a HIP graph."""
import os

import numpy as np
import pytest
import torch

from oracle import espnet_cpu as O
from oracle import frontend_cpu as FE
from tests.helpers import build_model, small_cfg

pytestmark = pytest.mark.gpu

# fp32 FFT (radix-2 in LDS) vs pocketfft: ~1e-6 relative on the band energies; log-mel atol:
FEAT_ATOL = 1e-4


def _golden():
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "frontend.npz"))


def test_fbank_kernel_vs_reference_golden(dev):
    from espnet_slurp_amd.asr.frontend.default import DefaultFrontend
    g = _golden()
    fe = DefaultFrontend()
    assert np.array_equal(fe.logmel.melmat.numpy(), g["melmat"])
    feats, flens = fe(torch.from_numpy(g["x"]).to(dev), torch.from_numpy(g["lens"]))
    torch.cuda.synchronize()
    assert np.array_equal(flens.numpy(), g["olens"])
    ref = g["feats"]
    got = feats.cpu().numpy()
    assert got.shape == ref.shape
    assert float(np.abs(got - ref).max()) < FEAT_ATOL
    for b, n in enumerate(g["olens"]):
        assert not got[b, n:].any()  # padded frames exactly 0 (log_mel.py:73)


@pytest.mark.parametrize("n_fft,hop,n_mels", [(512, 128, 80), (400, 160, 80), (256, 64, 40)])
def test_fbank_kernel_vs_oracle_ragged(dev, n_fft, hop, n_mels):
    """Ragged lengths (not multiples of hop, one short utterance), reflect padding at both ends
    of the (B, N) tensor, several STFT geometries (n_fft 400: the direct-DFT path)."""
    from espnet_slurp_amd.asr.frontend.default import DefaultFrontend
    g = torch.Generator().manual_seed(5)
    lens = torch.tensor([5000, 4123, 2999, 700])
    x = torch.randn(4, 5200, generator=g) * 0.5
    for b, n in enumerate(lens.tolist()):
        x[b, n:] = 0.0
    fe = DefaultFrontend(n_fft=n_fft, hop_length=hop, n_mels=n_mels)
    feats, flens = fe(x.to(dev), lens)
    ref, rlens = FE.default_frontend(x, lens, 16000, n_fft, hop, n_mels)
    assert torch.equal(flens, rlens)
    assert feats.shape == ref.shape
    assert float((feats.cpu() - ref).abs().max()) < FEAT_ATOL


def test_global_mvn_kernel_vs_reference_golden(dev, tmp_path):
    from espnet_slurp_amd.layers.global_mvn import GlobalMVN
    g = _golden()
    p = tmp_path / "feats_stats.npz"
    np.savez(p, count=g["stat_count"], sum=g["stat_sum"], sum_square=g["stat_sum_square"])
    gm = GlobalMVN(p)
    y, _ = gm(torch.from_numpy(g["feats"]).to(dev), torch.from_numpy(g["olens"]))
    assert float((y.cpu() - torch.from_numpy(g["normed"])).abs().max()) < 1e-5


def _frontend_model(dev):
    from espnet_slurp_amd.asr.frontend.default import DefaultFrontend
    cfg = small_cfg("latest")
    model = build_model(cfg, dev, frontend=DefaultFrontend())
    P = O.deterministic_params(cfg, 21)
    P["frontend.logmel.melmat"] = model.state_dict()["frontend.logmel.melmat"].cpu()  # state_dict key as the reference
    model.load_state_dict(P, strict=True)
    model.train()
    return cfg, model


def _wave_batch(seed):
    g = torch.Generator().manual_seed(seed)
    lens = torch.tensor([9000, 7731, 6400])
    x = torch.randn(3, 9000, generator=g) * 0.3
    for b, n in enumerate(lens.tolist()):
        x[b, n:] = 0.0
    text = torch.randint(2, 31, (3, 6), generator=g)
    tlen = torch.tensor([6, 4, 5])
    for b, n in enumerate(tlen.tolist()):
        text[b, n:] = -1
    return x, lens, text, tlen


def test_model_step_from_raw_samples_vs_oracle(dev):
    cfg, model = _frontend_model(dev)
    x, lens, text, tlen = _wave_batch(8)
    loss, stats, _ = model(x.to(dev), lens, text.clone(), tlen)
    loss.backward()
    torch.cuda.synchronize()
    feats, flens = FE.default_frontend(x, lens)
    P = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k)
         for k, v in O.deterministic_params(cfg, 21).items()}
    ref, rstats, _ = O.asr_forward(P, feats, flens, text.clone(), tlen, cfg, bn_state={})
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-4 * max(1.0, abs(ref.item())), (loss.item(), ref.item())
    g = model.encoder.encoders[0].feed_forward.w_1.weight.grad.cpu()
    r = P["encoder.encoders.0.feed_forward.w_1.weight"].grad
    assert float((g - r).abs().max()) <= 1e-3 * float(r.abs().max()) + 1e-6


def test_graph_replay_with_frontend(dev):
    """Trainer(cuda_graph=True): the captured step (raw samples -> fbank -> ... -> Adam) replays
    exactly like the eager step, also for a new batch with the same shapes."""
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions

    losses = []
    for graph in (False, True):
        cfg, model = _frontend_model(dev)
        opt = FusedAdam(model.parameters(), model.flat, lr=1e-3)
        tr = Trainer(model, opt, None, TrainerOptions(grad_clip=5.0), cuda_graph=graph)
        out = []
        for seed in (8, 9, 8):
            x, lens, text, tlen = _wave_batch(seed)
            out.append(tr.train_one_step(dict(speech=x.to(dev), speech_lengths=lens, text=text,
                                              text_lengths=tlen))["loss"].item())
        losses.append(out)
    assert all(abs(a - b) <= 1e-6 * max(1.0, abs(a)) for a, b in zip(*losses)), losses
