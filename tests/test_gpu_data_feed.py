"""Data feed on the GPU: ESPnetDataset (npy fbank + text_int) -> numel sampler -> pinned
CommonCollateFn -> DevicePrefetcher (side-stream H2D) -> Trainer.train_one_epoch.  The epoch
through the prefetcher must give the same losses and parameters as feeding the same batches
synchronously (the prefetch only changes WHEN the copies run)."""
import numpy as np
import pytest
import torch

from tests.helpers import build_model, load_seeded, small_cfg

pytestmark = pytest.mark.gpu


def _corpus(tmp_path, n=10, V=32):
    rng = np.random.RandomState(0)
    feats, text, shape = {}, {}, {}
    for i in range(n):
        k = f"utt{i:02d}"
        T = int(rng.randint(60, 120))
        p = tmp_path / f"{k}.npy"
        np.save(str(p), rng.randn(T, 80).astype(np.float32))
        feats[k], shape[k] = str(p), f"{T},80"
        text[k] = " ".join(str(t) for t in rng.randint(2, V - 1, int(rng.randint(3, 8))))
    for name, tab in (("feats.scp", feats), ("text", text), ("speech_shape", shape)):
        (tmp_path / name).write_text("".join(f"{k} {v}\n" for k, v in tab.items()))
    return tmp_path


def _run(dev, root, prefetch):
    from espnet_slurp_amd.iterators.sequence_iter_factory import DevicePrefetcher, SequenceIterFactory
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.samplers import build_batch_sampler
    from espnet_slurp_amd.train.collate_fn import CommonCollateFn
    from espnet_slurp_amd.train.dataset import ESPnetDataset
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions
    cfg = small_cfg("latest")
    model = build_model(cfg, dev, dropout=0.0)
    load_seeded(model, cfg, 3)
    opt = FusedAdam(model.parameters(), model.flat, lr=1e-3)
    tr = Trainer(model, opt, None, TrainerOptions(grad_clip=5.0))
    ds = ESPnetDataset([(str(root / "feats.scp"), "speech", "npy"), (str(root / "text"), "text", "text_int")])
    sampler = build_batch_sampler("numel", 1, 3 * 120 * 80, [str(root / "speech_shape")])
    fac = SequenceIterFactory(ds, list(sampler), seed=1, shuffle=True,
                              collate_fn=CommonCollateFn(0.0, -1, pin_memory=prefetch))
    losses = []

    class Rep:
        def __call__(self, stats):
            losses.append(stats["loss"].item())

    it = fac.build_iter(1)
    if prefetch:
        it = DevicePrefetcher(it, dev)
    else:
        it = ((ids, dict(b, speech=b["speech"].to(dev))) for ids, b in it)
    tr.train_one_epoch(it, reporter=Rep())
    torch.cuda.synchronize()
    return losses, model.flat.flat.detach().cpu().clone()


def test_prefetched_epoch_matches_sync_feed(dev, tmp_path):
    root = _corpus(tmp_path)
    l_sync, p_sync = _run(dev, root, False)
    l_pre, p_pre = _run(dev, root, True)
    assert len(l_sync) == len(l_pre) >= 3
    assert l_sync == l_pre
    assert torch.equal(p_sync, p_pre)
