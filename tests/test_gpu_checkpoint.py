"""Checkpoint interop on the GPU: resume from the reference's
checkpoint.pth (tests/golden/checkpoint_ref.pth) onto the device, then
  * one FusedAdam step (HIP kernel) equals torch.optim.Adam's step from the same checkpoint
    with the same gradient (the reference's optimizer, CPU fp32; tolerance: fp32 rounding of
    the update, 1e-6 absolute on parameters of magnitude <= ~1);
  * the HIP-graph trainer resumed from it trains exactly like the eager trainer resumed from it
    (the device-side Adam / WarmupLR counters are initialised from the loaded state)."""
import pytest
import torch

from oracle import espnet_cpu as O
from tests.test_checkpoint import REF_CKPT, _meta, _ours

pytestmark = pytest.mark.gpu


def test_resume_then_adam_step_matches_torch_adam(dev):
    from espnet_slurp_amd.train import checkpoint as CK
    model, opt, sch, rep = _ours(dev)
    CK.resume(REF_CKPT, model, rep, [opt], [sch], None, ngpu=1)
    ref = CK.safe_load(REF_CKPT)
    names = _meta()["param_names"]
    cpu = [torch.nn.Parameter(ref["model"][n].clone()) for n in names]
    tadam = torch.optim.Adam(cpu, lr=1.0)
    tadam.load_state_dict(ref["optimizers"][0])
    g = torch.Generator().manual_seed(3)
    params = dict(model.named_parameters())
    for n, p in zip(names, cpu):
        p.grad = torch.randn(p.shape, generator=g) * 0.1
        model.flat.gview(params[n]).copy_(p.grad)
    opt.step()
    tadam.step()
    torch.cuda.synchronize()
    assert opt.n_steps == 3
    for n, p in zip(names, cpu):
        assert float((params[n].detach().cpu() - p.detach()).abs().max()) < 1e-6, n


def test_graph_trainer_resumed_matches_eager_resumed(dev):
    from espnet_slurp_amd.train import checkpoint as CK
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions
    m = _meta()["cfg"]
    out = []
    for graph in (False, True):
        model, opt, sch, rep = _ours(dev, dropout=0.0)
        CK.resume(REF_CKPT, model, rep, [opt], [sch], None, ngpu=1)
        tr = Trainer(model, opt, sch, TrainerOptions(grad_clip=5.0), cuda_graph=graph)
        losses = []
        for seed in (31, 32):
            speech, slen, text, tlen = O.synthetic_batch(2, 48, 80, m["V"], [48, 40], [4, 3], seed)
            losses.append(tr.train_one_step(dict(speech=speech.to(dev), speech_lengths=slen, text=text,
                                                 text_lengths=tlen))["loss"].item())
        tr.resolve_pending()
        tr.sync_host_state()
        out.append((losses, opt.n_steps, sch.last_epoch, opt.param_groups[0]["lr"], model.flat.flat.cpu()))
    (le, ne, se, lre, pe), (lg, ng, sg, lrg, pg) = out
    assert (ne, se) == (ng, sg) == (4, 4)
    assert lre == lrg
    assert all(abs(a - b) <= 1e-6 * max(1.0, abs(a)) for a, b in zip(le, lg)), (le, lg)
    assert float((pe - pg).abs().max()) < 1e-6
