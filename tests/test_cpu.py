"""CPU suite (no GPU): the oracle against the reference's golden vectors, the host logic,
the C-ABI library's exports, interface compatibility, and the data-parallel reducer with
world_size=2 gloo processes."""
import ast
import math
import os
import re
import socket

import numpy as np
import pytest
import torch

from oracle import ctc_np
from oracle import espnet_cpu as O
from tests.helpers import golden, rel_err, small_cfg, c1_cfg, c2_cfg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ----------------------------------------------------------------------------- oracle pin
def _oracle_run(cfg, g, dtype=torch.float32):
    P = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k)
         for k, v in O.deterministic_params(cfg, int(g["seed"]), dtype).items()}
    bn = {}
    loss, stats, w = O.asr_forward(P, torch.from_numpy(g["speech"]).to(dtype), torch.from_numpy(g["speech_lengths"]),
                                   torch.from_numpy(g["text"]), torch.from_numpy(g["text_lengths"]), cfg, bn_state=bn)
    loss.backward()
    return loss, stats, P, bn


@pytest.mark.parametrize("name,rel", [("model_small_latest", "latest"), ("model_small_legacy", "legacy")])
def test_oracle_matches_reference_fixture(name, rel):
    g = golden(name)
    loss, stats, P, bn = _oracle_run(small_cfg(rel), g)
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    assert abs(stats["loss_ctc"].item() - float(g["loss_ctc"])) < 1e-5
    assert abs(stats["loss_att"].item() - float(g["loss_att"])) < 1e-5
    assert stats["acc"] == pytest.approx(float(g["acc"]), abs=1e-6)  # fixture holds the fp32 tensor
    for k in g:
        if k.startswith("grad/"):
            assert np.abs(P[k[5:]].grad.numpy() - g[k]).max() < 5e-5, k
        if k.startswith("buf/"):
            assert np.abs(bn[k[4:]].numpy() - g[k]).max() < 1e-6, k


def test_oracle_c1_fixture():
    g = golden("model_c1_transformer_ctc")
    loss, stats, P, _ = _oracle_run(c1_cfg(), g)
    assert abs(loss.item() - float(g["loss"])) < 1e-4
    for k in g:
        if k.startswith("gradnorm/"):
            ref = float(g[k])
            assert abs(P[k[9:]].grad.double().norm().item() - ref) <= 1e-4 * ref + 1e-7, k


def test_oracle_train_step_fixture():
    """2 reference optimizer steps (clip 5 + Adam + WarmupLR(10)) reproduced by the oracle."""
    g = golden("train_step")
    cfg = small_cfg("latest", D=32, blocks=1, V=16)
    P = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k)
         for k, v in O.deterministic_params(cfg, 3).items()}
    params = [P[k] for k in P if P[k].requires_grad]
    opt = torch.optim.Adam(params, lr=0.002, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-6)
    bn = {}
    for step in range(2):
        lr = 0.002 * 10 ** 0.5 * min((step + 1) ** -0.5, (step + 1) * 10 ** -1.5)
        for gr in opt.param_groups:
            gr["lr"] = lr
        assert abs(lr - float(g[f"lr{step}"])) < 1e-12
        speech, slen, text, tlen = O.synthetic_batch(2, 64, 80, cfg.vocab_size, [64, 50], [5, 3], 100 + step)
        loss, _, _ = O.asr_forward(P, speech, slen, text, tlen, cfg, bn_state=bn)
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(params, 5.0)
        assert abs(loss.item() - float(g[f"loss{step}"])) < 1e-5
        assert abs(gn.item() - float(g[f"gradnorm{step}"])) < 1e-4
        opt.step()
        opt.zero_grad()
    # Adam's first steps are sign-like (m/sqrt(v) ~ +-1): an element whose gradient is at
    # fp32 rounding-noise level (e.g. the exactly-zero key-bias / BN-fed conv-bias
    # gradients) moves by +-lr with an arbitrary sign.  So: 99.5% of elements within 2e-6,
    # every element within the sum of the two learning rates (zero-grad tensors ~0.2%).
    lr_sum = float(g["lr0"]) + float(g["lr1"])
    diffs = np.concatenate([np.abs(P[k[6:]].detach().numpy() - g[k]).ravel() for k in g if k.startswith("param/")])
    assert (diffs < 2e-6).mean() > 0.995, (diffs < 2e-6).mean()
    assert diffs.max() <= 2 * lr_sum + 1e-6


def test_oracle_fullsize_loss_gate():
    g = golden("fullsize_c2")
    cfg = c2_cfg("latest")
    P = O.deterministic_params(cfg, int(g["seed"]))
    speech, slen, text, tlen = O.synthetic_batch(2, 1500, 80, 600, list(g["lens"]), list(g["ulens"]), 43)
    with torch.no_grad():
        loss, _, _ = O.asr_forward(P, speech, slen, text, tlen, cfg, bn_state={})
    assert abs(loss.item() - float(g["loss_f32"])) < 2e-4


def test_ctc_numpy_oracle_vs_reference():
    g = golden("ctc")
    nll, grad = ctc_np.ctc_loss_np(g["logits"], g["ilens"], g["targets"], g["tlens"])
    ref = g["nll"]
    assert np.abs(nll - ref).max() < 1e-4
    B = g["logits"].shape[1]
    assert np.abs(grad / B - g["grad"]).max() < 1e-5


def test_forced_align_numpy_oracle_bit_exact():
    g = golden("align")
    for ci in range(4):
        ali = ctc_np.forced_align_np(g[f"lpz{ci}"], g[f"y{ci}"])
        assert np.array_equal(np.array(ali), g[f"ali{ci}"])
        assert np.array_equal(ctc_np.ctc_argmax_np(g[f"h{ci}"]), g[f"argmax{ci}"])


def test_forced_align_numpy_oracle_bit_exact_c2_shape():
    """The oracle against the reference's forced_align at the workload shape (align_c2.npz: T' = 374,
    V = 600, U = 20 / 40; random, tied and trained-like logits, the s = 0 wrap on several frames)."""
    g = golden("align_c2")
    assert int(g["wrap_frames"].max()) > 0
    for ci in range(len(g["kinds"])):
        ali, st = ctc_np.forced_align_np(g[f"lpz{ci}"], g[f"y{ci}"], return_states=True)
        assert np.array_equal(np.array(ali), g[f"ali{ci}"]), ci
        assert sum(1 for s in st if s < 0) == int(g["wrap_frames"][ci])
        assert np.array_equal(ctc_np.ctc_argmax_np(g[f"lpz{ci}"]), g[f"argmax{ci}"])
        if f"h{ci}" in g:
            assert np.array_equal(ctc_np.ctc_argmax_np(g[f"h{ci}"]), g[f"argmax_h{ci}"])


def test_specaug_oracle_vs_reference():
    g = golden("specaug")
    x = torch.from_numpy(g["x"])
    for s in (3, 4):
        y = O.time_warp_fixed(x, int(g[f"tw{s}_center"]), int(g[f"tw{s}_warped"]))
        assert np.abs(y.numpy() - g[f"tw{s}_y"]).max() < 1e-6
    for key, dim in (("freq", 2), ("time", 1)):
        y = O.mask_along_axis_fixed(x, torch.from_numpy(g[f"{key}_pos"]), torch.from_numpy(g[f"{key}_len"]), dim)
        assert np.array_equal(y.numpy(), g[f"{key}_y"])
    y = O.utterance_mvn(torch.from_numpy(g["mvn_x"]), torch.from_numpy(g["mvn_lens"]))
    assert np.abs(y.numpy() - g["mvn_y"]).max() < 1e-6


# ----------------------------------------------------------------------------- boundary
def _header_functions():
    src = open(os.path.join(ROOT, "include", "espnet_mi355.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(esp_\w+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from espnet_slurp_amd import _native
    lib_path = _native.LIB_PATH
    if not os.path.exists(lib_path):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = _native.load()  # loads without a GPU
    names = _header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_native.SIGNATURES), set(names) ^ set(_native.SIGNATURES)
    assert lib.esp_abi_version() == _native.ABI_VERSION


def test_workspace_size_queries():
    """esp_*_workspace_bytes (host arithmetic, no device call): the sizes the launchers check
    against, from the same code that picks their chunking."""
    from espnet_slurp_amd import _native
    W = _native.workspace_bytes
    M = 128 * 374
    bn = W("esp_bn_swish_fwd", M, 256)
    assert bn % (8 * 256) == 0 and 1 <= bn // (8 * 256) <= 1536      # <= BN_CHUNKS partial rows
    assert W("esp_bn_swish_bwd", M, 256) == 2 * bn
    assert W("esp_layernorm_bwd", M, 256) == 4 * 2 * 256 * ((M + 31) // 32)
    assert W("esp_colsum", 100, 7) == 4 * 7 * 4
    assert W("esp_ctc_loss", 128, 374, 40) == 8 * 2 * 128 * 374 * 81
    assert W("esp_conv2_dgrad", 256) == (4 + 6) * 9 * 256 * 256  # class weights + their bf16 split planes
    assert W("esp_grad_norm", 10 ** 8) == 8 * 1024
    assert W("esp_dwconv1d_wgrad", 128, 374, 256, 31) == 4 * 128 * ((374 + 63) // 64) * 256 * 31
    assert W("esp_relpos_dp", 128, 4, 374) == 4 * 4 * 16 * (2 * 374 - 1) * 64
    assert W("esp_conv1_wgrad", 128, 1500, 80, 256) == 4 * ((128 * 749 * 39 + 2047) // 2048) * 256 * 10
    for name in ("esp_bn_swish_fwd", "esp_layernorm_bwd", "esp_colsum"):
        assert W(name, 0, 256) == 0


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "espnet_slurp_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith(".py"):
                tree = ast.parse(open(os.path.join(dp, f)).read())
                for node in ast.walk(tree):
                    mods = []
                    if isinstance(node, ast.Import):
                        mods = [a.name for a in node.names]
                    elif isinstance(node, ast.ImportFrom):
                        mods = [node.module or ""]
                    for m in mods:
                        assert not m.startswith("oracle"), (f, m)
                        assert "reference" not in m, (f, m)


def _build_cpu(cfg):
    from tests.helpers import build_model
    return build_model(cfg, torch.device("cpu"))


@pytest.mark.parametrize("cfg_fn", [lambda: small_cfg("latest"), lambda: small_cfg("legacy"), c1_cfg,
                                    lambda: c2_cfg("latest", blocks=2)])
def test_state_dict_keys_match_reference(cfg_fn):
    cfg = cfg_fn()
    m = _build_cpu(cfg)
    sd = m.state_dict()
    ps = O.param_shapes(cfg)
    assert set(sd) == set(ps), set(sd) ^ set(ps)
    for k, shp in ps.items():
        assert tuple(sd[k].shape) == tuple(shp), k
    # round trip: the seeded reference-layout state_dict loads strictly
    m.load_state_dict(O.deterministic_params(cfg, 0), strict=True)


def test_flat_parameters_views_and_qkv_adjacency():
    m = _build_cpu(small_cfg("latest"))
    f = m.flat
    for _, p in f.params:
        assert p.data_ptr() == f.view(p).data_ptr()
        assert p.grad is not None and p.grad.data_ptr() == f.gview(p).data_ptr()
    att = m.encoder.encoders[0].self_attn
    w, b = att._wqkv()
    assert torch.equal(w[:64], att.linear_q.weight) and torch.equal(w[128:], att.linear_v.weight)
    m.load_state_dict(O.deterministic_params(small_cfg("latest"), 1))
    assert torch.equal(f.view(att.linear_k.weight), att.linear_k.weight)
    # every slot starts 8-float aligned (the whole-flat bf16 copy / planes keep each weight 16-B
    # aligned, kernels._flat_view) and the flat length is a multiple of 8
    assert all(o % 8 == 0 for o, _ in f.slots.values()) and f.numel % 8 == 0


def test_subsampled_lengths_and_sos_eos():
    from espnet_slurp_amd.asr.encoder.abs_encoder import subsampled_lengths
    from espnet_slurp_amd.asr.espnet_model import add_sos_eos
    for T in (7, 8, 9, 64, 120, 1499, 1500):
        lens = torch.tensor(sorted({T, max(1, T - 1), max(1, T // 2), 7, 1, 2, 3}))
        lens = lens[lens <= T]
        ref = O.subsampled_lengths(lens, T)
        assert torch.equal(subsampled_lengths(lens, T), ref), T
    for T in (11, 12, 13, 17, 64, 120, 1499, 1500):  # conv2d6: mask[:, :, :-2:2][:, :, :-4:3]
        lens = torch.tensor(sorted({T, max(1, T - 1), max(1, T // 2), 11, 7, 1, 2, 3, 5}))
        lens = lens[lens <= T]
        ref = O.subsampled_lengths(lens, T, "conv2d6")
        assert torch.equal(subsampled_lengths(lens, T, "conv2d6"), ref), T
        from espnet_slurp_amd.blocks import Conv2dSubsampling6
        assert Conv2dSubsampling6.out_frames(T) == int(ref.max()), T  # lens holds T: the full length
    ys = torch.tensor([[5, 6, 7, -1], [8, -1, -1, -1], [1, 2, 3, 4]])
    yi, yo, yl = add_sos_eos(ys, torch.tensor([3, 1, 4]), 9, 9, -1)
    ri, ro = O.add_sos_eos(ys, 9, 9, -1)
    assert torch.equal(yi, ri) and torch.equal(yo, ro) and yl.tolist() == [4, 2, 5]


def test_pos_tables_match_oracle():
    from espnet_slurp_amd.asr.encoder.abs_encoder import pos_table
    for T in (1, 29, 374):
        assert torch.equal(pos_table("latest", T, 64, "cpu"), O.rel_pos_table_latest(T, 64)[0])
        assert torch.equal(pos_table("legacy", T, 64, "cpu"), O.rel_pos_table_legacy(T, 64)[0])
        assert torch.equal(pos_table("abs", T, 64, "cpu"), O.abs_pos_table(T, 64)[0])


def test_warmup_lr_and_specaug_draws():
    from espnet_slurp_amd.asr.specaug.specaug import SpecAug
    from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1e-3)
    s = WarmupLR(opt, 100)
    for step in range(1, 300):
        exp = 1e-3 * 100 ** 0.5 * min(step ** -0.5, step * 100 ** -1.5)
        assert abs(opt.param_groups[0]["lr"] - exp) < 1e-15
        opt.step()
        s.step()
    sa = SpecAug(time_warp_window=5, freq_mask_width_range=(0, 30), num_freq_mask=2,
                 time_mask_width_range=(0, 40), num_time_mask=2)
    torch.manual_seed(3)
    d = sa.draw(4, 1500, 80, [1500] * 4)
    w = d["warp"]
    assert (w[:, 0] == w[0, 0]).all() and 5 <= int(w[0, 0]) < 1495
    assert abs(int(w[0, 1]) - int(w[0, 0])) <= 5
    assert d["fmask"].shape == (4, 2, 2) and int(d["fmask"][..., 1].max()) < 30
    d2 = sa.draw(3, 1500, 80, [1500, 1200, 9])
    assert int(d2["warp"][2, 0]) == 0  # too short to warp (t - window <= window)


# ----------------------------------------------------------------------------- distributed (gloo)
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dist_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok1 = ok2 = False
    try:
        from espnet_slurp_amd.flat import FlatParams
        from espnet_slurp_amd.train.distributed import FlatGradReducer, fused_stats_allreduce
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.Linear(64, 32), torch.nn.Linear(32, 8))
        f = FlatParams(m, torch.device("cpu"))
        red = FlatGradReducer(m, f, bucket_mb=0.005)
        assert len(red.buckets) >= 2
        f.grad.copy_(torch.arange(f.numel, dtype=torch.float32) * (rank + 1))
        red.module_done(m[2])
        red.module_done(m[1])
        red.finish()
        exp = torch.arange(f.numel, dtype=torch.float32) * (1 + 2) / 2
        ok1 = torch.allclose(f.grad, exp)
        stats = {"loss": torch.tensor([1.0 + rank]), "acc": torch.tensor([0.5 * rank])}
        avg, tot = fused_stats_allreduce(stats, torch.tensor([2 + rank]))
        ok2 = abs(tot.item() - 5.0) < 1e-6 and abs(avg["loss"].item() - (1 * 2 + 2 * 3) / 5) < 1e-6
    except Exception as e:  # report instead of hanging the parent
        print("worker", rank, "failed:", repr(e))
    finally:
        q.put((rank, ok1, ok2))
        dist.destroy_process_group()


def test_flat_grad_reducer_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r[0] for r in res) == [0, 1]
    assert all(r[1] and r[2] for r in res), res


def _stop_worker(rank, world, port, q):
    """Trainer._stop_aligned (iterator_stop, trainer.py:505-510): exact lengths on every rank
    -> counted stop at the shortest; any rank without an exact length -> the per-batch flag."""
    import types

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    try:
        from espnet_slurp_amd.train.trainer import Trainer
        fake = types.SimpleNamespace(distributed=True,
                                     model=types.SimpleNamespace(flat=types.SimpleNamespace(flat=torch.zeros(1))))

        class Hint(list):  # a len() that is only a hint: the iterator yields fewer items
            exact_len = False

            def __len__(self):
                return 10

        cases = [list(range(3 + 2 * rank)),                        # exact: 3 vs 5 -> 3
                 list(range(4)) if rank == 0 else iter(range(2)),  # rank 1 has no len() -> 2
                 Hint(range(2)) if rank == 1 else list(range(6))]  # rank 1 hints 10, yields 2 -> 2
        for it in cases:
            out.append(len(list(Trainer._stop_aligned(fake, it))))
    except Exception as e:  # report instead of hanging the parent
        print("worker", rank, "failed:", repr(e))
    finally:
        q.put((rank, out))
        dist.destroy_process_group()


def test_stop_aligned_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stop_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == [3, 2, 2] for r in res), res


# ----------------------------------------------------------------------------- front end (§8(f) rank 1)
def _frontend_golden():
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "frontend.npz"))


def test_frontend_oracle_vs_reference_golden():
    """oracle/frontend_cpu.py restates Stft / LogMel.forward / GlobalMVN; the fixture was produced
    by the reference modules themselves (tests/golden/make_golden.py frontend)."""
    from oracle import frontend_cpu as FE
    g = _frontend_golden()
    x, lens = torch.from_numpy(g["x"]), torch.from_numpy(g["lens"])
    spec, olens = FE.stft(x, lens, 512, 128)
    assert torch.equal(olens, torch.from_numpy(g["olens"]))
    assert float((spec - torch.from_numpy(g["spec"])).abs().max()) < 1e-5
    power = spec[..., 0] ** 2 + spec[..., 1] ** 2
    feats = FE.log_mel(power, olens, torch.from_numpy(g["melmat"]))
    assert float((feats - torch.from_numpy(g["feats"])).abs().max()) < 1e-5
    stats = {"count": g["stat_count"], "sum": g["stat_sum"], "sum_square": g["stat_sum_square"]}
    mean, std = FE.global_mvn_stats(stats)
    normed = FE.global_mvn(torch.from_numpy(g["feats"]), olens, mean, std)
    assert float((normed - torch.from_numpy(g["normed"])).abs().max()) < 1e-5
    # the fixture's mel matrix is the oracle's restated librosa Slaney filterbank (parity unpinned:
    # librosa is absent and the reference holds no mel fixture)
    assert np.array_equal(FE.mel_filters(16000, 512, 80, 0.0, 8000.0).T, g["melmat"])


def test_frontend_mel_restatements_agree():
    """The product's filterbank (asr/frontend/default.py) and the oracle's, written separately
    from librosa's published algorithm, agree (Slaney and HTK scales, band edges)."""
    from espnet_slurp_amd.asr.frontend.default import mel_filters
    from oracle import frontend_cpu as FE
    for args in ((16000, 512, 80, 0.0, 8000.0, False), (16000, 400, 40, 20.0, 7600.0, False),
                 (8000, 256, 23, 0.0, 4000.0, True)):
        a, b = mel_filters(*args), FE.mel_filters(*args)
        assert a.dtype == b.dtype == np.float32 and a.shape == b.shape
        assert np.allclose(a, b, rtol=1e-6, atol=1e-9), args


def test_frontend_and_global_mvn_state_dict_keys(tmp_path):
    from espnet_slurp_amd.asr.frontend.default import DefaultFrontend
    from espnet_slurp_amd.layers.global_mvn import GlobalMVN
    fe = DefaultFrontend()
    assert list(fe.state_dict()) == ["logmel.melmat"] and fe.state_dict()["logmel.melmat"].shape == (257, 80)
    assert fe.output_size() == 80 and fe.num_frames(3000) == 24
    p = tmp_path / "feats_stats.npz"
    np.savez(p, count=np.float64(10.0), sum=np.ones(80), sum_square=np.full(80, 2.0))
    gm = GlobalMVN(p)
    assert sorted(gm.state_dict()) == ["mean", "std"]
    assert np.allclose(gm.mean.numpy(), 0.1) and np.allclose(gm.std.numpy(), np.sqrt(0.2 - 0.01))
