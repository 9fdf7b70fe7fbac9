"""Bench-workload fixture (VERDICT r2 "next" 1): the C2 training step at the bench's own shape.

    python tests/golden/make_bench_fixture.py            # writes tests/golden/bench_c2_b128.npz

C2 Conformer (d=256, H=4, FF 1024, 12 blocks, latest rel-pos; decoder 6 x FF 2048; V=600)
at B=128 x 1500 frames -- bench.py's default workload -- with dropout 0 and SpecAug off, run
through the ORACLE restatement (oracle/espnet_cpu.py) in fp32 AND fp64.  The reference itself
cannot produce this fixture here: at B=128 its fp32 autograd graph needs ~75 GB and its fp64
one ~130 GB, over this container's 64 GB; the oracle runs on the GPU box's host (16 threads,
~4 min, ~130 GB peak), which is where this script is meant to run.  The oracle is pinned to
the reference at this exact model shape (tests/golden/fullsize_c2_grad_{latest,legacy}.npz,
B=2: since round 6 their generator, make_golden.fullsize_train_fixture, runs the oracle's fp64 step on the
same inputs and asserts its loss and EVERY parameter gradient equal the reference's fp64 ones to fp64
rounding before writing; until round 5 it checked nothing of the kind); what B=128 adds is the batch-coupled part
(BatchNorm statistics over B*T' = 47,872 frames, the 1/B loss normalisation) and, on the GPU
side, every shape-dependent code path of the bench (split-K counts, persistent-grid wrap,
implicit-im2col index ranges, attention grids with z = 512).

Stored: the seed, lengths and target lengths (the inputs are regenerated from the seed by
O.synthetic_batch), loss / loss_ctc / loss_att / acc, and per parameter the gradient L2
norm, max |g|, a fixed slice of elements and the whole-tensor fingerprint (fingerprint.py: 8 fp64
projections, per-row norms), for both precisions, plus the ReLU flip records of
conv.0 and the decoder norm3 slices (flipfix.py) (the format of make_golden.fullsize_train_fixture,
read by tests/helpers.grad_gate / loss_gate).
Test infrastructure only: never imported by the product.
"""
import gc
import os
import sys
import time
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import espnet_cpu as O  # noqa: E402

sys.path.insert(0, HERE)
import fingerprint as FP  # noqa: E402
import flipfix  # noqa: E402

B, T, V, SEED = 128, 1500, 600, 71
N_SLICE = 16


def bench_cfg():
    return O.ModelCfg(vocab_size=V,
                      enc=O.EncCfg(output_size=256, attention_heads=4, linear_units=1024, num_blocks=12,
                                   rel_pos_type="latest", dropout_rate=0.0, positional_dropout_rate=0.0,
                                   attention_dropout_rate=0.0),
                      dec=O.DecCfg(attention_heads=4, linear_units=2048, num_blocks=6))


def bench_lengths():
    """bench.py synthetic_batch shape: every utterance 1500 frames, targets U[20, 40]."""
    rng = np.random.Generator(np.random.PCG64(SEED + 1000))
    return [T] * B, [int(u) for u in rng.integers(20, 41, size=B)]


def slice_indices(name: str, numel: int) -> np.ndarray:
    """Same rule as make_golden.slice_indices: first 4, last 4, 8 seeded by the name."""
    if numel <= N_SLICE:
        return np.arange(numel, dtype=np.int64)
    rng = np.random.Generator(np.random.PCG64(zlib.crc32(name.encode())))
    idx = np.concatenate([np.arange(4), np.arange(numel - 4, numel), rng.integers(4, numel - 4, size=N_SLICE - 8)])
    return idx.astype(np.int64)


def run(dt, tag, out, recs, rows, shapes):
    cfg = bench_cfg()
    lens, ulens = bench_lengths()
    P = {k: v.requires_grad_(v.is_floating_point() and "running" not in k)
         for k, v in O.deterministic_params(cfg, SEED, dt).items()}
    speech, slen, text, tlen = O.synthetic_batch(B, T, 80, V, lens, ulens, SEED + 1)
    t0 = time.time()
    # the ReLU decisions near 0 (Conv2dSubsampling, decoder FFNs) and their slice contributions
    with flipfix.OracleProbe(O, P) as probe:
        loss, stats, _ = O.asr_forward(P, speech.to(dt), slen, text, tlen, cfg, bn_state={})
    print(f"{tag}: forward {time.time() - t0:.1f} s, loss {loss.item():.8f}", flush=True)
    t0 = time.time()
    loss.backward()
    print(f"{tag}: backward {time.time() - t0:.1f} s", flush=True)
    recs[tag] = probe.rec.detach()
    out[f"loss_{tag}"] = np.float64(loss.item())
    for k in ("loss_ctc", "loss_att", "acc"):
        out[f"{k}_{tag}"] = np.float64(float(stats[k]))
    for n, p in P.items():
        if p.grad is None:
            continue
        g = p.grad.detach().double().reshape(-1)
        idx = slice_indices(n, g.numel())
        out[f"gn_{tag}/{n}"] = np.float64(g.norm().item())
        out[f"gmax_{tag}/{n}"] = np.float64(g.abs().max().item())
        out[f"gidx/{n}"] = idx
        out[f"gs_{tag}/{n}"] = g[torch.from_numpy(idx)].numpy()
        FP.summarize(n, p.grad.detach(), tag, out, rows)
        shapes[n] = g.numel()


def main():
    n = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 8)
    torch.set_num_threads(n)
    print(f"bench fixture: B={B} T={T} on {n} threads", flush=True)
    out = {}
    recs = {}
    rows = {}
    shapes = {}
    run(torch.float32, "f32", out, recs, rows, shapes)
    gc.collect()
    run(torch.float64, "f64", out, recs, rows, shapes)
    gc.collect()
    FP.finish_rows(out, rows)
    gs32 = {k[len("gs_f32/"):]: v for k, v in out.items() if k.startswith("gs_f32/")}
    flipfix.flip_records(recs["f64"], recs["f32"], lambda n: out["gidx/" + n], out, gs32,
                         log=lambda m: print(m, flush=True), shapes=shapes)
    del recs
    gc.collect()
    lens, ulens = bench_lengths()
    out.update(lens=np.array(lens), ulens=np.array(ulens), seed=np.int64(SEED), B=np.int64(B), T=np.int64(T))
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "bench_c2_b128.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, flush=True)


if __name__ == "__main__":
    main()
