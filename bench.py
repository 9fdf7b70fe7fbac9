#!/usr/bin/env python3
"""Benchmark: utterances/sec of the full ESPnet2 Conformer CTC/attention training step.

    python bench.py [--gpus N --steps K --warmup W --batch B]
    (N>1: either launched by the caller, python -m torch.distributed.run --nproc-per-node N ...
    bench.py --gpus N ..., or started plainly: bench.py then launches the N ranks itself, one
    process per GPU over RCCL, as espnet2/tasks/abs_task.py:1049-1070 spawns its DDP workers)

Workload (BASELINE.json configs[1]): 80-dim fbank x 1500 frames,
Conformer encoder d=256, 4 heads, FF 1024, 12 blocks (macaron, rel-pos latest, cnn k=31),
Transformer decoder 6 x (4 heads, FF 2048), V=600, ctc_weight 0.3, lsm 0.1, dropout 0.1
everywhere (SLURP YAML), SpecAug on (time warp 5, 2 freq masks <30, 2 time masks <40),
UtteranceMVN, Adam + WarmupLR(25k) + grad clip 5.  A step = fwd + bwd + RCCL grad average
(N>1) + clip + Adam + LR step, on a resident synthetic batch per GPU (weak scaling).
Prints ONE JSON line (rank 0) with the roofline of the dominant kernel family (the MFMA
GEMM) measured live with HIP events, and a CPU baseline (the oracle restatement timed on
the host cores, rank 0 at N=1 only).
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: bf16 dense MFMA (no sparsity)
# BASELINE.json configs by name: (d, heads, ff, encoder blocks, bf16 GEMMs)
PRESETS = {"c2": (256, 4, 1024, 12, False), "c4": (512, 8, 2048, 17, False), "c5": (512, 8, 2048, 12, True)}
HBM_PEAK_GBS = 8000.0


def conformer_flops_per_utt(D, H, FF, L_enc, FF_dec, L_dec, V, T=1500, F=80, U1=41):
    """Algorithmic forward FLOPs per utterance (SURVEY.md §8(d) formula, 2 FLOP/MAC)."""
    T1, F1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
    Tp, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
    conv1 = 2 * 9 * D * T1 * F1
    embed = conv1 + 2 * 9 * D * D * Tp * F2 + 2 * Tp * F2 * D * D
    blk = (8 * Tp * D * FF + 8 * Tp * D * D + 2 * (2 * Tp - 1) * D * D + 2 * Tp * Tp * D
           + 2 * Tp * (2 * Tp - 1) * D + 2 * Tp * Tp * D + 4 * Tp * D * D + 2 * Tp * D * 31 + 2 * Tp * D * D)
    dec = L_dec * (8 * U1 * D * D + 4 * U1 * D * D + 4 * Tp * D * D + 4 * U1 * D * FF_dec + 4 * U1 * U1 * D
                   + 4 * U1 * Tp * D) + 2 * U1 * D * V
    ctc = 2 * Tp * D * V
    fwd = embed + L_enc * blk + dec + ctc
    return fwd, 3 * fwd - conv1


def build(args, device):
    from espnet_slurp_amd.asr.ctc import CTC
    from espnet_slurp_amd.asr.decoder.transformer_decoder import TransformerDecoder
    from espnet_slurp_amd.asr.encoder.conformer_encoder import ConformerEncoder
    from espnet_slurp_amd.asr.espnet_model import ESPnetASRModel
    from espnet_slurp_amd.asr.specaug.specaug import SpecAug
    from espnet_slurp_amd.layers.utterance_mvn import UtteranceMVN
    V = args.vocab
    tokens = ["<blank>", "<unk>"] + [f"t{i}" for i in range(V - 3)] + ["<sos/eos>"]
    enc = ConformerEncoder(input_size=80, output_size=args.d, attention_heads=args.heads, linear_units=args.ff,
                           num_blocks=args.layers, dropout_rate=0.1, positional_dropout_rate=0.1,
                           attention_dropout_rate=0.1, input_layer="conv2d", normalize_before=True,
                           macaron_style=True, rel_pos_type=args.rel_pos, pos_enc_layer_type="rel_pos",
                           selfattention_layer_type="rel_selfattn", activation_type="swish", use_cnn_module=True,
                           cnn_module_kernel=31)
    dec = TransformerDecoder(vocab_size=V, encoder_output_size=args.d, attention_heads=args.heads,
                             linear_units=2048, num_blocks=6, dropout_rate=0.1, positional_dropout_rate=0.1,
                             self_attention_dropout_rate=0.1, src_attention_dropout_rate=0.1)
    specaug = SpecAug(apply_time_warp=True, time_warp_window=5, time_warp_mode="bicubic", apply_freq_mask=True,
                      freq_mask_width_range=[0, 30], num_freq_mask=2, apply_time_mask=True,
                      time_mask_width_range=[0, 40], num_time_mask=2)
    model = ESPnetASRModel(vocab_size=V, token_list=tokens, frontend=None, specaug=specaug,
                           normalize=UtteranceMVN(), preencoder=None, encoder=enc, postencoder=None, decoder=dec,
                           ctc=CTC(V, args.d), joint_network=None, ctc_weight=0.3, lsm_weight=0.1,
                           length_normalized_loss=False)
    model = model.to(device)
    model.flatten()
    return model


def synthetic_batch(B, V, rank, device, variable=False, index=0):
    """SURVEY §8(d) synthetic inputs: N(0,1) fbank, lengths 1500 (or U[1000,1500] sorted
    descending with variable=True: each batch padded to its own longest utterance, as the
    reference's collate does), tokens U[2, V-2], label lengths U[20,40] padded -1."""
    g = torch.Generator().manual_seed(1234 + rank + 7919 * index)
    speech_lengths = torch.full((B,), 1500, dtype=torch.long)
    if variable:
        speech_lengths = torch.sort(torch.randint(1000, 1501, (B,), generator=g), descending=True)[0]
    speech = torch.randn(B, int(speech_lengths.max()), 80, generator=g).to(device)
    tl = torch.randint(20, 41, (B,), generator=g)
    text = torch.full((B, int(tl.max())), -1, dtype=torch.long)
    for i in range(B):
        text[i, : tl[i]] = torch.randint(2, V - 1, (int(tl[i]),), generator=g)
    return dict(speech=speech, speech_lengths=speech_lengths, text=text, text_lengths=tl)


def host_cores() -> int:
    """Every core this process may run on (its affinity set), capped by OMP_NUM_THREADS when the
    host sets it: the GPU box exports the per-GPU CPU share there (16), while os.cpu_count()
    reports the whole machine."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else max(1, n)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args):
    """The oracle (plain PyTorch CPU restatement, oracle/espnet_cpu.py) timed on the host
    cores: same C2 model shape, fp32, B=4 x 1500 frames, dropout 0.1, SpecAug on with the GPU step's
    configuration (time warp window 5, 2 frequency masks of width [0, 30), 2 time masks of width [0, 40);
    fresh draws every step, mask_along_axis.py:32-44 / time_warp.py:25-27), 1 warmup + 3 timed steps of
    fwd + bwd + clip + torch Adam -- the same step the GPU times."""
    from oracle import espnet_cpu as O
    n = host_cores()
    torch.set_num_threads(n)
    cfg = O.ModelCfg(vocab_size=args.vocab, enc=O.EncCfg(output_size=args.d, attention_heads=args.heads,
                                                          linear_units=args.ff, num_blocks=args.layers,
                                                          dropout_rate=0.1, positional_dropout_rate=0.1,
                                                          attention_dropout_rate=0.1, rel_pos_type=args.rel_pos),
                     dec=O.DecCfg(attention_heads=args.heads, linear_units=2048, num_blocks=6, dropout_rate=0.1,
                                  positional_dropout_rate=0.1, self_attention_dropout_rate=0.1,
                                  src_attention_dropout_rate=0.1))
    P = {k: v.requires_grad_(v.is_floating_point() and "running" not in k)
         for k, v in O.deterministic_params(cfg, 0).items()}
    params = [v for v in P.values() if v.requires_grad]
    opt = torch.optim.Adam(params, lr=2e-4)
    B = 4
    speech, slen, text, tlen = O.synthetic_batch(B, 1500, 80, args.vocab, [1500] * B, [40, 33, 27, 20], 7)
    bn = {}
    times = []
    gen = torch.Generator().manual_seed(11)

    def specaug_draws(T, F):
        center = int(torch.randint(5, T - 5, (1,), generator=gen)[0])
        warped = int(torch.randint(center - 5, center + 5, (1,), generator=gen)[0]) + 1
        d = {"center": center, "warped": warped}
        for key, D, hi in (("freq", F, 30), ("time", T, 40)):
            ml = torch.randint(0, hi, (B, 2), generator=gen)
            d[key + "_len"] = ml
            d[key + "_pos"] = torch.randint(0, max(1, D - int(ml.max())), (B, 2), generator=gen)
        return d

    for it in range(4):
        t0 = time.perf_counter()
        loss, _, _ = O.asr_forward(P, speech, slen, text, tlen, cfg, specaug=specaug_draws(1500, 80), bn_state=bn)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 5.0)
        opt.step()
        opt.zero_grad()
        times.append(time.perf_counter() - t0)
    t = sum(times[1:]) / len(times[1:])
    return {"value": round(B / t, 4), "unit": "utt/s", "cores": n, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"oracle/espnet_cpu.py {workload_name(args).split()[0]}-shape step (fwd+bwd+clip+Adam), "
                      f"d={args.d} {args.layers}L, B=4 x 1500 frames, fp32, SpecAug on, "
                      f"1 warmup + 3 timed steps, {t:.2f} s/step on {n} threads"}


def workload_name(args) -> str:
    """BASELINE.json config name of the shape being run (C2 is the default / headline)."""
    if (args.d, args.heads, args.ff, args.layers) == (256, 4, 1024, 12):
        return "C2 SLURP Conformer-medium"
    if (args.d, args.heads, args.ff, args.layers) == (512, 8, 2048, 17):
        return "C4-shape LibriSpeech Conformer-large (fp32)"
    if (args.d, args.heads, args.ff, args.layers) == (512, 8, 2048, 12):
        return ("C5 SLURP-entity Conformer + SpecAug, bf16 MFMA (fp32 master weights)" if args.amp
                else "C5-shape SLURP-entity Conformer (fp32)")
    return "custom Conformer"


def gemm_algorithmic_bytes(shapes) -> float:
    """Sum over the profiled GEMM launches of the bytes each must move at least once: A, B read,
    C written (fp32), plus the fused epilogue's own M x N streams (residual / pre-activation
    reads, aux writes).  An implicit-im2col operand counts its NHWC source map (~ 4/9 of the
    virtual M x K matrix for the 3x3 / stride-2 convolution)."""
    tot = 0.0
    for key, (n, _ms, _f, extra) in shapes.items():
        ma, mb, M, N, Kd, batch = key[:6]  # (+ a tag for the bf16-operand / score-gradient GEMMs)
        if key[6:] in (("conv2_dgrad",), ("conv2_dgrad_c1fold",)):  # the implicit conv2 input gradient: its entry
            # holds the whole count
            tot += extra
            continue
        a = M * Kd * (4 / 9 if ma >= 2 else 1.0)
        b = N * Kd * (4 / 9 if mb >= 2 else 1.0)
        # bf16-operand GEMMs read 2-byte A and B; B-planes GEMMs ("bp") read B as three bf16 planes,
        # planes GEMMs ("pl") both operands
        ea = 2.0 if key[6:] == ("bf16",) else 6.0 if key[6:] == ("pl",) else 4.0
        eb = 2.0 if key[6:] == ("bf16",) else 6.0 if key[6:] in (("bp",), ("pl",)) else 4.0
        tot += n * batch * (ea * a + eb * b + 4.0 * M * N) + extra
    return tot


def measured_gemm_traffic(args) -> dict:
    """HBM bytes per launch of the GEMM family from the newest committed PMC measurement
    (profiles/*_gemm_traffic.json, written by tools/pmc_traffic.py from two rocprofv3 --pmc
    passes of this bench); {} when none is present."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                          "*_gemm_traffic.json")))
    for f in reversed(files):  # newest measurement of THIS workload (batch, model shape, precision)
        d = json.load(open(f))
        shape = (d.get("d", 256), d.get("layers", 12), bool(d.get("amp", False)))
        if d.get("batch") == args.batch and shape == (args.d, args.layers, bool(args.amp)):
            d["source"] = os.path.relpath(f, os.path.dirname(os.path.abspath(__file__)))
            return d
    return {}


def host_utterances(B, V, rank, index=0):
    """The synthetic batch as the data feed sees it: per-utterance host arrays (uid, {"speech": (T, 80)
    float32, "text": (L,) int64}), collated per step by CommonCollateFn (collate_fn.py:10-37)."""
    b = synthetic_batch(B, V, rank, "cpu", index=index)
    out = []
    for i in range(B):
        n, u = int(b["speech_lengths"][i]), int(b["text_lengths"][i])
        out.append((f"utt{i}", {"speech": b["speech"][i, :n].numpy(), "text": b["text"][i, :u].numpy()}))
    return out


def data_feed_rate(trainer, utts, steps, world):
    """utt/s of the step fed by the data path: every step collates the host
    utterances into pinned buffers (CommonCollateFn, pin_memory) and DevicePrefetcher copies them on a
    side stream during the previous step (trainer.py:514's to_device), into the same graph replay.
    Reported beside `value`, which is the resident-batch rate of the timed region."""
    from espnet_slurp_amd.iterators.sequence_iter_factory import DevicePrefetcher
    from espnet_slurp_amd.train.collate_fn import CommonCollateFn
    collate = CommonCollateFn(float_pad_value=0.0, int_pad_value=-1, pin_memory=True)
    device = torch.device("cuda", torch.cuda.current_device())
    feed = DevicePrefetcher((collate(utts) for _ in range(steps + 1)), device)
    _, batch = next(feed)  # one untimed step: the first collate / copy
    trainer.train_one_step(batch)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        _, batch = next(feed)
        trainer.train_one_step(batch)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return world * len(utts) * steps / float(el.item())


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch(argv, gpus, env, port=None):
    """How this invocation runs (decided before anything touches the GPU).  Returns None to run the
    bench in this process (a single GPU, or one rank of a launcher that set WORLD_SIZE), or the
    command that starts `gpus` ranks on this node -- torch.distributed.run, one process per GPU,
    rendezvous on 127.0.0.1 -- whose exit status this process then returns.  A launcher whose
    WORLD_SIZE differs from --gpus is an error (the line would report the wrong n_gpus)."""
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher's WORLD_SIZE is {world}")
        return None
    if gpus <= 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port or free_port()}",
            os.path.abspath(__file__)] + list(argv)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # B per GPU ("tune; report B"): measured at C2 64 -> 848, 96 -> 875, 128 -> 906,
    # 192 -> 917, 256 -> 932 utt/s in round 1 (profiles/r01g_batch_sweep.txt); at the round-4 HEAD on one
    # box 128 -> 1299, 192 -> 1297, 256 -> 1342 (profiles/r04i_batch_sweep.txt).  Round 6: 384 (8-GPU global
    # batch 3072): 1471.4 / 1477.8 vs 1461.9 / 1464.3 utt/s at 256, alternating on one box, 211 GiB peak HBM on
    # the 1-GPU and the DP path (profiles/r06q_*); tests/test_gpu_bench_shape.py checks B=128 against the
    # oracle and B=256 / B=384 against B=128
    ap.add_argument("--batch", type=int, default=384, help="utterances per GPU")
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--heads", type=int, default=4)
    ap.add_argument("--ff", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--vocab", type=int, default=600)
    ap.add_argument("--rel-pos", default="latest", choices=["latest", "legacy"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--feed-steps", type=int, default=5,
                    help="steps of the data-feed rate (per-step collate + side-stream H2D; 0: skip)")
    ap.add_argument("--eager", action="store_true", help="launch kernel by kernel instead of replaying a HIP graph")
    ap.add_argument("--variable-lengths", action="store_true",
                    help="speech lengths U[1000,1500] sorted descending (SURVEY 8(d) variable variant): "
                         "4 batches of different lengths in turn, on length-bucketed HIP graphs")
    ap.add_argument("--graph-buckets", default="100,8",
                    help="frames,tokens bucket multiples of TrainerOptions.graph_buckets (--variable-lengths)")
    ap.add_argument("--amp", action="store_true", help="bf16 GEMM operands, fp32 accumulate (TrainerOptions.use_amp)")
    ap.add_argument("--dp-world1", action="store_true",
                    help="N=1 through the data-parallel path (a 1-rank RCCL group: segmented-graph capture, bucket "
                         "all-reduces) -- the per-rank HBM and step of the N-GPU job, measurable on one GPU")
    ap.add_argument("--config", choices=sorted(PRESETS), default=None,
                    help="BASELINE.json config preset (overrides --d/--heads/--ff/--layers; c5 implies --amp)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    cmd = rank_launch(sys.argv[1:], args.gpus, os.environ)
    if cmd is not None:
        # the N ranks as child processes (this process has not touched the GPU: counting devices
        # does not initialise it on this image)
        have = torch.cuda.device_count()
        if have < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but {have} GPU(s) visible")
        import subprocess
        sys.exit(subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode)
    if args.config:
        args.d, args.heads, args.ff, args.layers, amp = PRESETS[args.config]
        args.amp = args.amp or amp

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dp = world > 1 or args.dp_world1
    if dp:
        # enough RCCL channels that a ring uses all 7 xGMI links of each GPU
        os.environ.setdefault("NCCL_MIN_NCHANNELS", "8")
        if world == 1:  # --dp-world1: a 1-rank group of this process
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            dist.init_process_group("nccl", rank=0, world_size=1)
        else:
            dist.init_process_group("nccl")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    torch.manual_seed(0)

    from espnet_slurp_amd import kernels as K
    from espnet_slurp_amd.optimizers.fused_adam import FusedAdam
    from espnet_slurp_amd.schedulers.warmup_lr import WarmupLR
    from espnet_slurp_amd.train.trainer import Trainer, TrainerOptions

    model = build(args, device)
    model.train()
    opt = FusedAdam(model.parameters(), model.flat, lr=2e-4)
    sched = WarmupLR(opt, warmup_steps=25000)
    buckets = tuple(int(v) for v in args.graph_buckets.split(",")) if args.variable_lengths else None
    trainer = Trainer(model, opt, sched, TrainerOptions(grad_clip=5.0, use_amp=args.amp, graph_buckets=buckets),
                      distributed=dp, cuda_graph=not args.eager)
    batches = [synthetic_batch(args.batch, args.vocab, rank, device, args.variable_lengths, i)
               for i in range(4 if args.variable_lengths else 1)]
    batch = batches[0]

    for i in range(args.warmup):
        trainer.train_one_step(batches[i % len(batches)])
    torch.cuda.synchronize()

    if args.eager:
        K.profile_gemm_start()
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        stats = trainer.train_one_step(batches[i % len(batches)])
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the timed steps must have trained: the last step's loss and gradient norm are finite and
    # no optimizer step was skipped (read after the timed region: no host sync inside it)
    last_loss, last_gn = float(stats["loss"].item()), float(stats["grad_norm"].item())
    trainer.resolve_pending()
    trainer.sync_host_state()
    if not (math.isfinite(last_loss) and math.isfinite(last_gn)) or trainer.n_skipped:
        print(json.dumps({"error": "non-finite training step", "loss": last_loss, "grad_norm": last_gn,
                          "skipped_steps": trainer.n_skipped}), flush=True)
        sys.exit(3)
    feed_value = None
    if args.feed_steps > 0 and not args.variable_lengths:
        feed_value = data_feed_rate(trainer, host_utterances(args.batch, args.vocab, rank), args.feed_steps, world)
        trainer.resolve_pending()
        trainer.sync_host_state()
    if not args.eager:
        # the graph's kernels cannot be bracketed one by one: time the same GEMM launches (same
        # kernels, shapes and inputs) in one eager step right after the timed region
        eager = Trainer(model, opt, sched, TrainerOptions(grad_clip=5.0, use_amp=args.amp), distributed=dp)
        torch.cuda.synchronize()
        # hold the GPU for ~200 ms so the host enqueues the whole eager step (~1,500 launches)
        # before the first GEMM runs: each event pair then brackets its kernel back to back,
        # not the host's launch latency (which made the eager-replay figure box-dependent)
        torch.cuda._sleep(int(5e8))
        K.profile_gemm_start()
        eager.train_one_step(batch)
        eager.resolve_pending()
    gemm_flops, gemm_ms, gemm_launches, gemm_shapes = K.profile_gemm_stop(by_shape=True)
    attn_flops, attn_bytes, attn_ms, attn_launches = K.profile_attn_stop()

    el = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if dp:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    # peak HBM this rank reserved (the caching allocator, graph pools included), max over ranks
    peak = torch.tensor([torch.cuda.max_memory_reserved(device) / 2 ** 30], dtype=torch.float64, device=device)
    if dp:
        dist.all_reduce(peak, op=dist.ReduceOp.MAX)
    hbm_peak_gib = round(float(peak.item()), 1)

    if rank == 0:
        traffic = measured_gemm_traffic(args)
        fwd, train = conformer_flops_per_utt(args.d, args.heads, args.ff, args.layers, 2048, 6, args.vocab)
        value = world * args.batch * args.steps / elapsed
        achieved = gemm_flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else 0.0
        # fp32 GEMMs of a split build (esp_f32_gemm_products() == 6) issue six bf16 MFMA products
        # per fp32 product: their ceiling is the bf16 MFMA peak / 6
        from espnet_slurp_amd import _native
        f32_products = _native.load().esp_f32_gemm_products()
        peak = BF16_MFMA_PEAK_TFLOPS if args.amp else (
            round(BF16_MFMA_PEAK_TFLOPS / 6, 2) if f32_products == 6 else FP32_MFMA_PEAK_TFLOPS)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args)
        out = {
            "metric": "utterances/sec (fbank80x1500, Conformer-12L CTC+attn)",
            "value": round(value, 3),
            "unit": "utt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16-mfma/f32-accumulate" if args.amp else "f32",
            "f32_gemm": None if args.amp else (
                "bf16x6 split products on v_mfma_f32_32x32x16_bf16, fp32 accumulate (fp32-accurate: "
                "profiles/r03h_f32_gemm_accuracy.txt)" if f32_products == 6 else "v_mfma_f32_32x32x2_f32"),
            "data": "synthetic (N(0,1) fbank, random tokens U[20,40], random-init weights)",
            "launch": "eager" if args.eager else "hip_graph",
            "graphs_captured": len(trainer._graphs) if not args.eager else 0,
            "dp_path": dp,
            "hbm_peak_gib": hbm_peak_gib,
            "last_step": {"loss": round(last_loss, 4), "grad_norm": round(last_gn, 4),
                          "skipped_steps": trainer.n_skipped},
            "config": {"workload": f"{workload_name(args)} d={args.d} H={args.heads} FF={args.ff} "
                                   f"{args.layers}L enc / 6L dec, V={args.vocab}, rel_pos={args.rel_pos}, "
                                   "ctc 0.3, lsm 0.1, dropout 0.1, SpecAug on"
                                   + (", lengths U[1000,1500]" if args.variable_lengths else ""),
                       "global_batch": world * args.batch, "seq_len": 1500, "parallelism": f"dp{world}"},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                         "f32_mfma_peak_frac": None if args.amp else round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                         "traffic": traffic.get("hbm_bytes_per_launch"),
                         "traffic_source": traffic.get("source"),
                         "algorithmic_bytes_per_launch": round(gemm_algorithmic_bytes(gemm_shapes) / max(1, gemm_launches)),
                         "kernel": ("gemm_glds_kernel<BF16> (bf16 MFMA)" if args.amp else "gemm_glds_kernel")
                                   + " family (all MFMA GEMM launches of one step, HIP events"
                                   + (" in the timed region)" if args.eager else " on an eager replay of the step)"),
                         "launches": gemm_launches,
                         "avg_launch_us": round(1e3 * gemm_ms / max(1, gemm_launches), 2)},
            # the second kernel the round-1 verdict named: rel-pos attention probabilities
            # (algorithmic ac + bd work, 4 T'^2 d_k per head and utterance, no padded tiles; P and
            # its dropout copy written once)
            # peak: the MFMA form the kernel issues -- bf16 operands on the bf16 MFMA in the bf16 mode (the
            # bf16 dense peak), six split products per fp32 product otherwise (the split ceiling, as the GEMMs)
            "attention_roofline": None if not attn_launches else {
                "kernel": "relpos_probs_lds_kernel (esp_relpos_attn_probs), HIP events on the same eager replay",
                "flops_per_launch": round(attn_flops / attn_launches),
                "launches": attn_launches, "avg_launch_us": round(1e3 * attn_ms / attn_launches, 2),
                "achieved": round(attn_flops / (attn_ms * 1e-3) / 1e12, 2), "peak": peak,
                "unit": "TFLOP/s", "frac": round(attn_flops / (attn_ms * 1e-3) / 1e12 / peak, 4),
                "f32_mfma_peak_frac": None if args.amp else round(
                    attn_flops / (attn_ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4),
                "write_GBps": round(attn_bytes / (attn_ms * 1e-3) / 1e9, 1)},
            "step_roofline": {"train_gflop_per_utt": round(train / 1e9, 2),
                              "achieved_tflops": round(value / world * train / 1e12, 2),
                              "frac_of_mfma_peak": round(value / world * train / 1e12 / peak, 4)},
            "cpu_baseline": cpu,
            "data_feed": None if feed_value is None else {
                "value": round(feed_value, 3), "unit": "utt/s", "steps": args.feed_steps,
                "what": "the same step with every batch collated on the host into pinned buffers "
                        "(CommonCollateFn) and copied by DevicePrefetcher on a side stream (not the headline: "
                        "`value` keeps the resident synthetic batch of SURVEY 8(d))"},
        }
        print(json.dumps(out))
    if dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
