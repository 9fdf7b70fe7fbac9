"""Trainer — espnet2/train/trainer.py: the hot loop train_one_epoch (:463-720), its valid
pass validate_one_epoch (:724-772) and the epoch driver run (:154-447).

Per batch: forward (model(**batch)), weighted loss normalisation (:594-608), backward,
bucketed RCCL gradient average (replaces DDP), clip_grad_norm_(grad_clip) on device,
non-finite skip (:651-667), Adam + WarmupLR batch step (:671-686), zero_grad.
Host synchronisation: the finite flag of each optimizer step is read back asynchronously
(the reference reads torch.isfinite(grad_norm) on the host, :651, a sync per step); the
reporter's per-step values are snapshotted on device and read in one copy every
log_interval steps.
"""
from __future__ import annotations

import dataclasses
import logging
import time
from pathlib import Path
from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist

from ..optimizers.fused_adam import FusedAdam, clip_grad_norm_
from ..schedulers.warmup_lr import AbsBatchStepScheduler, AbsEpochStepScheduler, AbsValEpochStepScheduler
from .. import kernels as K
from .distributed import FlatGradReducer, fused_stats_allreduce


@dataclasses.dataclass
class TrainerOptions:
    grad_clip: float = 5.0
    grad_clip_type: float = 2.0
    accum_grad: int = 1
    no_forward_run: bool = False
    log_interval: Optional[int] = None
    # reduced-precision training (trainer.py:181-195,554 offer fp16 autocast + GradScaler under
    # `use_amp`): here every GEMM takes bf16 operands with fp32 accumulate (esp_set_gemm_compute);
    # parameters, gradients, optimizer state and all non-GEMM kernels stay fp32.  bf16 has the
    # fp32 exponent range, so the loss is never multiplied by a scale; the GradScaler's state is
    # still kept as the reference keeps it (Trainer.set_scaler).  SURVEY §8(d) C5.
    use_amp: bool = False
    # HIP-graph mode with variable-length data: pad each batch's frame axis up to a multiple of
    # graph_buckets[0] frames and its target axis to a multiple of graph_buckets[1] tokens, so
    # batches of nearby shapes replay one captured graph (bounded graph count over an epoch).
    # The padding is invisible to the result: lengths, SpecAug draws, BatchNorm statistics and
    # the depthwise-convolution boundary use the batch's own padded length (device tvalid).
    graph_buckets: Optional[Tuple[int, int]] = None
    # ---- epoch driver (Trainer.run, trainer.py:154-447; defaults of abs_task.py's arguments)
    resume: bool = True
    output_dir: Union[Path, str, None] = None
    max_epoch: int = 40
    seed: int = 0
    patience: Optional[int] = None
    keep_nbest_models: Union[int, List[int]] = 10
    nbest_averaging_interval: int = 0
    early_stopping_criterion: Sequence[str] = ("valid", "loss", "min")
    best_model_criterion: Sequence[Sequence[str]] = (("train", "loss", "min"), ("valid", "loss", "min"),
                                                     ("train", "acc", "max"), ("valid", "acc", "max"))
    val_scheduler_criterion: Sequence[str] = ("valid", "loss")


class _GraphEntry:
    """One captured training step for a batch signature (shapes): static inputs + outputs.
    Data-parallel entries hold the forward graph and the backward as segments, each followed
    by the gradient buckets that become complete with it."""
    __slots__ = ("graph", "speech", "prep", "stats", "weight", "fwd", "segs")


class Trainer:
    def __init__(self, model, optimizer: FusedAdam, scheduler=None, options: TrainerOptions = None,
                 distributed: bool = False, bucket_mb: float = 25.0, cuda_graph: bool = False):
        self.model = model
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.options = options or TrainerOptions()
        self.distributed = distributed and dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size() if self.distributed else 1
        # HIP-graph mode: the whole step (forward, backward, clip, Adam, zero_grad) is captured
        # once per batch signature and replayed: ~1500 launches per step cost one graph launch.
        # With DDP the forward and the backward segments are graphs, the collectives between
        # them eager (_dp_replay)
        self.cuda_graph = bool(cuda_graph) and model.flat.flat.is_cuda
        self._graphs = {}
        self.max_graphs = 32  # LRU bound on captured step graphs (each pins its workspace)
        self._key = None
        # DDP + graph: d loss of this replica = w_r / sum_r w / accum_grad, set on device between
        # the forward and the backward segments (the backward then yields pre-scaled gradients)
        self._scale = torch.ones(1, dtype=torch.float32, device=model.flat.flat.device)
        # graph DP replays: this replica's batch weight and the all-reduced sum (see _dp_replay)
        self._wloc = torch.ones(1, dtype=torch.float32, device=model.flat.flat.device)
        self._wsum = torch.ones(1, dtype=torch.float32, device=model.flat.flat.device)
        self._bufs_synced = False  # graph DP: the one broadcast of rank 0's buffers before the first step
        self.reducer = (FlatGradReducer(model, model.flat, bucket_mb, hooks=not self.cuda_graph)
                        if self.distributed else None)
        self.iiter = 0          # micro-batches (trainer.py:502 iiter)
        self.n_updates = 0      # optimizer steps attempted (every accum_grad micro-batches)
        self.n_skipped = 0      # ... of which skipped for a non-finite gradient norm
        self._synced_updates = 0  # n_updates at the last device->host counter sync (graph mode)
        self._clip = torch.empty(3, dtype=torch.float32, device=model.flat.flat.device)
        # finite flag of the last optimizer step, read back asynchronously (pinned buffer + event)
        # and acted on just before the NEXT optimizer step: the host never drains the queue
        cuda = self._clip.is_cuda
        self._flag_host = torch.empty(1, dtype=torch.float32, pin_memory=cuda)
        self._flag_event = torch.cuda.Event() if cuda else None
        self._pending = False
        self._last_weight = None  # the (all-reduced) weight of the last step, for the reporter
        self.scaler = None
        self._found_inf = None

    def set_scaler(self, scaler):
        """use_amp's loss-scaler state (trainer.py:181-195, 613-682): a torch GradScaler whose scale and
        growth tracker evolve as the reference's do -- after every optimizer step, x growth_factor once
        growth_interval consecutive steps were finite, x backoff_factor (and the step skipped) when the
        gradient norm was not -- updated on device from the step's finite flag (torch._amp_update_scale_,
        the op GradScaler.update runs; captured with the step in graph mode, so set it before the first
        step).  The bf16 arithmetic never multiplies the loss by the scale (bf16 has the fp32 exponent
        range: the unscaled gradients are the ones the reference unscales to), so the scale only travels in
        checkpoint.pth's "scaler" entry, which resumes either way."""
        self.scaler = scaler
        if scaler is not None and scaler.is_enabled():
            scaler._lazy_init_scale_growth_tracker(self._clip.device)
            self._found_inf = torch.zeros(1, dtype=torch.float32, device=self._clip.device)

    def _scaler_update(self):
        s = self.scaler
        if s is None or not s.is_enabled():
            return
        self._found_inf.fill_(1.0).sub_(self._clip[2:3])  # 1 where the step's gradient norm was non-finite
        torch._amp_update_scale_(s._scale, s._growth_tracker, self._found_inf, s._growth_factor,
                                 s._backoff_factor, s._growth_interval)

    @staticmethod
    def resume(checkpoint, model, reporter, optimizers, schedulers, scaler=None, ngpu: int = 0):
        """Trainer.resume (trainer.py:124-151): see train/checkpoint.resume."""
        from .checkpoint import resume
        resume(checkpoint, model, reporter, optimizers, schedulers, scaler, ngpu)

    def train_one_step(self, batch: Dict[str, torch.Tensor], check_finite: bool = True) -> Dict[str, torch.Tensor]:
        """One iteration of train_one_epoch's loop body; returns device-side stats."""
        with K.gemm_compute("bf16" if self.options.use_amp else "fp32"), K.param_cast_scope():
            stats = self._train_one_step(batch, check_finite)
        if K.GUARD:  # ESP_GUARD=1: workspace canaries checked after every step (syncs)
            K.check_guards()
        return stats

    def _train_one_step(self, batch, check_finite):
        if self.cuda_graph:
            return self._graph_step(batch)
        opts = self.options
        self.iiter += 1
        last = self.iiter % opts.accum_grad == 0
        model = self.model
        if self.reducer is not None:
            # gradient exchange once per optimizer step: the earlier micro-batches accumulate
            # locally (DDP.no_sync); averaging the accumulated sum equals the reference's
            # per-micro-batch DDP average (the all-reduce is linear)
            self.reducer.sync = last
            self.reducer.broadcast_buffers(model)
        loss, stats, weight = model(**batch)
        stats = {k: v for k, v in stats.items() if v is not None}
        self._last_weight = weight
        if self.distributed:
            w = weight.to(torch.float32).view(1)
            stats, wsum = fused_stats_allreduce(stats, weight)
            self._last_weight = wsum
            # (loss*weight).sum()/sum(weight)*world_size, DDP then averages  (trainer.py:594-606)
            loss = (loss * w).sum() / wsum * self.world
        loss = loss / opts.accum_grad
        loss.backward()
        if last:
            if self.reducer is not None:
                self.reducer.finish()
            self.resolve_pending()  # scheduler step of the previous update (if it was finite)
            self.n_updates += 1
            clip_grad_norm_(model.flat, opts.grad_clip, self._clip)
            # the Adam kernel itself skips a non-finite update on device (trainer.py:651-667)
            self.optimizer.step(clip=self._clip)
            self._scaler_update()
            if check_finite:
                self._flag_host.copy_(self._clip[2:3], non_blocking=True)
                if self._flag_event is not None:
                    self._flag_event.record()
                self._pending = True
            elif isinstance(self.scheduler, AbsBatchStepScheduler):
                self.scheduler.step()
            self.optimizer.zero_grad()
        stats["grad_norm"] = self._clip[0:1]
        return stats

    # ---------------------------------------------------------------- HIP-graph path
    def _graph_step(self, batch):
        model = self.model
        opts = self.options
        speech = batch["speech"]
        self.iiter += 1
        last = self.iiter % opts.accum_grad == 0
        tb = ub = None
        if opts.graph_buckets is not None:
            # frames padded to a multiple of bf (raw audio: the samples to the frame bucket's
            # sample count), targets to a multiple of bu
            bf, bu = opts.graph_buckets
            fe = getattr(model, "frontend", None)
            t_true = min(speech.shape[1], int(batch["speech_lengths"].max()))
            frames = fe.num_frames(t_true) if fe is not None else t_true
            tb = -(-frames // bf) * bf
            width = fe.samples_for_frames(tb) if fe is not None else tb
            ub = max(1, -(-int(batch["text_lengths"].max()) // bu)) * bu
            pad = (0, width - speech.shape[1]) if speech.dim() == 2 else (0, 0, 0, width - speech.shape[1])
            if speech.shape[1] < width:
                speech = torch.nn.functional.pad(speech, pad)
            elif speech.shape[1] > width:
                speech = speech[:, :width]
        prep = model.prepare(batch["speech_lengths"], batch["text"], batch["text_lengths"], speech.shape[1],
                             speech.shape[2] if speech.dim() == 3 else 0, t_bucket=tb, u_bucket=ub)
        sig = (tuple(speech.shape), prep.T, prep.Umax, prep.L, prep.get("n_samples", 0), last,
               tuple((k, tuple(v.shape)) for k, v in sorted(prep.host.items())))
        e = self._graphs.pop(sig, None)
        if self.distributed and not self._bufs_synced:
            # DDP broadcast_buffers (X7), outside the graph (a collective): once before the first step,
            # then at the END of every step (_dp_replay / _capture_dp), off the critical path --
            # training-mode outputs never read the running statistics and nothing writes them between
            # two steps, so every forward still starts from rank 0's buffers as with DDP's broadcast
            # before it.  Capture and replay steps issue the same collectives in the same order (a
            # rank may capture a new batch signature while another replays).
            self.reducer.broadcast_buffers(model)
            self._bufs_synced = True
        if last:
            self.n_updates += 1
        if e is None:  # the capture call's eager warm-up IS this iteration's step
            e = (self._capture_dp(speech, prep, last, float(prep.host["weight"].view(-1)[0])) if self.distributed
                 else self._capture(speech, prep, last))
        else:
            e.speech.copy_(speech, non_blocking=True)
            prep.copy_into(e.prep)
            if self.distributed:
                self._dp_replay(e, last, float(prep.host["weight"].view(-1)[0]))
            else:
                e.graph.replay()
        self._graphs[sig] = e  # most recently used last
        while len(self._graphs) > self.max_graphs:
            self._graphs.pop(next(iter(self._graphs)))
        if not self.distributed:
            self._last_weight = e.weight
        return e.stats

    def _device_body(self, speech, prep, with_opt: bool):
        """Device-only work of one step (nothing here talks to the host)."""
        K.rng_advance(self._key)
        loss, stats, weight = self.model.forward_prepared(speech, prep)
        (loss / self.options.accum_grad if self.options.accum_grad > 1 else loss).backward()
        stats = {k: v for k, v in stats.items() if v is not None}
        stats["grad_norm"] = self._clip[0:1]
        if with_opt:
            self._opt_tail()
        return stats, weight

    def _opt_tail(self):
        clip_grad_norm_(self.model.flat, self.options.grad_clip, self._clip)
        self.optimizer.step_device(self._clip, self.scheduler)  # counts itself only if finite
        self._scaler_update()
        self.model.flat.grad.zero_()

    # ---------------------------------------------------------------- DDP + HIP graph
    # DDP semantics (trainer.py:594-608 + DDP's bucketed average, overlapped with backward):
    #   sum w all-reduce (beside the forward replay) -> d loss_r = w_r / sum w (/ accum_grad) on device
    #   -> replay the backward in segments; after each segment the gradient buckets it completed are
    #   SUM-all-reduced asynchronously while the next segment runs -> stats all-reduce
    #   (recursive_average) and buffer broadcast launched -> wait -> clip + Adam.  Pre-scaling by
    #   d loss makes the SUM the weighted average, and accumulation over micro-batches is plain
    #   gradient accumulation (no_sync).
    def _dp_replay(self, e, last: bool, w_host: float):
        # The critical path is forward graph -> backward segments (+ their bucket all-reduces):
        #  * sum w: the batch weight is known on the host (espnet_model.prepare: weight = B, the
        #    reference's force_gatherable(batch_size)), so its all-reduce runs beside the forward
        #    replay, not between the forward and the first backward segment;
        #  * the reported stats' recursive_average and DDP's buffer broadcast are launched after the
        #    backward is queued and waited for at the end of the step (stream-ordered: the next step's
        #    kernels run after them).
        hw = self._dp_wsum(w_host, async_op=True)
        e.fwd.replay()
        hw.wait()
        self._dp_set_scale()
        handles = []
        for g, buckets in e.segs:
            g.replay()
            if last and buckets:
                handles += self.reducer.launch_sum(buckets)
        keys, vec = self._stats_vec(e.stats)
        tail = [dist.all_reduce(vec, async_op=True)] + self.reducer.broadcast_buffers(self.model, async_op=True)
        for h in handles:
            h.wait()
        if last:
            self._opt_tail()
        for h in tail:
            h.wait()
        self._stats_avg(e.stats, keys, vec)

    def _dp_wsum(self, w_host: float, async_op: bool):
        """sum_r w_r into self._wsum (this replica's w_r in self._wloc)."""
        self._wloc.fill_(w_host)
        self._wsum.copy_(self._wloc)
        return dist.all_reduce(self._wsum, async_op=async_op)

    def _dp_set_scale(self):
        torch.div(self._wloc, self._wsum, out=self._scale)
        if self.options.accum_grad > 1:
            self._scale.mul_(1.0 / self.options.accum_grad)

    def _stats_vec(self, stats):
        """recursive_average's all-reduce operand: the stats weighted by w_r, then w_r."""
        keys = [k for k in stats if k != "grad_norm"]
        return keys, torch.cat([stats[k].view(-1)[:1].float() * self._wloc for k in keys] + [self._wloc])

    def _stats_avg(self, stats, keys, vec):
        for i, k in enumerate(keys):
            stats[k].view(-1)[:1].copy_(vec[i:i + 1] / vec[-1:])
        self._last_weight = vec[-1:]

    def _dp_body(self, speech, prep):
        K.rng_advance(self._key)
        loss, stats, weight, ctx = self.model.forward_explicit(speech, prep)
        stats = {k: v for k, v in stats.items() if v is not None}
        stats["grad_norm"] = self._clip[0:1]
        return stats, weight, ctx

    def _capture_dp(self, speech, prep, last: bool, w_host: float):
        dev = self.model.flat.flat.device
        if self._key is None:
            self._key = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).to(dev)
        e = _GraphEntry()
        e.speech = speech.to(dev).clone()
        e.prep = prep.to_device(dev)
        model = self.model
        K.set_rng_key(self._key)
        try:
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):  # warm-up = this iteration's step (allocates workspaces)
                # the collectives of a replay (_dp_replay), in its order: sum w, the gradient buckets,
                # the stats, the buffer broadcast
                self._dp_wsum(w_host, async_op=False)
                stats, w, ctx = self._dp_body(e.speech, e.prep)
                # the replay takes the batch weight from the host (prepare()'s copy) for sum w, the loss
                # prescale and the stats average, where the eager path uses the device weight: they must
                # agree (one sync per capture)
                wd = float(w.view(-1)[0].item())
                if wd != w_host:
                    raise RuntimeError(f"graph DDP: device batch weight {wd} != host weight {w_host}")
                self._dp_set_scale()
                model.backward_explicit(ctx, self._scale)
                del ctx
                if last:
                    self.reducer.allreduce_sum()
                    self._opt_tail()
                keys, vec = self._stats_vec(stats)
                dist.all_reduce(vec)
                self._stats_avg(stats, keys, vec)
                self.reducer.broadcast_buffers(model)
                warm = {k: v.clone() for k, v in stats.items()}
                del stats, w
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            # release the warm-up step's cached blocks before the capture allocates the graph pool, as
            # torch.cuda.graph does on entry for the single-GPU capture: without it the DP step reserved the
            # warm-up's activations AND the pool's (230 vs 155 GiB at C2 B=256, r06b_bench_dp_b256.log)
            import gc
            gc.collect()
            torch.cuda.empty_cache()
            pool = torch.cuda.graph_pool_handle()
            cap = torch.cuda.Stream(device=dev)
            segs = []
            cur = [torch.cuda.CUDAGraph()]
            final = []

            def cut(ids):  # end the running segment where these buckets became complete
                if hook.done():
                    # the last buckets: nothing after them writes a gradient, so they ride the
                    # trailing segment (ending it here would capture an empty graph)
                    final.extend(ids)
                    return
                cur[0].capture_end()
                segs.append((cur[0], list(ids)))
                cur[0] = torch.cuda.CUDAGraph()
                cur[0].capture_begin(pool=pool, capture_error_mode="thread_local")

            hook = self.reducer.plan_hook(cut)
            with torch.cuda.stream(cap):
                gf = torch.cuda.CUDAGraph()
                gf.capture_begin(pool=pool, capture_error_mode="thread_local")
                e.stats, e.weight, ctx = self._dp_body(e.speech, e.prep)
                gf.capture_end()
                cur[0].capture_begin(pool=pool, capture_error_mode="thread_local")
                model.backward_explicit(ctx, self._scale, hook)
                del ctx
                cur[0].capture_end()
                segs.append((cur[0], final + hook.rest()))
            torch.cuda.current_stream(dev).wait_stream(cap)
            e.fwd, e.segs = gf, segs
        finally:
            K.set_rng_key(None)
        for k, v in warm.items():  # the warm-up step's values are this call's results
            e.stats[k].copy_(v)
        return e

    def _capture(self, speech, prep, last: bool = True):
        dev = self.model.flat.flat.device
        if self._key is None:  # dropout key from the CPU generator; advanced on device per step
            self._key = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).to(dev)
        e = _GraphEntry()
        e.speech = speech.to(dev).clone()
        e.prep = prep.to_device(dev)
        with_opt = last
        K.set_rng_key(self._key)
        grad_save = None
        try:
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):  # warm-up = this iteration's step (allocates workspaces)
                stats, w = self._device_body(e.speech, e.prep, with_opt)
                if not with_opt:  # the capture below must start from the same gradient state
                    grad_save = self.model.flat.grad.clone()
                    self.model.flat.grad.zero_()
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            # thread_local: the RCCL watchdog thread keeps querying its events during the capture
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                e.stats, e.weight = self._device_body(e.speech, e.prep, with_opt)
            e.graph = g
        finally:
            K.set_rng_key(None)  # eager calls keep their host seeds; the graph baked the key pointer
        if grad_save is not None:  # capturing ran nothing: restore the warm-up's gradient
            self.model.flat.grad.copy_(grad_save)
        for k, v in stats.items():  # the warm-up step's values are this call's results
            e.stats[k].copy_(v)
        return e

    def reset_dropout_stream(self):
        """HIP-graph mode: re-derive the device dropout key from the (just seeded) CPU generator and
        drop the captured graphs, whose host seeds were drawn at their capture.  Trainer.run calls
        it after each epoch's set_all_random_seed, so every epoch's masks follow from (seed, epoch)
        alone and a resumed run draws the masks of an uninterrupted one (eager steps draw their
        seeds from the CPU generator per step already)."""
        if not self.cuda_graph:
            return
        v = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64)
        if self._key is None:
            self._key = v.to(self.model.flat.flat.device)
        else:
            self._key.copy_(v)
        self._graphs.clear()

    def sync_host_state(self):
        """Bring the host-side optimizer / scheduler counters up to date after graph replays,
        and count the optimizer steps the device skipped (non-finite gradient norm)."""
        if self.cuda_graph and getattr(self.optimizer, "_dstate", None) is not None:
            before = self.optimizer.n_steps
            self.optimizer.sync_from_device(self.scheduler)
            taken = self.optimizer.n_steps - before
            self.n_skipped += (self.n_updates - self._synced_updates) - taken
        self._synced_updates = self.n_updates

    def resolve_pending(self):
        """Apply the bookkeeping of the last optimizer step once its finite flag is on the host:
        WarmupLR batch step if the gradient norm was finite, else count a skipped step
        (trainer.py:651-686).  Called before the next optimizer step and at epoch end."""
        if not self._pending:
            return
        if self._flag_event is not None:
            self._flag_event.synchronize()
        self._pending = False
        if float(self._flag_host[0]) != 0.0:
            if isinstance(self.scheduler, AbsBatchStepScheduler):
                self.scheduler.step()
        else:  # torch Adam would not have counted this step (the kernel skipped it on device)
            self.n_skipped += 1
            self.optimizer.n_steps -= 1

    def train_one_epoch(self, iterator: Iterable, reporter=None) -> bool:
        """Loop over (utt_id, batch) like trainer.py:502-714; returns True if every step was
        skipped (all_steps_are_invalid).  `reporter`: a SubReporter (train/reporter.py) gets,
        per batch, iter_time, the model's stats weighted by the batch weight, and on every
        optimizer step optim{i}_lr{j} + train_time, then next() (trainer.py:610,694-707);
        any other callable gets the step's device stats."""
        self.model.train()
        self.sync_host_state()
        up0, sk0 = self.n_updates, self.n_skipped
        rec = _EpochRecorder(self, reporter, train=True, iterator=iterator) if hasattr(reporter, "register") else None
        it = iter(self._stop_aligned(iterator))
        no_forward = False  # trainer.py:515-517: a no_forward_run batch makes the epoch valid
        t_step = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            try:
                _, batch = next(it)
            except StopIteration:
                break
            t_load = time.perf_counter() - t0
            if self.options.no_forward_run:  # trainer.py:515-517, 530-532
                no_forward = True
                if rec is not None:
                    rec.push_empty(t_load)
                continue
            stats = self.train_one_step(batch)
            if rec is not None:
                update = self.iiter % self.options.accum_grad == 0
                now = time.perf_counter()
                rec.push(stats, self._last_weight, t_load, update, now - t_step if update else None)
                if update:
                    t_step = now
            elif reporter is not None:
                reporter(stats)
        self.resolve_pending()
        self.sync_host_state()
        if rec is not None:
            rec.flush()
        # trainer.py:436-440: True when no optimizer step of the epoch was applied (and no batch
        # was passed over by no_forward_run, which the reference counts as valid)
        return not no_forward and (self.n_skipped - sk0) == (self.n_updates - up0)

    @torch.no_grad()
    def validate_one_epoch(self, iterator: Iterable, reporter=None) -> None:
        """trainer.py:724-772: the model in eval mode (no dropout / SpecAug, BatchNorm from its
        running statistics), per batch the stats weighted by the batch weight (recursive_average
        over the ranks: one fused all-reduce), iterator_stop across ranks."""
        self.model.eval()
        rec = _EpochRecorder(self, reporter, train=False, iterator=iterator) if reporter is not None else None
        for _, batch in self._stop_aligned(iterator):
            if self.options.no_forward_run:
                continue
            # one cast of the flat parameters per batch (param_cast_scope) instead of one planes copy per
            # weight per GEMM; a scope per batch, so no batch's activation copies outlive it.  fp32 like
            # the reference, whose validation runs outside autocast (trainer.py:724-772)
            with K.gemm_compute("fp32"), K.param_cast_scope():
                _, stats, weight = self.model(**batch)
            stats = {k: v for k, v in stats.items() if v is not None}
            if self.distributed:
                stats, weight = fused_stats_allreduce(stats, weight)
            if rec is not None:
                rec.push(stats, weight, None, False, None)
        if rec is not None:
            rec.flush()

    def run(self, train_iter_factory, valid_iter_factory, reporter=None, scaler=None) -> "object":
        """Trainer.run (trainer.py:154-447) for this trainer's model / optimizer / scheduler:
        resume from output_dir/checkpoint.pth, then per epoch: seed (seed + epoch), train, valid,
        epoch-step schedulers, and on rank 0 the checkpoint, {epoch}epoch.pth, latest.pth, the
        best-model links, n-best averaging and pruning; stop when every step of an epoch was
        invalid or on early stopping; finally the n-best averages.  Returns the Reporter."""
        from ..torch_utils.set_all_random_seed import set_all_random_seed
        from . import checkpoint as CK
        from .reporter import Reporter
        o = self.options
        keep = [o.keep_nbest_models] if isinstance(o.keep_nbest_models, int) else list(o.keep_nbest_models)
        if len(keep) == 0:
            logging.warning("No keep_nbest_models is given. Change to [1]")
            keep = [1]
        out = Path(o.output_dir) if o.output_dir is not None else None
        rank0 = not self.distributed or dist.get_rank() == 0
        reporter = reporter if reporter is not None else Reporter()
        schedulers = [self.scheduler]
        if out is not None and rank0:
            out.mkdir(parents=True, exist_ok=True)
        if scaler is None and o.use_amp and self.model.flat.flat.is_cuda and self.scaler is None:
            scaler = torch.amp.GradScaler("cuda")  # trainer.py:190-193 (use_amp)
        if scaler is not None:
            self.set_scaler(scaler)
        scaler = self.scaler
        if o.resume and out is not None and (out / "checkpoint.pth").exists():
            CK.resume(out / "checkpoint.pth", self.model, reporter, [self.optimizer], schedulers, scaler,
                      ngpu=1 if self.model.flat.flat.is_cuda else 0)
        start_epoch = reporter.get_epoch() + 1
        if start_epoch == o.max_epoch + 1:
            logging.warning(f"The training has already reached at max_epoch: {start_epoch}")
        crit = [tuple(c) for c in o.best_model_criterion]
        for iepoch in range(start_epoch, o.max_epoch + 1):
            logging.info(f"{iepoch}/{o.max_epoch}epoch started")
            set_all_random_seed(o.seed + iepoch)
            self.reset_dropout_stream()
            reporter.set_epoch(iepoch)
            with reporter.observe("train") as sub:
                all_invalid = self.train_one_epoch(train_iter_factory.build_iter(iepoch), reporter=sub)
            with reporter.observe("valid") as sub:
                self.validate_one_epoch(valid_iter_factory.build_iter(iepoch), reporter=sub)
            for sch in schedulers:
                if isinstance(sch, AbsValEpochStepScheduler):
                    sch.step(reporter.get_value(*o.val_scheduler_criterion))
                elif isinstance(sch, AbsEpochStepScheduler):
                    sch.step()
            if rank0:
                logging.info(reporter.log_message())
                if out is not None:
                    CK.save_checkpoint(out / "checkpoint.pth", self.model, reporter, [self.optimizer], schedulers,
                                       scaler, trainer=self)
                    CK.save_epoch(out, iepoch, self.model, reporter, crit, keep, o.nbest_averaging_interval)
            if all_invalid:
                logging.warning("The gradients at all steps are invalid in this epoch. Something seems wrong. "
                                f"This training was stopped at {iepoch}epoch")
                break
            if o.patience is not None and reporter.check_early_stopping(o.patience, *o.early_stopping_criterion):
                break
        else:
            logging.info(f"The training was finished at {o.max_epoch} epochs ")
        if rank0 and out is not None:
            CK.average_nbest_models(output_dir=out, reporter=reporter, best_model_criterion=crit, nbest=keep)
        return reporter

    def _stop_aligned(self, iterator):
        """iterator_stop (X1, trainer.py:505-510, 716-719): every rank stops when the first one
        runs out of batches.  The reference all-reduces a flag before EVERY batch (a host sync
        per step); here the ranks agree once on the shortest shard length up front, which
        gives the same batches when every rank's iterator knows its exact length (the sharded
        sampler iterators do: `exact_len`).  If ANY rank's iterator has no exact length (no
        len(), or a len() that is only a hint, e.g. an IterableDataset), every rank uses the
        reference's per-batch flag protocol, so a rank that runs out early cannot leave the
        others waiting in a collective."""
        if not self.distributed:
            yield from iterator
            return
        dev = self.model.flat.flat.device
        exact = hasattr(iterator, "__len__") and getattr(iterator, "exact_len", True) \
            and not isinstance(iterator, torch.utils.data.IterableDataset)
        n = len(iterator) if exact else 0
        # [shortest length, number of ranks WITHOUT an exact length]: one MIN and one SUM
        t = torch.tensor([n if exact else 2 ** 62, 0 if exact else 1], dtype=torch.int64, device=dev)
        t_min, t_cnt = t[:1].clone(), t[1:].clone()
        dist.all_reduce(t_min, op=dist.ReduceOp.MIN)
        dist.all_reduce(t_cnt, op=dist.ReduceOp.SUM)
        if int(t_cnt.item()) == 0:
            n_min = int(t_min.item())
            for i, item in enumerate(iterator):
                if i >= n_min:
                    break
                yield item
            return
        stop = torch.zeros(1, dtype=torch.int64, device=dev)
        for item in iterator:
            dist.all_reduce(stop)
            if int(stop.item()) > 0:
                return
            yield item
        stop.fill_(1)
        dist.all_reduce(stop)


class _EpochRecorder:
    """Reporter bookkeeping of one epoch pass without a host sync per step: each step's stats,
    weight and gradient-norm triple are copied into one small device tensor; every
    log_interval steps (and at the end) the snapshots come to the host in one copy and are
    registered in order, one reporter.next() per batch as the reference does."""

    def __init__(self, trainer: Trainer, reporter, train: bool, iterator=None):
        self.t = trainer
        self.rep = reporter
        self.train = train
        self.items = []
        li = trainer.options.log_interval
        if li is None:  # trainer.py:489-493: max(len(iterator) // 20, 10), 100 without a length
            try:
                li = max(len(iterator) // 20, 10)
            except TypeError:
                li = 100
        self.log_interval = li
        sch = trainer.scheduler
        self.sched_last = getattr(sch, "last_epoch", 0)
        self.n_logged = 0

    def push_empty(self, t_load):
        self.items.append(("empty", t_load))

    def push(self, stats, weight, t_load, update: bool, train_time):
        keys = [k for k, v in stats.items() if v is not None and k != "grad_norm"]
        dev = self.t.model.flat.flat.device
        vals = [stats[k].detach().reshape(-1)[:1].to(torch.float32) if torch.is_tensor(stats[k])
                else torch.tensor([float(stats[k])], dtype=torch.float32, device=dev) for k in keys]
        w = weight if torch.is_tensor(weight) else torch.tensor([float(weight)])
        w = w.detach().reshape(-1)[:1].to(device=dev, dtype=torch.float32)
        parts = vals + [w] + ([self.t._clip.detach().clone()] if update else [])
        snap = torch.cat([p.to(dev) for p in parts])
        self.items.append(("step", keys, snap, t_load, update, train_time))
        if len(self.items) >= self.log_interval:
            self.flush()
            if self.train and hasattr(self.rep, "log_message"):
                logging.info(self.rep.log_message(-self.log_interval))

    def flush(self):
        if not self.items:
            return
        snaps = [it[2] for it in self.items if it[0] == "step"]
        host = torch.cat(snaps).cpu().tolist() if snaps else []
        pos = 0
        for it in self.items:
            if it[0] == "empty":
                self.rep.register({"iter_time": it[1]})
                self.rep.next()
                continue
            _, keys, snap, t_load, update, train_time = it
            n = snap.numel()
            v = host[pos:pos + n]
            pos += n
            if t_load is not None:
                self.rep.register({"iter_time": t_load})
            self.rep.register(dict(zip(keys, v[:len(keys)])), v[len(keys)])
            if update:
                finite = v[len(keys) + 3] != 0.0
                lrs = self._lrs(finite)
                self.rep.register(dict({f"optim0_lr{j}": lr for j, lr in enumerate(lrs)}, train_time=train_time))
            self.rep.next()
        self.items = []

    def _lrs(self, finite: bool):
        """optim0_lr{j} after this optimizer step (trainer.py:694-705): the scheduler stepped iff
        the step was finite; WarmupLR's value is reconstructed from its step count."""
        sch = self.t.scheduler
        if finite and isinstance(sch, AbsBatchStepScheduler):
            self.sched_last += 1
        if hasattr(sch, "lr_at"):
            return sch.lr_at(self.sched_last)
        return [g["lr"] for g in self.t.optimizer.param_groups]
