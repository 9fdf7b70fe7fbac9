"""The collective schedule of the segmented-graph data-parallel step (VERDICT r5 'next' 6), on the CPU.

Trainer._capture_dp (a new batch signature: the eager warm-up is the step, then the capture) and
Trainer._dp_replay (a known signature) must issue the SAME collectives in the SAME order, because one rank
may capture while another replays (a first version broadcast before each capture and deadlocked exactly so,
DESIGN §5).  Two gloo ranks run the real _capture_dp / _dp_replay / FlatGradReducer code with the GPU parts
stubbed (HIP graphs and streams as no-ops, a stand-in model whose explicit backward fills the flat gradient
module by module and calls the bucket hook, as ESPnetASRModel.backward_explicit does); every
torch.distributed call is recorded.  Rank 0 captures a second signature while rank 1 replays the first,
then both replay; the per-step schedules must be equal across ranks and the gradient the weighted average.
"""
import contextlib
import os
import socket
import types

import torch

N_MODS = 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_CAPTURING = [None]


class _FakeGraph:
    """Work issued while capturing is recorded, not run; replay() runs it (as a HIP graph would)."""

    def __init__(self):
        self.ops = []

    def capture_begin(self, pool=None, capture_error_mode=None):
        _CAPTURING[0] = self

    def capture_end(self):
        _CAPTURING[0] = None

    def replay(self):
        for op in self.ops:
            op()


def _device_work(fn):
    if _CAPTURING[0] is not None:
        _CAPTURING[0].ops.append(fn)
    else:
        fn()


class _FakeStream:
    def wait_stream(self, other):
        pass


def _stub_cuda():
    torch.cuda.Stream = lambda device=None: _FakeStream()
    torch.cuda.stream = lambda s: contextlib.nullcontext()
    torch.cuda.current_stream = lambda device=None: _FakeStream()
    torch.cuda.synchronize = lambda device=None: None
    torch.cuda.graph_pool_handle = lambda: None
    torch.cuda.CUDAGraph = _FakeGraph


class _Model(torch.nn.Module):
    """Stand-in for ESPnetASRModel's explicit passes: N_MODS Linear modules (+ a BatchNorm, whose
    running statistics are the broadcast buffers); the backward writes each module's gradient
    (scale * a rank-dependent constant) from the last module to the first and calls the bucket hook."""

    def __init__(self, rank):
        super().__init__()
        self.mods = torch.nn.ModuleList([torch.nn.Linear(64, 64) for _ in range(N_MODS)])
        self.bn = torch.nn.BatchNorm1d(8)
        self.rank = rank
        from espnet_slurp_amd.flat import FlatParams
        self.flat = FlatParams(self, torch.device("cpu"))

    def forward_explicit(self, speech, prep):
        B = speech.shape[0]
        stats = {"loss": torch.tensor([1.0 + self.rank]), "acc": torch.tensor([0.25 * (self.rank + 1)])}
        return torch.tensor([1.0]), stats, torch.tensor([B]), object()

    def backward_explicit(self, ctx, scale, hook=None):
        for m in reversed(list(self.mods) + [self.bn]):
            def work(m=m):
                for p in m.parameters():
                    p.grad.add_(scale * float(self.rank + 1))
            _device_work(work)
            if hook is not None:  # host side, at capture time (the segment cuts)
                hook(m)


def _trainer(rank):
    from espnet_slurp_amd.train.distributed import FlatGradReducer
    from espnet_slurp_amd.train.trainer import Trainer
    tr = Trainer.__new__(Trainer)
    tr.model = _Model(rank)
    tr.reducer = FlatGradReducer(tr.model, tr.model.flat, bucket_mb=0.01, hooks=False)
    tr.options = types.SimpleNamespace(accum_grad=1)
    tr._key = None
    tr._clip = torch.zeros(4)
    tr._wloc = torch.zeros(1)
    tr._wsum = torch.zeros(1)
    tr._scale = torch.zeros(1)
    tr.opt_steps = 0

    def opt_tail():  # clip + Adam stand-in: record the averaged gradient, then zero it
        tr.last_grad = tr.model.flat.grad.clone()
        tr.opt_steps += 1
        tr.model.flat.grad.zero_()
    tr._opt_tail = opt_tail
    return tr


def _worker(rank, world, port, q):
    from datetime import timedelta

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    out = {"rank": rank, "ok": False}
    try:
        _stub_cuda()
        from espnet_slurp_amd import kernels as K
        K.set_rng_key = lambda key: None
        K.rng_advance = lambda key: None
        log = []
        ar0, bc0 = dist.all_reduce, dist.broadcast

        def all_reduce(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
            log.append(("all_reduce", str(op), t.numel()))
            return ar0(t, op=op, group=group, async_op=async_op)

        def broadcast(t, src, group=None, async_op=False):
            log.append(("broadcast", src, t.numel()))
            return bc0(t, src, group=group, async_op=async_op)
        dist.all_reduce, dist.broadcast = all_reduce, broadcast
        tr = _trainer(rank)
        nb = len(tr.reducer.buckets)
        B = 3 if rank == 0 else 2  # per-rank batch weights: w_r / sum w = 3/5, 2/5
        prep = types.SimpleNamespace(to_device=lambda dev: prep)
        sa = torch.zeros(B, 16, 80)
        sb = torch.zeros(B, 24, 80)
        steps = []
        grads = []
        # step 1: both capture A; step 2: rank 0 captures B while rank 1 replays A; step 3: both replay
        log.clear()
        ea = tr._capture_dp(sa, prep, True, float(B))
        steps.append(list(log))
        grads.append(tr.last_grad)
        log.clear()
        if rank == 0:
            tr._capture_dp(sb, prep, True, float(B))
        else:
            tr._dp_replay(ea, True, float(B))
        steps.append(list(log))
        grads.append(tr.last_grad)
        log.clear()
        tr._dp_replay(ea, True, float(B))
        steps.append(list(log))
        grads.append(tr.last_grad)
        # an accumulation micro-batch (not the last): no gradient bucket may be exchanged, capture or replay
        log.clear()
        tr.options.accum_grad = 2
        if rank == 0:
            tr._capture_dp(sb, prep, False, float(B))
        else:
            tr._dp_replay(ea, False, float(B))
        steps.append(list(log))
        out.update(steps=steps, nb=nb, grads=[g.tolist() for g in grads], opt_steps=tr.opt_steps, ok=True)
    except Exception as e:  # report instead of hanging the parent
        import traceback
        out["err"] = repr(e) + traceback.format_exc()
    finally:
        q.put(out)
        try:
            dist.destroy_process_group()
        except Exception:
            pass


def test_dp_capture_and_replay_issue_the_same_collectives():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
    assert all(r["ok"] for r in res), [r.get("err") for r in res]
    r0, r1 = res
    nb = r0["nb"]
    assert nb >= 3, nb  # several gradient buckets: the segment cuts are exercised
    for i, (s0, s1) in enumerate(zip(r0["steps"], r1["steps"])):
        assert s0 == s1, (i, s0, s1)
    # a last step: sum w, every gradient bucket once (SUM), the stats vector, the buffer broadcast
    full = r0["steps"][0]
    assert full[0][:2] == ("all_reduce", "RedOpType.SUM") and full[0][2] == 1
    assert sum(1 for c in full if c[0] == "all_reduce" and c[2] > 8) == nb
    assert full[-1][0] == "broadcast"
    # the accumulation micro-batch: no bucket exchange
    assert not any(c[0] == "all_reduce" and c[2] > 8 for c in r0["steps"][3])
    # gradient = sum_r (w_r / sum w) * (r + 1) = 3/5 * 1 + 2/5 * 2 = 1.4 on every element, every step
    for r in res:
        assert r["opt_steps"] == 3
        for g in r["grads"]:
            t = torch.tensor(g)
            assert torch.allclose(t[t != 0], torch.full_like(t[t != 0], 1.4)), (r["rank"], t.unique())
