"""Typed wrappers over the C ABI (include/espnet_mi355.h) for device torch tensors.

torch is used only as the device allocator / stream provider: every arithmetic op below
is a HIP kernel of libespnet_mi355.so launched on torch's current HIP stream.
"""
from __future__ import annotations

import math
import os
from typing import Optional, Sequence

import torch

from . import _native

KC, RC, I2C_KC, I2C_RC = 0, 1, 2, 3
ACT_NONE, ACT_RELU, ACT_SWISH = 0, 1, 2
ACT_MUL = 3          # bwd_act: dx = (dy W) * pre, pre holding dh/dv from an ACT_AUX_DERIV forward
ACT_AUX_DERIV = 16   # act flag: aux <- dh/dv of h = drop(act(v)) instead of v (gemm.hip fwd_elem)


def _p(t: Optional[torch.Tensor], off: int = 0):
    if t is None:
        return None
    return t.data_ptr() + off * t.element_size()


def _st():
    return torch.cuda.current_stream().cuda_stream


def _f32(*ts):
    for t in ts:
        if t is not None:
            assert t.dtype == torch.float32 and t.is_cuda, (t.dtype, t.device)


class _Workspace:
    """Grow-only scratch buffer per (device, stream): stream-ordered reuse is safe, and kernels
    on the weight-gradient side stream get their own buffer."""

    def __init__(self, zero: bool = False):
        self.buf = {}
        self.zero = zero  # zero-filled at allocation (the GEMM pool: split-K tickets, esp_gemm_f32)

    def get(self, nbytes: int, device) -> torch.Tensor:
        dev = torch.device(device)
        key = (str(dev), torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0)
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            b = (torch.zeros if self.zero else torch.empty)(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            self.buf[key] = b
        return b

    def reserve(self, nbytes: int, device):
        self.get(nbytes, device)


WS = _Workspace()
_WS2 = _Workspace()
_WS_C1 = _Workspace()  # esp_conv2_dgrad_c1fold's per-block records
_GEMM_WS = _Workspace(zero=True)  # split-K partials (stream-ordered reuse) + arrival tickets (last 64 KB)
_GEMM_WS_BYTES = 64 << 20


def _work(nbytes, device):
    return WS.get(nbytes, device)


# ESP_GUARD=1: every workspace handed to a launcher gets a 256-byte canary right after the bytes
# the launcher asked for (esp_*_workspace_bytes); after the launch a stream-ordered (and graph-
# capturable) compare folds "canary overwritten" into a per-launcher device flag, and
# check_guards() -- called by the trainer after every step in this mode -- raises naming the
# launcher.  A debug mode: it adds a fill + compare per workspace launch and a sync per step.
GUARD = os.environ.get("ESP_GUARD", "0") == "1"
GUARD_BYTES = 256
_GUARD_NAMES: list = []
_GUARD_FLAGS = {}


def _ws(pool: "_Workspace", launcher: str, nbytes: int, device) -> torch.Tensor:
    """A workspace of at least nbytes for `launcher` (+ its canary in guard mode)."""
    if not GUARD:
        return pool.get(nbytes, device)
    buf = pool.get(nbytes + GUARD_BYTES, device)
    buf[nbytes:nbytes + GUARD_BYTES].fill_(0xA5)
    return buf


def _guard_post(launcher: str, buf: torch.Tensor, nbytes: int):
    if not GUARD:
        return
    if launcher not in _GUARD_NAMES:
        _GUARD_NAMES.append(launcher)
    i = _GUARD_NAMES.index(launcher)
    key = str(buf.device)
    if key not in _GUARD_FLAGS:
        _GUARD_FLAGS[key] = torch.zeros(64, dtype=torch.int32, device=buf.device)
    bad = (buf[nbytes:nbytes + GUARD_BYTES] != 0xA5).any()
    _GUARD_FLAGS[key][i:i + 1].add_(bad.to(torch.int32).view(1))


def check_guards():
    """Raise if any workspace canary was overwritten since the last check (ESP_GUARD=1)."""
    for key, f in _GUARD_FLAGS.items():
        hit = f.nonzero().flatten().tolist()
        if hit:
            f.zero_()
            raise RuntimeError("espnet_slurp_amd: workspace overrun by " + ", ".join(_GUARD_NAMES[i] for i in hit)
                               + f" on {key}")


def _wsize(launcher: str, *dims) -> int:
    return _native.workspace_bytes(launcher, *dims)


def h2d(t: torch.Tensor, device) -> torch.Tensor:
    """Host tensor -> device through pinned memory, non-blocking: a pageable H2D copy would
    make the host wait for the stream to drain (a hidden synchronisation per call)."""
    device = torch.device(device)
    if device.type != "cuda" or t.is_cuda:
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


# ----------------------------------------------------------------------------- GEMM
_PROF = None  # when a list: (algorithmic flops, start event, end event) per GEMM launch


_PROF_ATTN = None  # when a list: (algorithmic flops, bytes written, start event, end event) per attention-probabilities launch


def profile_gemm_start():
    """Record a HIP event pair around every GEMM launch (on the launch stream) from now on, and
    around every rel-pos attention-probabilities launch (profile_attn_stop)."""
    global _PROF, _PROF_ATTN
    _PROF = []
    _PROF_ATTN = []


def profile_attn_stop():
    """-> (MFMA flops, bytes written, kernel ms, launches) of the esp_relpos_attn_probs launches
    since profile_gemm_start()."""
    global _PROF_ATTN
    prof, _PROF_ATTN = _PROF_ATTN or [], None
    torch.cuda.synchronize()
    return (sum(p[0] for p in prof), sum(p[1] for p in prof), sum(p[2].elapsed_time(p[3]) for p in prof), len(prof))


def profile_gemm_stop(by_shape: bool = False):
    """-> (total algorithmic FLOPs, total kernel ms, launches) since profile_gemm_start();
    with by_shape, also {(modes, M, N, K, batch): [launches, ms, flops, epilogue bytes]}."""
    global _PROF
    prof, _PROF = _PROF or [], None
    torch.cuda.synchronize()
    flops = sum(p[0] for p in prof)
    ms = 0.0
    shapes = {}
    for f, a, b, key, extra in prof:
        t = a.elapsed_time(b)
        ms += t
        s = shapes.setdefault(key, [0, 0.0, 0.0, 0.0])
        s[0] += 1
        s[1] += t
        s[2] += f
        s[3] += extra
    if by_shape:
        return flops, ms, len(prof), shapes
    return flops, ms, len(prof)


# Reduced-precision mode (esp_set_gemm_compute(1), TrainerOptions.use_amp): the unbatched KC / RC
# GEMMs (every nn.Linear forward / input / weight gradient) take bf16 operands from HBM
# (esp_gemm_bf16: PREC 2 LDS-DMA staging, transposing LDS reads for RC operands) after a
# round-to-nearest-even cast of each operand; the batched attention contractions and the conv2
# implicit-im2col GEMMs keep fp32 operands rounded to bf16 in LDS staging (PREC 1).  Same
# numerics either way: bf16-rounded operands, fp32 accumulate and epilogue.
# _AMP_BF16_OPERANDS = False keeps every GEMM on PREC 1 (A/B measurements).
_AMP_BF16_OPERANDS = True
# a Linear input's forward bf16 copy is kept for its weight gradient (_bf16_copy roles)
_KEEP_X16 = True
_COMPUTE = [0]  # mirror of esp_get_gemm_compute (set_gemm_compute)


# The bf16 copy of a weight gradient's dy (A of dW = dy^T x) is handed to the input-gradient GEMM
# that every nn.Linear backward runs right after it on the same dy (dx = dy W): linear_bwd_weight
# leaves it in _DY16 and only the next GEMM launch may take it, when its A is the same region
# (nothing runs between the two calls at any call site: blocks.py Linear / FFN / attention /
# convolution-module backward).  Any other launch drops it.
_DY16 = [None]


# Step-scoped casts: inside param_cast_scope (the Trainer's step: forward + backward, weights
# constant until the optimizer step that ends it) a weight's bf16 copy is made once and reused by
# its forward and input-gradient GEMMs, and a Linear input's forward copy by its weight gradient
# (_bf16_copy roles).  Parameter storage is registered by FlatParams (weakly: a dead model's range
# is ignored).
_W16 = [None]
_PARAM_RANGES = []


def register_param_storage(t: torch.Tensor):
    import weakref
    _PARAM_RANGES.append((weakref.ref(t), t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()))


class param_cast_scope:
    def __enter__(self):
        self.prev = _W16[0], _WP[0]
        _W16[0] = {}
        _WP[0] = {}
        return self

    def __exit__(self, *exc):
        _W16[0], _WP[0] = self.prev
        _DY16[0] = None


# fp32 GEMMs whose B operand is a weight take B as its three bf16 split planes (esp_gemm_f32_bp,
# gemm_kernels.h PREC 3): the same split products as the in-register split, bit for bit, with only A
# split in the k-loop.  A weight's planes are made once per step inside param_cast_scope (the
# Trainer's step; keyed like _W16, holding the fp32 source), else per GEMM.  _BPLANES = False: off
# (A/B measurements).
_BPLANES = True
# producers of GEMM-only activations write them as Planes: by default in the bf16 mode only (n = 1, the
# bf16 value its GEMMs round to: 805 vs 760 utt/s at C5 B=64); in the fp32 mode the consumers then
# need both operands as planes (PREC 5, 64-wide tiles), measured slower than splitting A in registers
# beside B's planes (PREC 3): 1222 vs 1333 utt/s at C2 B=128 (profiles/r04a_*).  _XPLANES = True: both
# modes, False: neither (tests/test_gpu_kernels.py sets both)
_XPLANES = "bf16"
_F32_PRODUCTS = [None]  # esp_f32_gemm_products() of the loaded build (set at first use)
_WP = [None]


class Planes:
    """An fp32 matrix held as its bf16 split planes, the operand format of the planes GEMMs: n = 3
    (esp_f32_to_planes: value = hi + mid + lo exactly, the fp32 path) or n = 1 (hi = bf16(value), round
    to nearest even: the reduced-precision path's bf16 operand).  rows x cols, row pitch ld (bf16
    elements, cols rounded up to 8), plane p at buf[p * ps], ps = rows * ld.  Producers write it in
    place of the fp32 tensor when only GEMMs read the value (LayerNorm outputs, the FFN hidden state,
    the attention context, the convolution module's BatchNorm + Swish output)."""
    __slots__ = ("buf", "rows", "cols", "ld", "ps", "n")

    def __init__(self, rows: int, cols: int, device, n: int = 3, buf=None):
        self.rows, self.cols, self.n = rows, cols, n
        self.ld = (cols + 7) // 8 * 8
        self.ps = rows * self.ld
        self.buf = torch.empty(n * self.ps, dtype=torch.bfloat16, device=device) if buf is None else buf

    @property
    def shape(self):
        return (self.rows, self.cols)

    @property
    def device(self):
        return self.buf.device

    def data_ptr(self) -> int:
        return self.buf.data_ptr()

    def float(self) -> torch.Tensor:
        """The fp32 values (hi + mid + lo, exact; tests and tools)."""
        p = self.buf.view(self.n, self.rows, self.ld)[:, :, : self.cols].float()
        return p.sum(0) if self.n == 3 else p[0]

    @staticmethod
    def of(x2d: torch.Tensor, n: int = 3) -> "Planes":
        """Split a contiguous-row fp32 matrix (esp_f32_to_planes; n = 1: its bf16 cast)."""
        rows, cols = x2d.shape
        p = Planes(rows, cols, x2d.device, n)
        if n == 3:
            _native.call("esp_f32_to_planes", _p(x2d), _p(p.buf), rows, cols, x2d.stride(0), p.ld, p.ps, _st())
        else:
            _native.call("esp_f32_to_bf16", _p(x2d), _p(p.buf), rows, cols, x2d.stride(0), p.ld, 0, _st())
        return p


def planes_mode() -> int:
    """Planes a producer writes for a GEMM-only tensor in the current compute mode: 3 (fp32 split
    products), 1 (bf16 GEMM operands), 0 (write fp32: _XPLANES False or an f32-MFMA build)."""
    if not _XPLANES or _XPLANES == "0":
        return 0
    if _F32_PRODUCTS[0] is None:
        _F32_PRODUCTS[0] = int(_native.load().esp_f32_gemm_products())
    if _COMPUTE[0] == GEMM_BF16:
        return 1 if _AMP_BF16_OPERANDS else 0
    return 3 if _F32_PRODUCTS[0] == 6 and _XPLANES in ("1", True) else 0


# Inside param_cast_scope, a parameter's bf16 copy / split planes are views into ONE copy of the whole
# flat parameter buffer made by one launch at its first use in the step (the FlatParams slots are
# 8-float aligned, so every weight's copy starts 16-B aligned): 155 per-weight launches per C2 step
# become one.  _FLAT_CAST = False: per-weight copies (A/B measurements).
_FLAT_CAST = True


def _param_flat(ptr: int, nbytes: int):
    """(flat tensor, its base address) of the registered parameter storage holding [ptr, ptr + nbytes)."""
    for r, a, b in _PARAM_RANGES:
        t = r()
        if t is not None and a <= ptr and ptr + nbytes <= b:
            return t, a
    return None


def _flat_view(kind: str, X, off: int, rows: int, cols: int, ld: int, wc):
    """(copy, element offset, flat numel) of a parameter matrix in the step's whole-flat copy (kind
    'bf16': esp_f32_to_bf16; 'planes': esp_f32_to_planes), or None when it does not qualify."""
    if not _FLAT_CAST or wc is None or ld != cols or cols % 8:
        return None
    ptr = X.data_ptr() + off * 4
    pf = _param_flat(ptr, ((rows - 1) * ld + cols) * 4)
    if pf is None:
        return None
    flat, base = pf
    e = (ptr - base) // 4
    n = flat.numel()
    if e % 8 or n % 8 or not flat.is_contiguous():
        return None
    key = ("flat", kind, base, n, torch.cuda.is_current_stream_capturing())
    hit = wc.get(key)
    if hit is None:
        if kind == "bf16":
            out = torch.empty(n, dtype=torch.bfloat16, device=flat.device)
            _native.call("esp_f32_to_bf16", _p(flat), _p(out), 1, n, n, n, 0, _st())
        else:
            out = torch.empty(3 * n, dtype=torch.bfloat16, device=flat.device)
            _native.call("esp_f32_to_planes", _p(flat), _p(out), 1, n, n, n, n, _st())
        hit = (out, flat)
        wc[key] = hit
    return hit[0], e, n


def planes(X, off: int, rows: int, cols: int, ld: int):
    """(planes, ldp, pstride): the three bf16 planes (esp_f32_to_planes) of the rows x cols fp32
    matrix at X[off] with row pitch ld; plane row pitch ldp = cols rounded up to 8."""
    fv = _flat_view("planes", X, off, rows, cols, ld, _WP[0])
    if fv is not None:  # (a parameter: a view into the step's planes of the whole flat buffer)
        buf, e, n = fv
        return buf[e:], cols, n
    key = (X.data_ptr() + off * 4, rows, cols, ld, torch.cuda.is_current_stream_capturing())
    wc = _WP[0]
    if wc is not None:
        hit = wc.get(key)
        if hit is not None:
            return hit[0], hit[1], hit[2]
    ldp = (cols + 7) // 8 * 8
    ps = rows * ldp
    out = torch.empty(3 * ps, dtype=torch.bfloat16, device=X.device)
    _native.call("esp_f32_to_planes", _p(X, off), _p(out), rows, cols, ld, ldp, ps, _st())
    if wc is not None:
        wc[key] = (out, ldp, ps, X)
    return out, ldp, ps


def _is_param(ptr: int, nbytes: int) -> bool:
    return any(r() is not None and a <= ptr and ptr + nbytes <= b for r, a, b in _PARAM_RANGES)


def _bf16_copy(X, off: int, rows: int, cols: int, ld: int, role: str = "") -> torch.Tensor:
    """bf16 (RNE) copy of the rows x cols fp32 matrix at X[off] with row pitch ld; the copy's row
    pitch is cols rounded up to 8 (esp_f32_to_bf16).  role "a_kc": the A operand of a KC GEMM (in
    the forward: a Linear's input x), kept for the step; role "b_rc": the B operand of an RC GEMM
    (a weight gradient's x), which takes the forward's copy of the same region.  Kept copies hold
    a reference to their fp32 source, so its memory cannot be handed to another tensor while the
    copy can be found; a Linear's input is never written between its forward and its weight
    gradient (the fp32 path reads it there too)."""
    key = (X.data_ptr() + off * 4, rows, cols, ld)
    memo, _DY16[0] = _DY16[0], None
    if memo is not None and memo[0] == key:
        return memo[1], memo[2]
    wc = _W16[0]
    if wc is not None:
        # a copy made outside a HIP-graph capture (the capture's eager warm-up) is never replayed by
        # the graph: entries are per capture state
        ckey = key + (torch.cuda.is_current_stream_capturing(),)
        param = _is_param(key[0], ((rows - 1) * ld + cols) * 4)
        if param:
            fv = _flat_view("bf16", X, off, rows, cols, ld, wc)
            if fv is not None:  # (a view into the step's bf16 copy of the whole flat buffer)
                return fv[0][fv[1]:], cols
        if param or role == "b_rc":
            hit = wc.get(ckey)
            if hit is not None:
                return hit[0], hit[1]
    ldy = (cols + 7) // 8 * 8
    out = torch.empty(rows * ldy, dtype=torch.bfloat16, device=X.device)
    _native.call("esp_f32_to_bf16", _p(X, off), _p(out), rows, cols, ld, ldy, 0, _st())
    if wc is not None and (param or (role == "a_kc" and _KEEP_X16)):
        wc[ckey] = (out, ldy, X)
    return out, ldy


def _gemm_amp_operands(M, N, K, A, B, C, mode_a, lda, mode_b, ldb, ldc, a_off, b_off, c_off, bias, alpha, beta,
                       R, r_off, act, aux, drop_p, seed, bwd_act, pre, rowsum, keep_a=False):
    """The bf16-operand form of gemm() (see _AMP_BF16_OPERANDS); False when not applicable."""
    if K % 8 or (mode_a == RC and M % 8) or (mode_b == RC and N % 8) or K < 64:
        _DY16[0] = None
        return False
    A16, la = _bf16_copy(A, a_off, M, K, lda, "a_kc") if mode_a == KC else _bf16_copy(A, a_off, K, M, lda)
    B16, lb = _bf16_copy(B, b_off, N, K, ldb) if mode_b == KC else _bf16_copy(B, b_off, K, N, ldb, "b_rc")
    if keep_a:  # (holding A: its memory cannot be handed to another tensor while the memo lives)
        _DY16[0] = ((A.data_ptr() + a_off * 4, K, M, lda), A16, la, A)
    # (a fused bias gradient, rowsum, sums the bf16 A values in fp32: torch AMP's sum of a bf16 dy)
    ws = _ws(_GEMM_WS, "esp_gemm_bf16", _GEMM_WS_BYTES, C.device)
    if _PROF is not None:  # the GEMM kernel alone (the operand casts are their own kernels)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    _native.call("esp_gemm_bf16", mode_a, mode_b, M, N, K, 1, 1, _p(A16), la, 0, 0, _p(B16), lb, 0, 0,
                 _p(C, c_off), ldc, 0, 0, _p(bias), float(alpha), float(beta), _p(R, r_off or 0), act,
                 _p(aux, c_off) if aux is not None else None, float(drop_p), seed & 0xFFFFFFFFFFFFFFFF,
                 int(bwd_act), _p(pre, c_off) if pre is not None else None, _p(rowsum), _p(ws), _GEMM_WS_BYTES,
                 _st())
    _guard_post("esp_gemm_bf16", ws, _GEMM_WS_BYTES)
    if _PROF is not None:
        ev1.record()
        extra = 4.0 * M * N * ((R is not None) + (aux is not None) + (pre is not None))
        _PROF.append((2.0 * M * N * K, ev0, ev1, (mode_a, mode_b, M, N, K, 1, "bf16"), extra))
    return True


def gemm(M: int, N: int, K: int, A, B, C, *, mode_a=KC, lda, mode_b=KC, ldb, ldc,
         a_off=0, b_off=0, c_off=0, batch=1, nb2=1, sa=(0, 0), sb=(0, 0), sc=(0, 0),
         bias=None, alpha=1.0, beta=0.0, R=None, r_off=None, act=ACT_NONE, aux=None,
         drop_p=0.0, seed=0, ic_a: Optional[Sequence[int]] = None, ic_b: Optional[Sequence[int]] = None,
         bwd_act=ACT_NONE, pre=None, rowsum=None, _keep_a16=False, b_weight=False, b_planes=None):
    """C[z](m,n) = alpha*epi(sum_k A(m,k)B(k,n) + bias) + beta*R (see gemm.hip).
    bwd_act/pre: epilogue drop'(.)*act'(pre) (FFN backward); rowsum: += sum_k A(m,k) (bias grad).
    b_weight: B is a weight-like operand, constant for the step (its split planes may be cached
    like a parameter's, see planes())."""
    if R is not None and r_off is None:
        r_off = c_off
    if isinstance(A, Planes) or isinstance(B, Planes) or isinstance(C, Planes):
        return _gemm_planes(M, N, K, A, B, C, mode_a, lda, mode_b, ldb, ldc, a_off, b_off, c_off, bias, alpha,
                            beta, R, r_off, act, aux, drop_p, seed, bwd_act, pre, rowsum, b_weight, batch, nb2, sa,
                            sb, sc, keep_a=_keep_a16)
    if (_COMPUTE[0] == GEMM_BF16 and _AMP_BF16_OPERANDS and batch == 1 and mode_a in (KC, RC)
            and mode_b in (KC, RC) and ic_a is None and ic_b is None and M > 0 and N > 0):
        if _gemm_amp_operands(M, N, K, A, B, C, mode_a, lda, mode_b, ldb, ldc, a_off, b_off, c_off, bias, alpha,
                              beta, R, r_off, act, aux, drop_p, seed, bwd_act, pre, rowsum, _keep_a16):
            return
    _DY16[0] = None
    ws = _ws(_GEMM_WS, "esp_gemm_f32", _GEMM_WS_BYTES, C.device)
    ica = (_native.I * 5)(*ic_a) if ic_a is not None else None
    icb = (_native.I * 5)(*ic_b) if ic_b is not None else None
    bp = None  # (planes pointer, plane row pitch, batch strides, plane stride)
    if (_BPLANES and _COMPUTE[0] == 0 and batch == 1 and mode_b in (KC, RC) and mode_a in (KC, RC, I2C_KC)
            and ic_b is None and M > 0 and N > 0 and K > 0):
        rows, cols = (N, K) if mode_b == KC else (K, N)
        if b_weight or _is_param(B.data_ptr() + b_off * 4, ((rows - 1) * ldb + cols) * 4):
            buf, ldp, ps = planes(B, b_off, rows, cols, ldb)
            bp = (_p(buf), ldp, 0, 0, ps)
    if (b_planes is not None and bp is None and _COMPUTE[0] == 0 and mode_b in (KC, RC) and mode_a in (KC, RC)
            and ic_a is None and ic_b is None and M > 0 and N > 0 and K > 0):
        # planes of B's whole source matrix, same element layout (ld): b_off and the batch strides carry over
        buf, ldp, ps = b_planes
        assert ldp == ldb, (ldp, ldb)
        bp = (_p(buf, b_off), ldp, sb[0], sb[1], ps)
    if _PROF is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    if bp is not None:
        _native.call("esp_gemm_f32_bp", mode_a, mode_b, M, N, K, batch, nb2,
                     _p(A, a_off), lda, sa[0], sa[1], _p(B, b_off), ldb, sb[0], sb[1],
                     _p(C, c_off), ldc, sc[0], sc[1], _p(bias), float(alpha), float(beta),
                     _p(R, r_off or 0), act, _p(aux, c_off) if aux is not None else None,
                     float(drop_p), seed & 0xFFFFFFFFFFFFFFFF,
                     int(bwd_act), _p(pre, c_off) if pre is not None else None, _p(rowsum),
                     ctypes_ptr(ica), _p(ws), _GEMM_WS_BYTES, bp[0], bp[1], bp[2], bp[3], bp[4], _st())
    else:
        _native.call("esp_gemm_f32", mode_a, mode_b, M, N, K, batch, nb2,
                     _p(A, a_off), lda, sa[0], sa[1], _p(B, b_off), ldb, sb[0], sb[1],
                     _p(C, c_off), ldc, sc[0], sc[1], _p(bias), float(alpha), float(beta),
                     _p(R, r_off or 0), act, _p(aux, c_off) if aux is not None else None,
                     float(drop_p), seed & 0xFFFFFFFFFFFFFFFF,
                     int(bwd_act), _p(pre, c_off) if pre is not None else None, _p(rowsum),
                     ctypes_ptr(ica), ctypes_ptr(icb), _p(ws), _GEMM_WS_BYTES, _st())
    _guard_post("esp_gemm_f32", ws, _GEMM_WS_BYTES)
    if _PROF is not None:
        ev1.record()
        # fused-epilogue streams the launch must move besides A, B, C: residual R and
        # pre-activation / derivative reads, aux writes (each one M x N fp32 tensor per batch)
        extra = 4.0 * M * N * batch * ((R is not None) + (aux is not None) + (pre is not None))
        key = (mode_a, mode_b, M, N, K, batch) + (("bp",) if bp is not None else ())
        _PROF.append((2.0 * M * N * K * batch, ev0, ev1, key, extra))


# _PLANES_DY_MEMO = False: the planes path casts a weight gradient's dy again for the input gradient
# (A/B measurements)
_PLANES_DY_MEMO = True


def _gemm_planes(M, N, K, A, B, C, mode_a, lda, mode_b, ldb, ldc, a_off, b_off, c_off, bias, alpha, beta, R, r_off,
                 act, aux, drop_p, seed, bwd_act, pre, rowsum, b_weight, batch=1, nb2=1, sa=(0, 0), sb=(0, 0),
                 sc=(0, 0), keep_a=False):
    """gemm() with an operand given as Planes (KC / RC; unbatched planes operands) or C written as
    Planes (fp32 mode: the plain and FFN w_1 epilogues): esp_gemm_f32_pl in the fp32 mode (the other
    operand's planes from the step cache when it is a weight, else split here), the hi planes as bf16
    operands in the reduced-precision mode (esp_gemm_bf16).  keep_a: a weight gradient's fp32 dy, whose
    bf16 copy is handed to the input-gradient GEMM that follows (_DY16), as in _gemm_amp_operands -- the
    fused q / k / v projections' dqkv beside their LayerNorm output's planes were cast twice."""
    memo = _DY16[0]
    _DY16[0] = None
    assert mode_a in (KC, RC) and mode_b in (KC, RC), (mode_a, mode_b)
    for X, off in ((A, a_off), (B, b_off)):
        if isinstance(X, Planes):
            assert off == 0 and batch == 1, "a Planes operand is a whole (unbatched) matrix"
    cp = C if isinstance(C, Planes) else None
    amp = _COMPUTE[0] == GEMM_BF16
    if amp and not (K % 8 == 0 and (mode_a == KC or M % 8 == 0) and (mode_b == KC or N % 8 == 0)):
        # shapes the bf16-operand kernel does not take (e.g. K = an odd token count): the fp32 operands of
        # the planes (the bf16 values themselves) through the fp32-operand launch, which rounds them to the
        # same bf16 in staging
        if isinstance(A, Planes):
            A, lda = A.float(), A.cols
        if isinstance(B, Planes):
            B, ldb = B.float(), B.cols
        if cp is None:
            return gemm(M, N, K, A, B, C, mode_a=mode_a, lda=lda, mode_b=mode_b, ldb=ldb, ldc=ldc, a_off=a_off,
                        b_off=b_off, c_off=c_off, batch=batch, nb2=nb2, sa=sa, sb=sb, sc=sc, bias=bias, alpha=alpha,
                        beta=beta, R=R, r_off=r_off, act=act, aux=aux, drop_p=drop_p, seed=seed, bwd_act=bwd_act,
                        pre=pre, rowsum=rowsum)
        b_weight = False  # (the fp32-operand planes-output launch below)
    if cp is not None:
        assert cp.n == (1 if amp else 3) and R is None and rowsum is None, cp.n
        if not isinstance(A, Planes) and not isinstance(B, Planes) and (
                amp and not (K % 8 == 0 and (mode_a == KC or M % 8 == 0) and (mode_b == KC or N % 8 == 0))
                or not b_weight and not _is_param(B.data_ptr() + b_off * 4, 4)):
            # fp32 operands, planes output (the attention context): esp_gemm_f32_pl without operand planes
            ws = _ws(_GEMM_WS, "esp_gemm_f32", _GEMM_WS_BYTES, cp.device)
            if _PROF is not None:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                ev0.record()
            _native.call("esp_gemm_f32_pl", mode_a, mode_b, M, N, K, batch, nb2, _p(A, a_off), lda, sa[0], sa[1],
                         None, 0, 0, 0, 0, _p(B, b_off), ldb, sb[0], sb[1], None, 0, 0, 0, 0,
                         _p(cp.buf, c_off), ldc, sc[0], sc[1], _p(bias), float(alpha), float(beta), None, act,
                         _p(aux, c_off) if aux is not None else None, float(drop_p), seed & 0xFFFFFFFFFFFFFFFF,
                         int(bwd_act), _p(pre, c_off) if pre is not None else None, None, cp.n, cp.ps, _p(ws),
                         _GEMM_WS_BYTES, _st())
            if _PROF is not None:
                ev1.record()
                extra = 4.0 * M * N * batch * (aux is not None) + (2.0 if cp.n == 3 else -2.0) * M * N * batch  # 6-/2-B out
                _PROF.append((2.0 * M * N * K * batch, ev0, ev1, (mode_a, mode_b, M, N, K, batch), extra))
            return
    assert batch == 1, "planes operands: unbatched GEMMs"
    if amp:
        def b16(X, off, rows, cols, ld, role="", m=None):
            if isinstance(X, Planes):
                return X.buf, X.ld
            _DY16[0] = m  # (A only: _bf16_copy hands the memo's copy over when it names this region)
            return _bf16_copy(X, off, rows, cols, ld, role)
        A16, la = b16(A, a_off, M, K, lda, "a_kc", memo) if mode_a == KC else b16(A, a_off, K, M, lda, "", memo)
        B16, lb = b16(B, b_off, N, K, ldb) if mode_b == KC else b16(B, b_off, K, N, ldb, "b_rc")
        _DY16[0] = None
        if keep_a and _PLANES_DY_MEMO and not isinstance(A, Planes):  # (holding A, as _gemm_amp_operands)
            _DY16[0] = ((A.data_ptr() + a_off * 4, K, M, lda), A16, la, A)
        ws = _ws(_GEMM_WS, "esp_gemm_bf16", _GEMM_WS_BYTES, C.device)
        if _PROF is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        if cp is not None:  # the bf16 result plane (the reduced-precision GEMM-only activations)
            _native.call("esp_gemm_bf16_pl", mode_a, mode_b, M, N, K, 1, 1, _p(A16), la, 0, 0, _p(B16), lb, 0, 0,
                         _p(cp.buf, c_off), ldc, 0, 0, _p(bias), float(alpha), float(beta), act,
                         _p(aux, c_off) if aux is not None else None, float(drop_p), seed & 0xFFFFFFFFFFFFFFFF,
                         int(bwd_act), _p(pre, c_off) if pre is not None else None, cp.n, cp.ps, _p(ws),
                         _GEMM_WS_BYTES, _st())
        else:
            _native.call("esp_gemm_bf16", mode_a, mode_b, M, N, K, 1, 1, _p(A16), la, 0, 0, _p(B16), lb, 0, 0,
                         _p(C, c_off), ldc, 0, 0, _p(bias), float(alpha), float(beta), _p(R, r_off or 0), act,
                         _p(aux, c_off) if aux is not None else None, float(drop_p), seed & 0xFFFFFFFFFFFFFFFF,
                         int(bwd_act), _p(pre, c_off) if pre is not None else None, _p(rowsum), _p(ws),
                         _GEMM_WS_BYTES, _st())
        _guard_post("esp_gemm_bf16", ws, _GEMM_WS_BYTES)
        if _PROF is not None:
            ev1.record()
            extra = 4.0 * M * N * ((R is not None) + (aux is not None) + (pre is not None))
            extra -= 2.0 * M * N if cp is not None else 0.0  # a 2-B result, not 4-B
            _PROF.append((2.0 * M * N * K, ev0, ev1, (mode_a, mode_b, M, N, K, 1, "bf16"), extra))
        return

    def pl(X, off, rows, cols, ld, weight):
        if isinstance(X, Planes):
            assert X.n == 3 and (X.rows, X.cols) == (rows, cols), ((X.rows, X.cols, X.n), (rows, cols))
            return None, 0, (X.buf, X.ld, X.ps)
        if weight or _is_param(X.data_ptr() + off * 4, ((rows - 1) * ld + cols) * 4):
            return X, off, planes(X, off, rows, cols, ld)
        return X, off, None
    ra, ca = (M, K) if mode_a == KC else (K, M)
    rb, cb = (N, K) if mode_b == KC else (K, N)
    Af, ao, ap = pl(A, a_off, ra, ca, lda, False)
    Bf, bo, bq = pl(B, b_off, rb, cb, ldb, b_weight)
    if bq is None:  # A given as planes: B's planes made here (the planes kernel needs both)
        bq = planes(B, b_off, rb, cb, ldb)
    ws = _ws(_GEMM_WS, "esp_gemm_f32", _GEMM_WS_BYTES, C.device)
    if _PROF is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    _native.call("esp_gemm_f32_pl", mode_a, mode_b, M, N, K, 1, 1,
                 _p(Af, ao) if Af is not None else None, lda if Af is not None else 0, 0, 0,
                 _p(ap[0]) if ap else None, ap[1] if ap else 0, 0, 0, ap[2] if ap else 0,
                 _p(Bf, bo) if Bf is not None else None, ldb if Bf is not None else 0, 0, 0,
                 _p(bq[0]), bq[1], 0, 0, bq[2],
                 _p(cp.buf if cp is not None else C, c_off), ldc, 0, 0, _p(bias), float(alpha), float(beta),
                 _p(R, r_off or 0), act, _p(aux, c_off) if aux is not None else None, float(drop_p),
                 seed & 0xFFFFFFFFFFFFFFFF, int(bwd_act), _p(pre, c_off) if pre is not None else None, _p(rowsum),
                 cp.n if cp is not None else 0, cp.ps if cp is not None else 0, _p(ws), _GEMM_WS_BYTES, _st())
    _guard_post("esp_gemm_f32", ws, _GEMM_WS_BYTES)
    if _PROF is not None:
        ev1.record()
        extra = 4.0 * M * N * ((R is not None) + (aux is not None) + (pre is not None)) + (2.0 * M * N if cp is not None else 0.0)
        _PROF.append((2.0 * M * N * K, ev0, ev1, (mode_a, mode_b, M, N, K, 1, "pl" if ap else "bp"), extra))


def gemm_bf16(M: int, N: int, K: int, A16, B16, C, *, lda, ldb, ldc, c_off=0, bias=None, alpha=1.0, beta=0.0,
              R=None, act=ACT_NONE, aux=None, drop_p=0.0, seed=0, bwd_act=ACT_NONE, pre=None, mode_a=KC,
              mode_b=KC):
    """C = alpha*epi(sum_k A(m,k) B(k,n) + bias) + beta*R with bf16 operands (torch.bfloat16) in
    mode KC ([rows][K]) or RC ([K][rows]) and the fp32 epilogue of gemm() (esp_gemm_bf16)."""
    assert A16.dtype == torch.bfloat16 and B16.dtype == torch.bfloat16
    ws = _ws(_GEMM_WS, "esp_gemm_bf16", _GEMM_WS_BYTES, C.device)
    if _PROF is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    _native.call("esp_gemm_bf16", mode_a, mode_b, M, N, K, 1, 1, _p(A16), lda, 0, 0, _p(B16), ldb, 0, 0,
                 _p(C, c_off), ldc, 0, 0, _p(bias), float(alpha), float(beta), _p(R, c_off) if R is not None else None,
                 act, _p(aux, c_off) if aux is not None else None, float(drop_p), seed & 0xFFFFFFFFFFFFFFFF,
                 int(bwd_act), _p(pre, c_off) if pre is not None else None, None, _p(ws), _GEMM_WS_BYTES, _st())
    _guard_post("esp_gemm_bf16", ws, _GEMM_WS_BYTES)
    if _PROF is not None:
        ev1.record()
        extra = 4.0 * M * N * ((R is not None) + (aux is not None) + (pre is not None))
        _PROF.append((2.0 * M * N * K, ev0, ev1, (mode_a, mode_b, M, N, K, 1, "bf16"), extra))


def to_bf16(x, rows: int, cols: int, ldx: int, transpose: bool = False, out=None):
    """bf16 copy (round to nearest even) of a rows x cols fp32 matrix with row pitch ldx;
    transpose: the cols x rows matrix (esp_f32_to_bf16)."""
    if out is None:
        out = torch.empty((cols, rows) if transpose else (rows, cols), dtype=torch.bfloat16, device=x.device)
    _native.call("esp_f32_to_bf16", _p(x), _p(out), rows, cols, ldx, out.stride(0), int(transpose), _st())
    return out


def ctypes_ptr(arr):
    import ctypes
    return ctypes.cast(arr, ctypes.c_void_p) if arr is not None else None


def linear_fwd(x2d, W, b, out, *, act=ACT_NONE, aux=None, drop_p=0.0, seed=0, alpha=1.0, R=None, beta=1.0,
               out_off=0, ldo=None, b_weight=False):
    """out = alpha*drop(act(x W^T + b)) (+ beta*R); x (M,K) (fp32 or Planes), W (N,K).  b_weight: W is a
    step-constant weight that is not a parameter view (a re-laid copy): its split planes are cached
    like one."""
    M, K = x2d.shape
    N = W.shape[0]
    gemm(M, N, K, x2d, W, out, mode_a=KC, lda=x2d.ld if isinstance(x2d, Planes) else x2d.stride(0), mode_b=KC, ldb=W.stride(0),
         ldc=ldo or N, c_off=out_off, bias=b, alpha=alpha, beta=beta if R is not None else 0.0, R=R,
         act=act, aux=aux, drop_p=drop_p, seed=seed, b_weight=b_weight)
    return out


def _ld(x):
    return x.ld if isinstance(x, Planes) else x.stride(0)


def linear_bwd_data(dy, W, dx, *, accumulate=False):
    """dx (+)= dy W ; dy (M,N) fp32 or Planes, W (N,K)."""
    M, N = dy.shape
    K = W.shape[1]
    gemm(M, K, N, dy, W, dx, mode_a=KC, lda=_ld(dy), mode_b=RC, ldb=W.stride(0), ldc=dx.stride(0),
         R=dx if accumulate else None, beta=1.0)
    return dx


def linear_bwd_data_act(dy, W, dx, pre, act, drop_p=0.0, seed=0, b_weight=False):
    """dx = drop'(dy W) * act'(pre): the input gradient of w_2 fused with the backward of
    h = drop(act(pre)) (positionwise_feed_forward.py:32)."""
    M, N = dy.shape
    K = W.shape[1]
    gemm(M, K, N, dy, W, dx, mode_a=KC, lda=_ld(dy), mode_b=RC, ldb=W.stride(0), ldc=_ld(dx),
         bwd_act=act, pre=pre, drop_p=drop_p, seed=seed, b_weight=b_weight)
    return dx


def linear_bwd_weight(dy, x, dW, db=None):
    """dW += dy^T x ; db += colsum(dy) (fused into the same GEMM pass over dy); x fp32 or Planes.  An fp32 x
    that carries its split planes (`twin_planes`: a LayerNorm output written by esp_layernorm_fwd_dual) is
    taken as B planes (PREC 3: only dy is split in the k-loop)."""
    M, N = dy.shape
    K = x.shape[1]
    tw = twin_planes(x) if _COMPUTE[0] == 0 else None
    gemm(N, K, M, dy, x, dW, mode_a=RC, lda=_ld(dy), mode_b=RC, ldb=_ld(x), ldc=dW.stride(0), R=dW, beta=1.0,
         rowsum=db, _keep_a16=True, b_planes=None if tw is None else (tw.buf, tw.ld, tw.ps))


# fp32 tensors that also carry their three split planes (an attribute of the tensor object, so it lives
# exactly as long as the tensor the backward keeps): the fp32 mode's LayerNorm outputs that feed Linears
# (forward: fp32 A beside the weight planes; weight gradient: these planes as B, PREC 3).  Measured neutral
# at C2 B=256 (profiles/r05k_wgrad_xplanes_ab.txt: 66 weight gradients 176 -> 174 us on PREC 3, the dual
# LayerNorm 33 -> 47 us), so off: the RC x RC k-loop is not bound by B's split alone (its dy operand still
# splits in registers from ds_read_b32 fragments).  The path stays tested
# (test_layernorm_dual_and_weight_gradient_on_twin_planes) for A-side planes.
WGRAD_XPLANES = False


def wgrad_xplanes_ok() -> bool:
    """The fp32 mode of a split-product build (the planes are the B operand of a PREC 3 weight gradient)."""
    if not WGRAD_XPLANES or _COMPUTE[0] != 0:
        return False
    if _F32_PRODUCTS[0] is None:
        _F32_PRODUCTS[0] = int(_native.load().esp_f32_gemm_products())
    return _F32_PRODUCTS[0] == 6


def twin_planes(x):
    pl = getattr(x, "_esp_planes", None)
    return pl if pl is not None and pl.rows == x.shape[0] and pl.cols == x.shape[1] else None


def layernorm_fwd_dual(x2d, w, b, y, mean, rstd, eps=1e-12):
    """esp_layernorm_fwd_dual: y (fp32) and its split planes, attached to y (twin_planes)."""
    M, D = x2d.shape
    pl = Planes(M, D, x2d.device, 3)
    _native.call("esp_layernorm_fwd_dual", _p(x2d), _p(w), _p(b), _p(y), _p(pl.buf), pl.ld, pl.ps, 3, _p(mean),
                 _p(rstd), M, D, float(eps), _st())
    y._esp_planes = pl
    return y


def colsum(x2d, out, accumulate=True, M=None, N=None, ld=None):
    M = M if M is not None else x2d.shape[0]
    N = N if N is not None else x2d.shape[1]
    ld = ld if ld is not None else x2d.stride(0)
    n = _wsize("esp_colsum", M, N)
    w = _ws(WS, "esp_colsum", n, x2d.device)
    _native.call("esp_colsum", _p(x2d), M, N, ld, _p(out), int(accumulate), _p(w), n, _st())
    _guard_post("esp_colsum", w, n)


# ----------------------------------------------------------------------------- elementwise
def act_bwd(dy, h, dx, act, drop_p=0.0, seed=0, idx_off=0):
    _native.call("esp_act_bwd", _p(dy), _p(h), _p(dx), dy.numel(), act, float(drop_p), seed, idx_off, _st())
    return dx


def scale_dropout(x, y, alpha=1.0, drop_p=0.0, seed=0, r=None, beta=1.0):
    """y = alpha * drop(x) (+ beta * r); y fp32 or Planes (no residual; x contiguous rows)."""
    if isinstance(y, Planes):
        assert r is None and y.ld == y.cols and x.numel() == y.rows * y.cols
        _native.call("esp_scale_dropout_planes", _p(x), _p(y.buf), x.numel(), y.ps, y.n, float(alpha), float(drop_p),
                     seed, _st())
        return y
    _native.call("esp_scale_dropout", _p(x), _p(y), x.numel(), float(alpha), float(drop_p), seed, _p(r),
                 float(beta), _st())
    return y


def grad_planes_like(x2d):
    """A backward gradient that only GEMMs read (a branch's weight- and input-gradient GEMMs), as Planes in
    the fp32 mode (n = 3) or their bf16 plane in the reduced-precision mode (n = 1: the bf16 value the GEMMs
    would round it to), None otherwise (the caller keeps fp32)."""
    M, D = x2d.shape
    n = planes_mode()
    if n and D % 8 == 0 and x2d.is_contiguous():
        return Planes(M, D, x2d.device, n)
    return None


def scale_by_dev(x, s):
    _native.call("esp_scale_by_dev", _p(x), x.numel(), _p(s), _st())


def embed_fwd(tok, E, pe, y, L, xscale, drop_p, seed):
    _native.call("esp_embed_fwd", _p(tok), _p(E), _p(pe), _p(y), tok.numel(), L, E.shape[1], float(xscale),
                 float(drop_p), seed, _st())


def embed_bwd(tok, dy, dE, xscale, drop_p, seed):
    _native.call("esp_embed_bwd", _p(tok), _p(dy), _p(dE), tok.numel(), dE.shape[0], dE.shape[1],
                 float(xscale), float(drop_p), seed, _st())


def specaug(x, y, lens_i32, warp_i32, fmask_i32, tmask_i32):
    B, T, F = x.shape
    nf = 0 if fmask_i32 is None else fmask_i32.shape[1]
    nt = 0 if tmask_i32 is None else tmask_i32.shape[1]
    _native.call("esp_specaug", _p(x), _p(y), B, T, F, _p(lens_i32), _p(warp_i32), _p(fmask_i32), nf,
                 _p(tmask_i32), nt, _st())


def utterance_mvn(x, lens_i32):
    B, T, F = x.shape
    _native.call("esp_utterance_mvn", _p(x), B, T, F, _p(lens_i32), _st())


def grad_norm(g, max_norm, out3):
    n = _wsize("esp_grad_norm", g.numel())
    w = _ws(_WS2, "esp_grad_norm", n, g.device)
    _native.call("esp_grad_norm", _p(g), g.numel(), float(max_norm), _p(w), n, _p(out3), _st())
    _guard_post("esp_grad_norm", w, n)


def adam(p, g, m, v, clip3, lr, b1, b2, eps, wd, step):
    _native.call("esp_adam", _p(p), _p(g), _p(m), _p(v), p.numel(), _p(clip3), float(lr), float(b1), float(b2),
                 float(eps), float(wd), int(step), _st())


def adam_amsgrad(p, g, m, v, vmax, clip3, lr, b1, b2, eps, wd, step):
    _native.call("esp_adam_amsgrad", _p(p), _p(g), _p(m), _p(v), _p(vmax), p.numel(), _p(clip3), float(lr), float(b1),
                 float(b2), float(eps), float(wd), int(step), _st())


def adam_dev_amsgrad(p, g, m, v, vmax, clip3, hyper3, b1, b2, eps, wd):
    _native.call("esp_adam_dev_amsgrad", _p(p), _p(g), _p(m), _p(v), _p(vmax), p.numel(), _p(clip3), _p(hyper3),
                 float(b1), float(b2), float(eps), float(wd), _st())


def opt_hyper(state_f64, base_lr, warmup, b1, b2, hyper3):
    _native.call("esp_opt_hyper", _p(state_f64), float(base_lr), float(warmup), float(b1), float(b2), _p(hyper3),
                 _st())


def adam_dev(p, g, m, v, clip3, hyper3, b1, b2, eps, wd):
    _native.call("esp_adam_dev", _p(p), _p(g), _p(m), _p(v), p.numel(), _p(clip3), _p(hyper3), float(b1), float(b2),
                 float(eps), float(wd), _st())


def opt_advance(state_f64, clip3):
    _native.call("esp_opt_advance", _p(state_f64), _p(clip3), _st())


GEMM_FP32, GEMM_BF16 = 0, 1


def set_gemm_compute(dtype) -> int:
    """Select the MFMA input type of every later GEMM launch: "fp32"/0 (default, exact f32
    fma chain) or "bf16"/1 (operands rounded to bf16 in LDS staging, fp32 accumulate and
    outputs).  Process-wide; returns the previous setting (esp_set_gemm_compute)."""
    code = {"fp32": GEMM_FP32, "float32": GEMM_FP32, "bf16": GEMM_BF16, "bfloat16": GEMM_BF16}.get(dtype, dtype)
    lib = _native.load()
    prev = lib.esp_set_gemm_compute(int(code))
    if prev < 0:
        raise _native.NativeError(f"esp_set_gemm_compute failed: {lib.esp_last_error().decode()}")
    _COMPUTE[0] = int(code)
    return prev


def set_splitk_mode(mode: int) -> int:
    """0: split-K partials combined by a separate reduction launch (default); 1: in-kernel by the
    last-arriving unit of each tile (esp_set_splitk_mode).  Returns the previous mode."""
    lib = _native.load()
    prev = lib.esp_set_splitk_mode(int(mode))
    if prev < 0:
        raise _native.NativeError(f"esp_set_splitk_mode failed: {lib.esp_last_error().decode()}")
    return prev


def get_gemm_compute() -> int:
    return _native.load().esp_get_gemm_compute()


class gemm_compute:
    """Context manager: GEMMs inside the block run with the given input type."""

    def __init__(self, dtype):
        self.dtype = dtype

    def __enter__(self):
        self.prev = set_gemm_compute(self.dtype)
        return self

    def __exit__(self, *exc):
        set_gemm_compute(self.prev)


def set_rng_key(key_u64: Optional[torch.Tensor]):
    """Route every dropout kernel's seed through *key (device int64 tensor) or switch it off."""
    _native.call("esp_set_rng_key", _p(key_u64))


def rng_advance(key_u64):
    _native.call("esp_rng_advance", _p(key_u64), _st())


# ----------------------------------------------------------------------------- norms
def layernorm_fwd(x2d, w, b, y, mean, rstd, eps=1e-12):
    M, D = x2d.shape
    _native.call("esp_layernorm_fwd", _p(x2d), _p(w), _p(b), _p(y), _p(mean), _p(rstd), M, D, float(eps), _st())


def layernorm_fwd_planes(x2d, w, b, y: "Planes", mean, rstd, eps=1e-12):
    M, D = x2d.shape
    _native.call("esp_layernorm_fwd_planes", _p(x2d), _p(w), _p(b), _p(y.buf), y.ld, y.ps, y.n, _p(mean), _p(rstd),
                 M, D, float(eps), _st())


def layernorm_bwd(dy, x, w, mean, rstd, dx, dw, db, accumulate=False):
    M, D = x.shape
    n = _wsize("esp_layernorm_bwd", M, D)
    ws = _ws(WS, "esp_layernorm_bwd", n, x.device)
    _native.call("esp_layernorm_bwd", _p(dy), _p(x), _p(w), _p(mean), _p(rstd), _p(dx), int(accumulate), _p(dw),
                 _p(db), M, D, _p(ws), n, _st())
    _guard_post("esp_layernorm_bwd", ws, n)


def glu_fwd(u, g):
    rows, D = g.shape
    _native.call("esp_glu_fwd", _p(u), _p(g), rows, D, _st())


def glu_bwd(u, dg, du):
    """du: fp32 [rows, 2D] or Planes (esp_glu_bwd_planes)."""
    rows, D = dg.shape
    if isinstance(du, Planes):
        assert du.ld == 2 * D
        _native.call("esp_glu_bwd_planes", _p(u), _p(dg), _p(du.buf), du.ps, du.n, rows, D, _st())
        return
    _native.call("esp_glu_bwd", _p(u), _p(dg), _p(du), rows, D, _st())


# tvalid: optional device int32 (1,) — the batch is padded to T frames per utterance, only the
# first tvalid[0] are frames of the reference batch (length-bucketed graphs, norm.hip valid_T)
def dwconv1d(x, W, bias, y, Bn, T, D, K, flip=False, tvalid=None):
    _native.call("esp_dwconv1d", _p(x), _p(W), _p(bias), _p(y), Bn, T, D, K, int(flip), _p(tvalid), _st())


def dwconv1d_wgrad(dy, x, dW, Bn, T, D, K, tvalid=None):
    n = _wsize("esp_dwconv1d_wgrad", Bn, T, D, K)
    ws = _ws(WS, "esp_dwconv1d_wgrad", n, x.device)
    _native.call("esp_dwconv1d_wgrad", _p(dy), _p(x), _p(dW), Bn, T, D, K, _p(ws), n, _p(tvalid), _st())
    _guard_post("esp_dwconv1d_wgrad", ws, n)


def bn_swish_fwd(y, gamma, beta, s, mean, rstd, run_mean, run_var, momentum=0.1, eps=1e-5, T=0, tvalid=None):
    """s: fp32 [M, D] or Planes (esp_bn_swish_fwd_planes)."""
    M, D = y.shape
    n = _wsize("esp_bn_swish_fwd", M, D)
    ws = _ws(WS, "esp_bn_swish_fwd", n, y.device)
    if isinstance(s, Planes):
        _native.call("esp_bn_swish_fwd_planes", _p(y), _p(gamma), _p(beta), _p(s.buf), s.ld, s.ps, s.n, _p(mean),
                     _p(rstd), _p(run_mean), _p(run_var), float(momentum), float(eps), M, D, _p(ws), n, int(T),
                     _p(tvalid), _st())
    else:
        _native.call("esp_bn_swish_fwd", _p(y), _p(gamma), _p(beta), _p(s), _p(mean), _p(rstd), _p(run_mean),
                     _p(run_var), float(momentum), float(eps), M, D, _p(ws), n, int(T), _p(tvalid), _st())
    _guard_post("esp_bn_swish_fwd", ws, n)


def bn_swish_eval(y, gamma, beta, s, run_mean, run_var, mean, rstd, eps=1e-5):
    """Eval-mode BatchNorm (running statistics) fused with Swish."""
    M, D = y.shape
    _native.call("esp_bn_swish_eval", _p(y), _p(gamma), _p(beta), _p(s), _p(run_mean), _p(run_var), float(eps), M, D,
                 _p(mean), _p(rstd), _st())


def bn_swish_bwd(ds, y, mean, rstd, gamma, beta, dy, dgamma, dbeta, sums, T=0, tvalid=None):
    M, D = y.shape
    n = _wsize("esp_bn_swish_bwd", M, D)
    ws = _ws(WS, "esp_bn_swish_bwd", n, y.device)
    _native.call("esp_bn_swish_bwd", _p(ds), _p(y), _p(mean), _p(rstd), _p(gamma), _p(beta), _p(dy), _p(dgamma),
                 _p(dbeta), M, D, _p(ws), n, _p(sums), int(T), _p(tvalid), _st())
    _guard_post("esp_bn_swish_bwd", ws, n)


# ----------------------------------------------------------------------------- attention
def heads_split(src, ld, col0, B, T, H, dk, bias, dst):
    _native.call("esp_heads_split", _p(src), ld, col0, B, T, H, dk, _p(bias), _p(dst), _st())


def heads_split2(src, ld, col0, B, T, H, dk, bias_a, dst_a, bias_b, dst_b):
    """dst_a = head-major(src) + bias_a and dst_b = head-major(src) + bias_b in one pass."""
    _native.call("esp_heads_split2", _p(src), ld, col0, B, T, H, dk, _p(bias_a), _p(dst_a), _p(bias_b), _p(dst_b),
                 _st())


def add2d(x, ldx, y, ldy, M, N, x_off=0, y_off=0):
    _native.call("esp_add2d", _p(x, x_off), ldx, _p(y, y_off), ldy, M, N, _st())


# row pitch granularity of score-like buffers (floats)
SCORE_ALIGN = 4


def pitch(n: int) -> int:
    """Row pitch of score-like buffers: a multiple of SCORE_ALIGN (>= 4) floats, so every row is 16-B
    aligned and the GEMMs reading them take the LDS-DMA path."""
    return (n + SCORE_ALIGN - 1) // SCORE_ALIGN * SCORE_ALIGN


def attn_softmax_fwd(ac, bd, relpos, P, sqrt_dk, klen_i32, nb, causal, attn, pdrop, drop_p, seed, Z, Tq, Tk,
                     lds=None, ldp=None, tvalid=None):
    _native.call("esp_attn_softmax_fwd", _p(ac), _p(bd), relpos, P, float(sqrt_dk), _p(klen_i32), nb, int(causal),
                 _p(attn), _p(pdrop), float(drop_p), seed, Z, Tq, Tk, lds or Tk, ldp or max(P, 1), _p(tvalid), _st())


def relpos_softmax_fwd(q_v, p, ldp_row, nb, H, ac, sqrt_dk, klen_i32, attn, pdrop, drop_p, seed, T, lds):
    """Fused latest rel-pos bd window (MFMA) + rel_shift + masked softmax + dropout copy."""
    _f32(q_v, p, ac, attn, pdrop)
    _native.call("esp_relpos_softmax_fwd", _p(q_v), _p(p), ldp_row, nb, H, _p(ac), float(sqrt_dk), _p(klen_i32),
                 _p(attn), _p(pdrop), float(drop_p), int(seed) & (2 ** 64 - 1), T, lds, _st())


def relpos_attn_fwd(q_u, q_v, kmat, ldk, p, ldp_row, nb, H, sqrt_dk, klen_i32, attn, pdrop, drop_p, seed, T, lds,
                    k_off=0):
    """Fused latest rel-pos attention probabilities (ac and the bd band on the MFMA in-kernel)."""
    _f32(q_u, q_v, kmat, p, attn, pdrop)
    _native.call("esp_relpos_attn_fwd", _p(q_u), _p(q_v), _p(kmat, k_off), ldk, _p(p), ldp_row, nb, H,
                 float(sqrt_dk), _p(klen_i32), _p(attn), _p(pdrop), float(drop_p), int(seed) & (2 ** 64 - 1), T, lds,
                 _st())


def relpos_attn_probs(q_u, q_v, kmat, ldk, p, ldp_row, relpos, nb, H, sqrt_dk, klen_i32, attn, pdrop, drop_p, seed,
                      T, lds, k_off=0, tvalid=None):
    """Rel-pos attention probabilities, latest (relpos 1) or legacy (relpos 2), one wave per 16
    query rows (esp_relpos_attn_probs); tvalid: legacy length-bucket T' (device int32)."""
    _f32(q_u, q_v, kmat, p, attn, pdrop)
    if _PROF_ATTN is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    _native.call("esp_relpos_attn_probs", _p(q_u), _p(q_v), _p(kmat, k_off), ldk, _p(p), ldp_row, int(relpos), nb, H,
                 float(sqrt_dk), _p(klen_i32), _p(attn), _p(pdrop), float(drop_p), int(seed) & (2 ** 64 - 1), T, lds,
                 _p(tvalid), _st())
    if _PROF_ATTN is not None:
        ev1.record()
        # algorithmic: per (head, utterance) ac = q_u k^T and the T' rel-pos (bd) columns each row
        # keeps after rel_shift, 2 * T'^2 * d_k each (no padded tiles)
        flops = 4.0 * T * T * 64 * nb * H
        written = 4.0 * nb * H * T * T * (2 if (pdrop is not None and drop_p > 0) else 1)
        _PROF_ATTN.append((flops, written, ev0, ev1))


def attn_bwd_prep(dctx, ldd, ctx, ldc, nb, H, dk, T, dot, dbd, ldp, relpos):
    """Row dots dctx_i . ctx_i per head and the source-less bd-gradient elements zeroed."""
    _f32(dctx, ctx, dot, dbd)
    _native.call("esp_attn_bwd_prep", _p(dctx), ldd, _p(ctx), ldc, nb, H, dk, T, _p(dot), _p(dbd), ldp, int(relpos),
                 _st())


def attn_dscores(dctx, ldd, vmat, ldv, attn, dot, dS, dbd, ldp, relpos, nb, H, dk, sqrt_dk, drop_p, seed, T, lds,
                 v_off=0):
    """dS and the rel_shift-adjoint dbd straight from the dP = dctx V^T GEMM's epilogue."""
    _f32(dctx, vmat, attn, dot, dS, dbd)
    if _PROF is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    _native.call("esp_attn_dscores", _p(dctx), ldd, _p(vmat, v_off), ldv, _p(attn), _p(dot), _p(dS), _p(dbd), ldp,
                 int(relpos), nb, H, dk, float(sqrt_dk), float(drop_p), int(seed) & (2 ** 64 - 1), T, lds, _st())
    if _PROF is not None:
        ev1.record()
        # epilogue streams besides A, B, C: P read, dbd written (band) — M x N per batch each
        _PROF.append((2.0 * T * T * dk * nb * H, ev0, ev1, (KC, KC, T, T, dk, nb * H, "dscores"),
                      8.0 * T * T * nb * H))


def relpos_probs_ok(T: int, dk: int) -> bool:
    """Whether esp_relpos_attn_probs covers this shape (d_k 64, T <= 512)."""
    return dk == 64 and T <= 512


def relpos_fused_ok(T: int, dk: int) -> bool:
    """Whether esp_relpos_softmax_fwd covers this shape (d_k 64, 32-row window in 64 KB LDS)."""
    return dk == 64 and (32 * (32 * ((T + 62) // 32) + 4) + 256) * 4 <= 65536


def attn_softmax_bwd(attn, dP, dS, drop_p, seed, sqrt_dk, rows, Tk, lds=None):
    _native.call("esp_attn_softmax_bwd", _p(attn), _p(dP), _p(dS), float(drop_p), seed, float(sqrt_dk), rows, Tk,
                 lds or Tk, _st())


def attn_softmax_bwd_relpos(attn, dP, dS, dbd, ldp, drop_p, seed, sqrt_dk, rows, T, lds, relpos=1, tvalid=None):
    """Softmax backward fused with the latest (relpos 1) or legacy (relpos 2) rel_shift adjoint
    (writes dS and dbd); tvalid: legacy length-bucket T' (device int32)."""
    _native.call("esp_attn_softmax_bwd_relpos", _p(attn), _p(dP), _p(dS), _p(dbd), ldp, int(relpos), float(drop_p),
                 seed, float(sqrt_dk), rows, T, lds, _p(tvalid), _st())


def attn_softmax_bwd_relpos_band(attn, dP, dS, dbd, ldp, drop_p, seed, sqrt_dk, rows, T, lds):
    """The latest-rel_shift adjoint writing only dbd's band (esp_attn_softmax_bwd_relpos_band); dbd must be
    a relpos_band_buffer (zero outside the band)."""
    _native.call("esp_attn_softmax_bwd_relpos_band", _p(attn), _p(dP), _p(dS), _p(dbd), ldp, float(drop_p), seed,
                 float(sqrt_dk), rows, T, lds, _st())


def relpos_dqv(dbd, ldp, p, ldpm, out, ldo, nb, H, T):
    """dq_v[z] = dbd[z] . p_h over each row tile's rel_shift band (esp_relpos_dqv; latest, d_k = 64)."""
    ws = _ws(_GEMM_WS, "esp_gemm_f32", _GEMM_WS_BYTES, out.device)
    if _PROF is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    _native.call("esp_relpos_dqv", _p(dbd), ldp, _p(p), ldpm, _p(out), ldo, nb, H, T, _p(ws), _GEMM_WS_BYTES, _st())
    _guard_post("esp_gemm_f32", ws, _GEMM_WS_BYTES)
    if _PROF is not None:  # algorithmic work: the band only (T x T of the 2T-1 columns per row)
        ev1.record()
        _PROF.append((2.0 * T * 64 * T * nb * H, ev0, ev1, (KC, RC, T, 64, T, nb * H, "band"), 0.0))


# dbd buffers of the latest rel_shift adjoint, kept per (device, Z, T, pitch) and zeroed once: the band
# kernel writes each row's T band columns only, so the rest stays 0 for every layer and step (half the
# adjoint's dbd bytes).  Made outside graph capture only (a buffer made inside would live in the graph's
# pool); a few shapes at most (length buckets), beyond that the full-row kernel.  One buffer cannot serve
# two shapes: graphs of different length buckets replay interleaved, and each writes its own band pattern,
# which is out-of-band garbage in the other's layout -- so the buffers are per shape, and bounded by a
# byte cap per device (at C2 B=256 one buffer is 1.15 GB: three shapes fit the cap), not by count alone.
# Nothing frees a buffer while the process runs (a captured graph holds its address);
# release_relpos_band_buffers() does, for tests and for a caller that has dropped its graphs.
_DBD_BUFS = {}
_DBD_MAX_SHAPES = 4
_DBD_MAX_BYTES = 4 << 30


def release_relpos_band_buffers():
    """Drop the kept dbd buffers (tests; a process that changes its batch shapes for good)."""
    _DBD_BUFS.clear()


def relpos_band_buffer(Z, T, Pp, device):
    key = (str(device), Z, T, Pp)
    buf = _DBD_BUFS.get(key)
    if buf is None:
        if len(_DBD_BUFS) >= _DBD_MAX_SHAPES or torch.cuda.is_current_stream_capturing():
            return None
        held = sum(b.numel() * 4 for k, b in _DBD_BUFS.items() if k[0] == str(device))
        if held + Z * T * Pp * 4 > _DBD_MAX_BYTES:
            return None
        buf = torch.zeros(Z * T * Pp, dtype=torch.float32, device=device)
        _DBD_BUFS[key] = buf
    return buf


FUSED_ATTN_BWD = False
# ATTN_FWD32 = True: the 32-row-block fused forward (relpos_attn_fwd_kernel, latest only) instead of
# the 16-row-wave kernel (esp_relpos_attn_probs); kept for A/B measurements
ATTN_FWD32 = False
# ATTN_DSCORES = True: the softmax / rel_shift adjoints in the dP GEMM's epilogue (esp_attn_dscores,
# FlashAttention-2's row dot) instead of the dP GEMM + the row-wise adjoint pass.  Opt-in: measured
# at C2 B=128 it is 412 + 73 us per layer against 59 + 266 (the epilogue's rel_shift scatter is one
# scalar store per element; the row-wise pass writes each shifted bd row contiguously)
ATTN_DSCORES = False
def relpos_attn_bwd(dctx, ldd, vmat, ldv, attn, dS, dbd, ldp, nb, H, sqrt_dk, drop_p, seed, T, lds, v_off=0):
    """Fused latest rel-pos attention backward: dP = dctx V^T (MFMA), dropout/softmax/rel_shift adjoints."""
    _f32(dctx, vmat, attn, dS, dbd)
    _native.call("esp_relpos_attn_bwd", _p(dctx), ldd, _p(vmat, v_off), ldv, _p(attn), _p(dS), _p(dbd), ldp, nb, H,
                 float(sqrt_dk), float(drop_p), int(seed) & (2 ** 64 - 1), T, lds, _st())


# Flash-style rel-pos attention (csrc/flash_relpos.hip), d_k = 64, T <= 512, latest and legacy.
# Opt-in (FLASH_ATTN = True): in fp32 at T' = 374 the recompute it trades for the (Z,T,T)
# probability traffic costs about what that traffic did (fp32 MFMA is 157 TF against 8 TB/s:
# 32 flop per P byte at d_k = 64), and measured per layer at C2 B=128 (tools/flash_bench.py):
# forward 0.84 vs 0.99 ms (flash wins), backward 2.10 vs 1.79 ms (materialised wins) -> off.
FLASH_ATTN = False
_DP_WS = _Workspace()


def flash_ok(T: int, dk: int) -> bool:
    return FLASH_ATTN and dk == 64 and 1 <= T <= 512


def relpos_flash_fwd(q_u, q_v, kmat, ldk, vmat, ldv, p, ldp_row, rel, nb, H, sqrt_dk, klen_i32, ctx, ldc, stats,
                     drop_p, seed, T, k_off=0, v_off=0):
    """ctx = dropout(softmax((q_u k^T + rel_shift(q_v p^T)) / sqrt_dk)) v in one kernel per
    (z, 32 rows); stats (Z, T, 2) = row max and 1/sum for the backward."""
    _f32(q_u, q_v, kmat, vmat, p, ctx, stats)
    _native.call("esp_relpos_flash_fwd", _p(q_u), _p(q_v), _p(kmat, k_off), ldk, _p(vmat, v_off), ldv, _p(p), ldp_row,
                 int(rel), nb, H, float(sqrt_dk), _p(klen_i32), _p(ctx), ldc, _p(stats), float(drop_p),
                 int(seed) & (2 ** 64 - 1), T, _st())


def relpos_flash_bwd(q_u, q_v, kmat, ldk, vmat, ldv, p, ldp_row, rel, nb, H, sqrt_dk, klen_i32, ctx, dctx, ldc,
                     stats, drop_p, seed, T, dq, ldq, dS, pdrop, lds, bias_part, carry, k_off=0, v_off=0, dq_off=0):
    _f32(q_u, q_v, kmat, vmat, p, ctx, dctx, stats, dq, dS, pdrop, bias_part, carry)
    _native.call("esp_relpos_flash_bwd", _p(q_u), _p(q_v), _p(kmat, k_off), ldk, _p(vmat, v_off), ldv, _p(p),
                 ldp_row, int(rel), nb, H, float(sqrt_dk), _p(klen_i32), _p(ctx), _p(dctx), ldc, _p(stats),
                 float(drop_p), int(seed) & (2 ** 64 - 1), T, _p(dq, dq_off), ldq, _p(dS), _p(pdrop), lds,
                 _p(bias_part), _p(carry), _st())


def relpos_dp(dS, lds, q_v, rel, nb, H, T, dp, ldp, bias_part, carry, du, dv, dq, ldq, dq_off=0):
    """linear_pos gradient input dp (P x 64H) from dS along its diagonals; pos_bias grads += the
    flash backward's column sums; legacy carries into dq."""
    _f32(dS, q_v, dp, bias_part, carry, du, dv, dq)
    n = _wsize("esp_relpos_dp", nb, H, T)
    ws = _ws(_DP_WS, "esp_relpos_dp", n, dS.device)
    _native.call("esp_relpos_dp", _p(dS), lds, _p(q_v), int(rel), nb, H, T, _p(dp), ldp, _p(bias_part), _p(carry),
                 _p(du), _p(dv), _p(dq, dq_off), ldq, _p(ws), n // 4, _st())
    _guard_post("esp_relpos_dp", ws, n)


def relshift_bwd(dS, dbd, relpos, Z, T, P, lds=None, ldp=None):
    _native.call("esp_relshift_bwd", _p(dS), lds or T, _p(dbd), ldp or P, relpos, Z, T, P, _st())


# ----------------------------------------------------------------------------- subsampling
def conv1_fwd(x, W, b, z, B, T, F, D, z16=None, zbits=None):
    """z16 (bf16, optional): the output's bf16 copy too (esp_conv1_fwd_bf16); zbits (int32, B*T1*F1*D/32,
    optional): the ReLU mask as a packed bit map too (esp_conv1_fwd_bits)."""
    if zbits is not None:
        assert zbits.dtype == torch.int32 and zbits.is_contiguous()
        _native.call("esp_conv1_fwd_bits", _p(x), _p(W), _p(b), _p(z), _p(z16) if z16 is not None else None,
                     _p(zbits), B, T, F, D, _st())
        return
    if z16 is not None:
        _native.call("esp_conv1_fwd_bf16", _p(x), _p(W), _p(b), _p(z), _p(z16), B, T, F, D, _st())
        return
    _native.call("esp_conv1_fwd", _p(x), _p(W), _p(b), _p(z), B, T, F, D, _st())


def conv2_bf16_ok(D: int) -> bool:
    """The bf16 mode runs the conv2 forward and input gradient on bf16 operands (esp_conv2_fwd_bf16 /
    esp_conv2_dgrad_bf16) when D % 64 == 0."""
    return _COMPUTE[0] == GEMM_BF16 and _AMP_BF16_OPERANDS and D % 64 == 0


def conv2_fwd_bf16(z1_16, w16, bias, z2, B, T1, F1, D):
    """z2 = ReLU(im2col(z1) W^T + b) on bf16 operands (esp_conv2_fwd_bf16)."""
    ws = _ws(_GEMM_WS, "esp_gemm_bf16", _GEMM_WS_BYTES, z2.device)
    if _PROF is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    _native.call("esp_conv2_fwd_bf16", _p(z1_16), _p(w16), _p(bias), _p(z2), B, T1, F1, D, _p(ws), _GEMM_WS_BYTES,
                 _st())
    _guard_post("esp_gemm_bf16", ws, _GEMM_WS_BYTES)
    if _PROF is not None:
        ev1.record()
        T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
        M = B * T2 * F2
        _PROF.append((2.0 * M * D * 9 * D, ev0, ev1, (I2C_KC, KC, M, D, 9 * D, 1, "bf16"), 0.0))


def col2im_relu(dcol, z1, dz1, B, T1, F1, D):
    _native.call("esp_col2im_relu", _p(dcol), _p(z1), _p(dz1), B, T1, F1, D, _st())


def im2col_nhwc(x, col, B, T1, F1, C, k, s):
    """NHWC [B, T1, F1, C] -> columns [B*T2*F2, k*k*C], (kt, kf, c) per row (esp_im2col_nhwc)."""
    _f32(x, col)
    _native.call("esp_im2col_nhwc", _p(x), _p(col), B, T1, F1, C, k, s, _st())


def col2im_relu_nhwc(dcol, z, dx, B, T1, F1, C, k, s):
    """dx = relu'(z) * the adjoint of im2col_nhwc applied to dcol (esp_col2im_relu_nhwc)."""
    _f32(dcol, z, dx)
    _native.call("esp_col2im_relu_nhwc", _p(dcol), _p(z), _p(dx), B, T1, F1, C, k, s, _st())


def conv1_wgrad(x, dz1, dW, db, B, T, F, D):
    n = _wsize("esp_conv1_wgrad", B, T, F, D)
    ws = _ws(WS, "esp_conv1_wgrad", n, x.device)
    _native.call("esp_conv1_wgrad", _p(x), _p(dz1), _p(dW), _p(db), B, T, F, D, _p(ws), n, _st())
    _guard_post("esp_conv1_wgrad", ws, n)


def permute3(inp, out, O, Bd, Ad, accumulate=False):
    _native.call("esp_permute3", _p(inp), _p(out), O, Bd, Ad, int(accumulate), _st())


# ----------------------------------------------------------------------------- losses
def log_softmax(x, y, rows, V):
    _native.call("esp_log_softmax", _p(x), _p(y), rows, V, _st())


def _need_f64(*ts):
    for t in ts:
        if t is not None and t.dtype != torch.float64:
            raise TypeError(f"espnet_slurp_amd: expected a float64 buffer, got {t.dtype}")


def ctc_loss(lp, labels, Umax, ilen_i32, tlen_i32, B, T, V, blank, gscale, zero_infinity, nll, grad):
    _need_f64(nll)
    n = _wsize("esp_ctc_loss", B, T, Umax)  # fp64 alpha / beta
    ws = _ws(WS, "esp_ctc_loss", n, lp.device)
    _native.call("esp_ctc_loss", _p(lp), _p(labels), Umax, _p(ilen_i32), _p(tlen_i32), B, T, V, blank,
                 float(gscale), int(zero_infinity), _p(nll), _p(grad), _p(ws), n, _st())
    _guard_post("esp_ctc_loss", ws, n)


def label_smoothing(x, target, V, ignore, smoothing, gscale, grad, row_loss, row_stat):
    _need_f64(row_loss)
    _native.call("esp_label_smoothing", _p(x), _p(target), target.numel(), V, ignore, float(smoothing),
                 float(gscale), _p(grad), _p(row_loss), _p(row_stat), _st())


def reduce_losses(nll, B, zero_inf, row_loss, row_stat, R, denom, ctc_w, out4):
    _need_f64(nll, row_loss)
    _native.call("esp_reduce_losses", _p(nll), B, int(zero_inf), _p(row_loss), _p(row_stat), R, float(denom),
                 float(ctc_w), _p(out4), _st())


def argmax(x, out, rows, V):
    _native.call("esp_argmax", _p(x), _p(out), rows, V, _st())


def ctc_forced_align(lpz, y, blank=0):
    """espnet1 CTC.forced_align on device: lpz (T,V) fp32 log-probs, y (U,) int64 -> (T,) int64."""
    T, V = lpz.shape
    U = y.numel()
    path = torch.empty(T * (2 * U + 1), dtype=torch.int32, device=lpz.device)
    out = torch.empty(T, dtype=torch.int64, device=lpz.device)
    _native.call("esp_ctc_forced_align", _p(lpz), T, V, _p(y), U, blank, _p(path), _p(out), _st())
    return out


def ctc_forced_align_batch(lpz, tlen, y, ulen, blank=0):
    """forced_align of every utterance of a batch in one launch: lpz (B, T, V) fp32 log-probs, tlen (B,) frames,
    y (B, Umax) labels, ulen (B,) label counts -> (B, T) int64, -1 past each utterance's frames."""
    B, T, V = lpz.shape
    Umax = y.shape[1]
    dev = lpz.device
    lpz = lpz.contiguous()
    _f32(lpz)
    y = y.to(dev).long().contiguous()
    tl = torch.as_tensor(tlen).to(device=dev, dtype=torch.int32).contiguous()
    ul = torch.as_tensor(ulen).to(device=dev, dtype=torch.int32).contiguous()
    if tl.numel() != B or ul.numel() != B or y.shape[0] != B:
        raise ValueError(f"ctc_forced_align_batch: B={B}, tlen {tl.numel()}, ulen {ul.numel()}, y {tuple(y.shape)}")
    path = torch.empty(B * T * (2 * Umax + 1), dtype=torch.int32, device=dev)
    out = torch.empty(B, T, dtype=torch.int64, device=dev)
    _native.call("esp_ctc_forced_align_batch", _p(lpz), B, T, V, _p(tl), _p(y), Umax, _p(ul), blank, _p(path),
                 _p(out), _st())
    return out


def ctc_prefix_init(lp, blank=0):
    """Initial CTC prefix state (T, 2) of the <sos> prefix for one utterance's log-probs lp (T, V)."""
    T, V = lp.shape
    r0 = torch.empty(T, 2, dtype=torch.float32, device=lp.device)
    _native.call("esp_ctc_prefix_init", _p(lp), T, V, blank, _p(r0), _st())
    return r0


def ctc_prefix_score(lp, r_prev, last, out_len, cands, blank, eos):
    """CTCPrefixScore for NH hypotheses x C candidates: r_prev (NH, T, 2), last (NH,) int64,
    cands (NH, C) int64 -> (log_psi (NH, C), r_new (NH, C, T, 2))."""
    T, V = lp.shape
    NH, C = cands.shape
    assert r_prev.shape == (NH, T, 2) and last.shape == (NH,)
    assert int(cands.min()) >= 0 and int(cands.max()) < V
    r_new = torch.empty(NH, C, T, 2, dtype=torch.float32, device=lp.device)
    psi = torch.empty(NH, C, dtype=torch.float32, device=lp.device)
    _native.call("esp_ctc_prefix_score", _p(lp), T, V, _p(r_prev), _p(last), int(out_len), _p(cands), NH, C,
                 int(blank), int(eos), _p(r_new), _p(psi), _st())
    return psi, r_new


def reserve_workspace(nbytes, device):
    WS.reserve(nbytes, device)


# ----------------------------------------------------------------------------- front end
def fbank_fwd(wave, lens_i32, B, N, n_fft, hop, window, twiddle, melw, mel_lo, mel_hi, n_mels, out, T, nvalid=None):
    """STFT -> power -> log-mel in one kernel (esp_fbank_fwd); wave (B, ldw) fp32 on device;
    nvalid: device int32, the reflection point of a length-bucketed batch."""
    _f32(wave, window, twiddle, melw, out)
    _native.call("esp_fbank_fwd", _p(wave), wave.stride(0), _p(lens_i32), B, N, n_fft, hop, _p(window), _p(twiddle),
                 _p(melw), _p(mel_lo), _p(mel_hi), n_mels, _p(out), T, _p(nvalid), _st())


def global_mvn(x, lens_i32, mean, std, norm_means=True, norm_vars=True):
    """In place: ((x - mean), padded frames zeroed) / std."""
    _f32(x, mean, std)
    B, T, F = x.shape
    _native.call("esp_global_mvn", _p(x), _p(lens_i32), B, T, F, _p(mean), _p(std), int(norm_means),
                 int(norm_vars), _st())


_ZEROS = {}
# conv2 input gradient as 4 implicit parity-class GEMMs with the ReLU mask in a specialised
# row-mapped epilogue (EPI_RMASKMAP, 128-wide tiles): 10.2 ms vs 12.4 ms for the column GEMM +
# col2im at C2 B=128 (tools/conv2_dgrad_bench.py), bench 1067 vs 1050 utt/s.  CONV2_IMPLICIT_DGRAD = False:
# the column path.
CONV2_IMPLICIT_DGRAD = True
# training: conv1 also writes its ReLU mask as a packed bit map (esp_conv1_fwd_bits) and the implicit input
# gradient's epilogue reads it (esp_conv2_dgrad_bits) instead of the fp32 map -- 1/32 of the mask bytes; about
# neutral alone (class GEMMs -58 us each, conv1 +0.1-0.2 ms), needed by CONV1_FOLD
CONV2_DGRAD_BITS = True
# training: conv1's weight gradient folded into the conv2 input gradient's epilogue (esp_conv2_dgrad_c1fold: the
# 7.7 GB conv1-map gradient of C2 B=256 is never stored nor re-read): 1470.4 vs 1458.0 utt/s with False
# (esp_conv2_dgrad_bits + esp_conv1_wgrad; profiles/r06i_bench*.log; A/B: tools/bench_with.py kernels.CONV1_FOLD=0)
CONV1_FOLD = True


def conv2_wgrad_bf16(dz2_16, z1_16, dw, db, B, T1, F1, D):
    """dw (D x 9D) = dz2^T im2col(z1), db += colsum(dz2), on bf16 operands (esp_conv2_wgrad_bf16)."""
    ws = _ws(_GEMM_WS, "esp_gemm_bf16", _GEMM_WS_BYTES, dw.device)
    if _PROF is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    _native.call("esp_conv2_wgrad_bf16", _p(dz2_16), _p(z1_16), _p(dw), _p(db), B, T1, F1, D, _p(ws), _GEMM_WS_BYTES,
                 _st())
    _guard_post("esp_gemm_bf16", ws, _GEMM_WS_BYTES)
    if _PROF is not None:
        ev1.record()
        T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
        npix = B * T2 * F2
        _PROF.append((2.0 * D * 9 * D * npix, ev0, ev1, (RC, I2C_RC, D, 9 * D, npix, 1, "bf16"), 0.0))


def conv2_dgrad_c1fold(dz2, W, z1bits, x, T, F, dW1, db1, B, T1, F1, D, dz2_16=None):
    """The implicit conv2 input gradient with conv1's weight / bias gradient folded into its epilogue
    (esp_conv2_dgrad_c1fold): dW1 (D x 9) and db1 (D) accumulate sum dz1 * x-patch and sum dz1 over the conv1
    map; dz1 is never materialised.  The mask comes from conv1_fwd's bit map; x is the conv1 input."""
    assert dz2 is not None or dz2_16 is not None
    assert z1bits.dtype == torch.int32
    _f32(dz2, W, x, dW1, db1)
    key = str(W.device)
    if key not in _ZEROS:
        _ZEROS[key] = torch.zeros(64, dtype=torch.float32, device=W.device)
    n = _wsize("esp_conv2_dgrad", D)
    wc = _ws(_WS2, "esp_conv2_dgrad", n, W.device)
    n1 = _wsize("esp_conv2_c1fold")
    w1 = _ws(_WS_C1, "esp_conv2_c1fold", n1, W.device)
    if _PROF is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    _native.call("esp_conv2_dgrad_c1fold", None if dz2_16 is not None else _p(dz2), _p(dz2_16), _p(W), _p(z1bits),
                 _p(x), T, F, _p(dW1), _p(db1), B, T1, F1, D, _p(_ZEROS[key]), _p(wc), n, _p(w1), n1, _st())
    _guard_post("esp_conv2_dgrad", wc, n)
    if _PROF is not None:  # the 4 class GEMMs (+ the records' two small reductions) as one family entry
        ev1.record()
        T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
        npix2 = B * T2 * F2
        # algorithmic bytes: dz2 (4 B, or 2 B as bf16) and W read, the bit map and the conv1 input read; no dz1
        eb = 2.0 if dz2_16 is not None else 4.0
        _PROF.append((2.0 * npix2 * 9 * D * D, ev0, ev1, (4, RC, B * T1 * F1, D, 9 * D, 1, "conv2_dgrad_c1fold"),
                      eb * npix2 * D + 4.0 * 9 * D * D + B * T1 * F1 * D / 8.0 + 4.0 * B * T * F))


def conv2_c1fold_ok(D: int) -> bool:
    """esp_conv2_dgrad_c1fold takes D % 128 == 0, D <= 512 (CONV1_FOLD: off -> esp_conv2_dgrad_bits + esp_conv1_wgrad)."""
    return CONV1_FOLD and CONV2_DGRAD_BITS and CONV2_IMPLICIT_DGRAD and D % 128 == 0 and D <= 512


def conv2_dgrad(dz2, W, z1, dz1, B, T1, F1, D, dz2_16=None, z1bits=None):
    """Conv2d(D, D, 3, 2) input gradient x conv1 ReLU mask as 4 implicit parity-class GEMMs; dz2_16 (the
    bf16 mode): dz2 as bf16, the class GEMMs on bf16 operands (esp_conv2_dgrad_bf16; dz2 may then be None);
    z1bits (conv1_fwd's bit map): the mask from it instead of z1 (esp_conv2_dgrad_bits; z1 may be None)."""
    assert dz2 is not None or dz2_16 is not None
    assert z1 is not None or z1bits is not None
    _f32(dz2, W, z1, dz1)
    key = str(W.device)
    if key not in _ZEROS:
        _ZEROS[key] = torch.zeros(64, dtype=torch.float32, device=W.device)
    n = _wsize("esp_conv2_dgrad", D)
    wc = _ws(_WS2, "esp_conv2_dgrad", n, W.device)
    if _PROF is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    if z1bits is not None:
        assert z1bits.dtype == torch.int32
        _native.call("esp_conv2_dgrad_bits", None if dz2_16 is not None else _p(dz2),
                     _p(dz2_16) if dz2_16 is not None else None, _p(W), _p(z1bits), _p(dz1), B, T1, F1, D,
                     _p(_ZEROS[key]), _p(wc), n, _st())
    elif dz2_16 is not None:
        _native.call("esp_conv2_dgrad_bf16", _p(dz2_16), _p(W), _p(z1), _p(dz1), B, T1, F1, D, _p(_ZEROS[key]), _p(wc),
                     n, _st())
    else:
        _native.call("esp_conv2_dgrad", _p(dz2), _p(W), _p(z1), _p(dz1), B, T1, F1, D, _p(_ZEROS[key]), _p(wc), n,
                     _st())
    _guard_post("esp_conv2_dgrad", wc, n)
    if _PROF is not None:  # the 4 class GEMMs as one family entry: A = dz2 (gathered), B = W, C = dz1 + ReLU mask read
        ev1.record()
        T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
        npix2 = B * T2 * F2
        # algorithmic bytes (the whole entry): dz2 and W read, z1 (ReLU mask) read, dz1 written
        _PROF.append((2.0 * npix2 * 9 * D * D, ev0, ev1, (4, RC, B * T1 * F1, D, 9 * D, 1, "conv2_dgrad"),
                      4.0 * (npix2 * D + 9 * D * D + 2 * B * T1 * F1 * D)))
