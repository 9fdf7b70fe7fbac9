"""Import shim for the read-only reference (fixture generation ONLY, this container only).

The reference (BriansIDP/espnet_slurp at /root/reference) does not import as shipped
(SURVEY.md §0.1).  This module installs in-memory stubs for six absent third-party
packages and five semantics-preserving fork-skew shims, then
exposes the reference's own classes.  Nothing here is imported by the product package,
by `-m gpu` tests, by smoke() or by bench.py: the GPU box has no /root/reference.
"""
import os
import sys
import types

REF = "/root/reference"


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install():
    if "espnet2.asr.espnet_model" in sys.modules:
        return
    sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

    class _Raiser:
        def __getattr__(self, k):
            raise ImportError("stubbed third-party module (not on the hot path)")

    _stub("typeguard", check_argument_types=lambda *a, **k: True,
          check_return_type=lambda *a, **k: True, check_type=lambda *a, **k: None)
    _stub("humanfriendly", format_timespan=str, format_size=str)
    def _levenshtein(a, b):  # editdistance.eval: unit-cost edit distance over two sequences
        a, b = list(a), list(b)
        prev = list(range(len(b) + 1))
        for i, x in enumerate(a, 1):
            cur = [i] + [0] * len(b)
            for j, y in enumerate(b, 1):
                cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
            prev = cur
        return prev[-1]

    _stub("editdistance", eval=_levenshtein)
    lib = _stub("librosa")
    lib.filters = _Raiser()
    lib.util = _Raiser()
    tc = _stub("torch_complex")
    tct = _stub("torch_complex.tensor")

    class ComplexTensor:  # noqa: D401 - placeholder, raises on use
        def __init__(self, *a, **k):
            raise ImportError("torch_complex stub")

    tct.ComplexTensor = ComplexTensor
    tc.tensor = tct
    tc.ComplexTensor = ComplexTensor
    tcf = _stub("torch_complex.functional")
    tc.functional = tcf
    ident = lambda *a, **k: (a[0] if (len(a) == 1 and callable(a[0])) else (lambda f: f))
    _stub("numba", jit=ident, njit=ident, prange=range)

    if REF not in sys.path:
        sys.path.insert(0, REF)

    import torch
    import espnet.nets.pytorch_backend.transformer.subsampling as sub

    class Conv2dSubsampling2(torch.nn.Module):  # S1: only reachable for input_layer=conv2d2
        def __init__(self, *a, **k):
            raise NotImplementedError("conv2d2 not in this fork")

    sub.Conv2dSubsampling2 = Conv2dSubsampling2
    import espnet.nets.pytorch_backend.transducer.utils as tu  # S2

    tu.select_k_expansions = None
    tu.subtract = None

    import espnet.nets.pytorch_backend.transformer.repeat as rp

    _orig_repeat = rp.repeat

    def repeat(N, fn, layer_drop_rate=0.0):  # S3
        assert layer_drop_rate == 0.0
        return _orig_repeat(N, fn)

    import espnet.nets.pytorch_backend.nets_utils as nu

    _orig_mpm = nu.make_pad_mask

    def make_pad_mask(lengths, xs=None, length_dim=-1, maxlen=None):  # S5
        if maxlen is not None:
            assert xs is None
            ref = torch.zeros(len(lengths), int(maxlen))
            return _orig_mpm(lengths, ref, length_dim)
        return _orig_mpm(lengths, xs, length_dim)

    from espnet.nets.pytorch_backend.conformer.encoder_layer import EncoderLayer as _EL

    class EncoderLayer(_EL):  # S4
        def __init__(self, *args):
            if len(args) == 9:
                assert args[8] == 0.0
                args = args[:8]
            super().__init__(*args)

    import espnet2.asr.encoder.conformer_encoder as ce
    import espnet2.asr.decoder.transformer_decoder as td
    import espnet2.asr.encoder.transformer_encoder as te

    ce.repeat = repeat
    ce.EncoderLayer = EncoderLayer
    td.repeat = repeat
    td.make_pad_mask = make_pad_mask
    te.repeat = repeat
    import espnet2.asr.espnet_model  # noqa: F401
