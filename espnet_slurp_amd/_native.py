"""ctypes loader for libespnet_mi355.so (the C ABI in include/espnet_mi355.h).

There is no CPU fallback: if the library is missing or cannot be loaded, importing the
compute path raises.  Build it with `make -C espnet_slurp_amd/csrc` (or
`__graft_entry__.build()`).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ESP_LIB_VARIANT=_x: an experiment build of the same sources (make VARIANT=_x EXTRA=-D...), for
# A/B runs on one box
LIB_PATH = os.path.join(_HERE, "libespnet_mi355%s.so" % os.environ.get("ESP_LIB_VARIANT", ""))

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float
U64 = ctypes.c_ulonglong

# name -> argtypes (all return int status unless listed in _RESTYPES)
SIGNATURES = {
    "esp_last_error": [],
    "esp_abi_version": [],
    "esp_gemm_bf16": [I, I, I, I, I, I, I, P, L, L, L, P, L, L, L, P, L, L, L, P, F, F, P, I, P, F, U64, I, P, P, P, L,
                      P],
    "esp_gemm_bf16_pl": [I, I, I, I, I, I, I, P, L, L, L, P, L, L, L, P, L, L, L, P, F, F, I, P, F, U64, I, P, I,
                         L, P, L, P],
    "esp_f32_to_bf16": [P, P, L, I, L, L, I, P],
    "esp_conv2_fwd_bf16": [P, P, P, P, I, I, I, I, P, L, P],
    "esp_conv2_dgrad_bf16": [P, P, P, P, I, I, I, I, P, P, L, P],
    "esp_conv1_fwd_bf16": [P, P, P, P, P, I, I, I, I, P],
    "esp_conv2_wgrad_bf16": [P, P, P, P, I, I, I, I, P, L, P],
    "esp_gemm_f32": [I, I, I, I, I, I, I, P, L, L, L, P, L, L, L, P, L, L, L, P, F, F, P, I, P, F, U64, I, P, P,
                     P, P, P, L, P],
    "esp_gemm_f32_bp": [I, I, I, I, I, I, I, P, L, L, L, P, L, L, L, P, L, L, L, P, F, F, P, I, P, F, U64, I, P, P,
                        P, P, L, P, L, L, L, L, P],
    "esp_f32_to_planes": [P, P, L, I, L, L, L, P],
    "esp_gemm_f32_pl": [I, I, I, I, I, I, I, P, L, L, L, P, L, L, L, L, P, L, L, L, P, L, L, L, L, P, L, L, L, P, F, F,
                        P, I, P, F, U64, I, P, P, I, L, P, L, P],
    "esp_set_gemm_compute": [I],
    "esp_get_gemm_compute": [],
    "esp_f32_gemm_products": [],
    "esp_set_splitk_mode": [I],
    "esp_act_bwd": [P, P, P, L, I, F, U64, L, P],
    "esp_scale_dropout": [P, P, L, F, F, U64, P, F, P],
    "esp_scale_dropout_planes": [P, P, L, L, I, F, F, U64, P],
    "esp_scale_by_dev": [P, L, P, P],
    "esp_embed_fwd": [P, P, P, P, I, I, I, F, F, U64, P],
    "esp_embed_bwd": [P, P, P, I, I, I, F, F, U64, P],
    "esp_specaug": [P, P, I, I, I, P, P, P, I, P, I, P],
    "esp_utterance_mvn": [P, I, I, I, P, P],
    "esp_grad_norm": [P, L, F, P, L, P, P],
    "esp_adam": [P, P, P, P, L, P, F, ctypes.c_double, ctypes.c_double, F, F, I, P],
    "esp_opt_hyper": [P, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, P, P],
    "esp_adam_dev": [P, P, P, P, L, P, P, ctypes.c_double, ctypes.c_double, F, F, P],
    "esp_adam_amsgrad": [P, P, P, P, P, L, P, F, ctypes.c_double, ctypes.c_double, F, F, I, P],
    "esp_adam_dev_amsgrad": [P, P, P, P, P, L, P, P, ctypes.c_double, ctypes.c_double, F, F, P],
    "esp_opt_advance": [P, P, P],
    "esp_set_rng_key": [P],
    "esp_rng_advance": [P, P],
    "esp_layernorm_fwd": [P, P, P, P, P, P, I, I, F, P],
    "esp_layernorm_fwd_planes": [P, P, P, P, L, L, I, P, P, I, I, F, P],
    "esp_layernorm_fwd_dual": [P, P, P, P, P, L, L, I, P, P, I, I, F, P],
    "esp_layernorm_bwd": [P, P, P, P, P, P, I, P, P, I, I, P, L, P],
    "esp_colsum": [P, I, I, L, P, I, P, L, P],
    "esp_glu_fwd": [P, P, L, I, P],
    "esp_glu_bwd": [P, P, P, L, I, P],
    "esp_glu_bwd_planes": [P, P, P, L, I, L, I, P],
    "esp_dwconv1d": [P, P, P, P, I, I, I, I, I, P, P],
    "esp_dwconv1d_wgrad": [P, P, P, I, I, I, I, P, L, P, P],
    "esp_bn_swish_fwd": [P, P, P, P, P, P, P, P, F, F, I, I, P, L, I, P, P],
    "esp_bn_swish_eval": [P, P, P, P, P, P, F, I, I, P, P, P],
    "esp_bn_swish_fwd_planes": [P, P, P, P, L, L, I, P, P, P, P, F, F, I, I, P, L, I, P, P],
    "esp_bn_swish_bwd": [P, P, P, P, P, P, P, P, P, I, I, P, L, P, I, P, P],
    "esp_heads_split": [P, L, I, I, I, I, I, P, P, P],
    "esp_heads_split2": [P, L, I, I, I, I, I, P, P, P, P, P],
    "esp_add2d": [P, L, P, L, I, I, P],
    "esp_attn_softmax_fwd": [P, P, I, I, F, P, I, I, P, P, F, U64, I, I, I, L, L, P, P],
    "esp_attn_softmax_bwd": [P, P, P, F, U64, F, L, I, L, P],
    "esp_relshift_bwd": [P, L, P, L, I, I, I, I, P],
    "esp_relpos_softmax_fwd": [P, P, L, I, I, P, F, P, P, P, F, U64, I, L, P],
    "esp_relpos_attn_fwd": [P, P, P, L, P, L, I, I, F, P, P, P, F, U64, I, L, P],
    "esp_relpos_attn_probs": [P, P, P, L, P, L, I, I, I, F, P, P, P, F, U64, I, L, P, P],
    "esp_attn_bwd_prep": [P, L, P, L, I, I, I, I, P, P, L, I, P],
    "esp_attn_dscores": [P, L, P, L, P, P, P, P, L, I, I, I, I, F, F, U64, I, L, P],
    "esp_attn_softmax_bwd_relpos": [P, P, P, P, L, I, F, U64, F, L, I, L, P, P],
    "esp_attn_softmax_bwd_relpos_band": [P, P, P, P, L, F, U64, F, L, I, L, P],
    "esp_relpos_dqv": [P, L, P, L, P, L, I, I, I, P, L, P],
    "esp_relpos_attn_bwd": [P, L, P, L, P, P, P, L, I, I, F, F, U64, I, L, P],
    "esp_relpos_flash_fwd": [P, P, P, L, P, L, P, L, I, I, I, F, P, P, L, P, F, U64, I, P],
    "esp_relpos_flash_bwd": [P, P, P, L, P, L, P, L, I, I, I, F, P, P, P, L, P, F, U64, I, P, L, P, P, L, P, P, P],
    "esp_relpos_dp": [P, L, P, I, I, I, I, P, L, P, P, P, P, P, L, P, L, P],
    "esp_fbank_fwd": [P, L, P, I, I, I, I, P, P, P, P, P, I, P, I, P, P],
    "esp_global_mvn": [P, P, I, I, I, P, P, I, I, P],
    "esp_conv2_dgrad": [P, P, P, P, I, I, I, I, P, P, L, P],
    "esp_conv1_fwd": [P, P, P, P, I, I, I, I, P],
    "esp_conv1_fwd_bits": [P, P, P, P, P, P, I, I, I, I, P],
    "esp_conv2_dgrad_bits": [P, P, P, P, P, I, I, I, I, P, P, L, P],
    "esp_conv2_dgrad_c1fold": [P, P, P, P, P, I, I, P, P, I, I, I, I, P, P, L, P, L, P],
    "esp_conv2_c1fold_workspace_bytes": [],
    "esp_col2im_relu": [P, P, P, I, I, I, I, P],
    "esp_conv1_wgrad": [P, P, P, P, I, I, I, I, P, L, P],
    "esp_permute3": [P, P, I, I, I, I, P],
    "esp_im2col_nhwc": [P, P, I, I, I, I, I, I, P],
    "esp_col2im_relu_nhwc": [P, P, P, I, I, I, I, I, I, P],
    "esp_log_softmax": [P, P, L, I, P],
    "esp_ctc_loss": [P, P, I, P, P, I, I, I, I, F, I, P, P, P, L, P],
    "esp_label_smoothing": [P, P, L, I, I, F, F, P, P, P, P],
    "esp_reduce_losses": [P, I, I, P, P, I, F, F, P, P],
    "esp_argmax": [P, P, L, I, P],
    "esp_ctc_forced_align": [P, I, I, P, I, I, P, P, P],
    "esp_attn_slot_check_errors": [],
    "esp_ctc_forced_align_batch": [P, I, I, I, P, P, I, P, I, P, P, P],
    "esp_ctc_prefix_init": [P, I, I, I, P, P],
    "esp_ctc_prefix_score": [P, I, I, P, P, I, P, I, I, I, I, P, P, P],
    # workspace-size queries (host arithmetic; return bytes)
    "esp_grad_norm_workspace_bytes": [L],
    "esp_layernorm_bwd_workspace_bytes": [I, I],
    "esp_colsum_workspace_bytes": [I, I],
    "esp_dwconv1d_wgrad_workspace_bytes": [I, I, I, I],
    "esp_bn_swish_fwd_workspace_bytes": [I, I],
    "esp_bn_swish_bwd_workspace_bytes": [I, I],
    "esp_conv1_wgrad_workspace_bytes": [I, I, I, I],
    "esp_conv2_dgrad_workspace_bytes": [I],
    "esp_ctc_loss_workspace_bytes": [I, I, I],
    "esp_relpos_dp_workspace_bytes": [I, I, I],
}
_RESTYPES = {"esp_last_error": ctypes.c_char_p, "esp_abi_version": I, "esp_attn_slot_check_errors": I, "esp_set_gemm_compute": I,
             "esp_get_gemm_compute": I, "esp_set_splitk_mode": I,
             "esp_f32_gemm_products": I}
_RESTYPES.update({k: L for k in SIGNATURES if k.endswith("_workspace_bytes")})
ABI_VERSION = 32  # bumped whenever a signature in include/espnet_mi355.h changes

_lib = None


def load() -> ctypes.CDLL:
    """Load the native library once; raise loudly when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"espnet_slurp_amd: native library not found at {LIB_PATH}; "
            "build it with `make -C espnet_slurp_amd/csrc` (no CPU fallback exists)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, I)
    if lib.esp_abi_version() != ABI_VERSION:
        raise RuntimeError(f"espnet_slurp_amd: {LIB_PATH} has ABI {lib.esp_abi_version()}, expected "
                           f"{ABI_VERSION}; rebuild with `make -C espnet_slurp_amd/csrc`")
    _lib = lib
    return lib


class NativeError(RuntimeError):
    pass


def workspace_bytes(launcher: str, *dims) -> int:
    """Bytes of scratch the launcher `launcher` needs for these sizes (esp_<op>_workspace_bytes):
    the same host code that picks the launcher's chunking answers, so callers never restate it."""
    n = getattr(load(), launcher + "_workspace_bytes")(*dims)
    if n < 0:
        raise NativeError(f"{launcher}_workspace_bytes{dims} failed")
    return int(n)


def call(name: str, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.esp_last_error().decode(errors="replace")
        raise NativeError(f"{name} failed ({rc}): {msg}")
    return rc
