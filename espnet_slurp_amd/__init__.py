"""espnet_slurp_amd — MI355X-native (gfx950) drop-in for the ESPnet2 ASR training step of
BriansIDP/espnet_slurp: Conformer/Transformer encoder, Transformer decoder, hybrid
CTC/attention loss, SpecAug/UtteranceMVN, fused Adam + WarmupLR, data-parallel over RCCL.

Compute lives in libespnet_mi355.so (hand-written HIP for CDNA4, C ABI in
include/espnet_mi355.h); PyTorch supplies device memory, streams and torch.distributed.
"""
__version__ = "0.1.0"
