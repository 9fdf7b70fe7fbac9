"""Import path of espnet2/samplers/folded_batch_sampler.py; implementation in samplers/_core.py."""
from ._core import FoldedBatchSampler  # noqa: F401
