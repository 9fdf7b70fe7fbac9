"""Import path of espnet2/samplers/length_batch_sampler.py; implementation in samplers/_core.py."""
from ._core import LengthBatchSampler  # noqa: F401
