"""Import path of espnet2/samplers/unsorted_batch_sampler.py; implementation in samplers/_core.py."""
from ._core import UnsortedBatchSampler  # noqa: F401
