"""Import path of espnet2/samplers/sorted_batch_sampler.py; implementation in samplers/_core.py."""
from ._core import SortedBatchSampler  # noqa: F401
