"""Import path of espnet2/samplers/num_elements_batch_sampler.py; implementation in samplers/_core.py."""
from ._core import NumElementsBatchSampler  # noqa: F401
