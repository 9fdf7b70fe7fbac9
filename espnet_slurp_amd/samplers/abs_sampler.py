"""Import path of espnet2/samplers/abs_sampler.py; implementation in samplers/_core.py."""
from ._core import AbsSampler  # noqa: F401
