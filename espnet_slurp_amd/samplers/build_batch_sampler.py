"""Import path of espnet2/samplers/build_batch_sampler.py; implementation in samplers/_core.py."""
from ._core import build_batch_sampler  # noqa: F401
