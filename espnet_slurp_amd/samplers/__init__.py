from ._core import (BATCH_TYPES, AbsSampler, FoldedBatchSampler, LengthBatchSampler, NumElementsBatchSampler,
                    SortedBatchSampler, UnsortedBatchSampler, build_batch_sampler)

__all__ = ["AbsSampler", "FoldedBatchSampler", "LengthBatchSampler", "NumElementsBatchSampler",
           "SortedBatchSampler", "UnsortedBatchSampler", "build_batch_sampler", "BATCH_TYPES"]
