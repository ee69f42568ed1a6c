from .dist import (DistInfo, init_distributed, info, is_initialized, barrier, all_reduce_mean,
                   all_reduce_max, destroy)
from .ddp import DataParallelEngine
from .sampler import DistributedSampler, InfiniteRandomSampler

__all__ = ["DistInfo", "init_distributed", "info", "is_initialized", "barrier", "all_reduce_mean",
           "all_reduce_max", "destroy", "DataParallelEngine", "DistributedSampler",
           "InfiniteRandomSampler"]
