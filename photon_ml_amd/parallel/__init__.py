from .dist import (DistributedGLMData, all_reduce_, all_reduce_scalar, barrier, init_distributed, is_dist, rank,
                   world_size)

__all__ = ["DistributedGLMData", "all_reduce_", "all_reduce_scalar", "barrier", "init_distributed", "is_dist",
           "rank", "world_size"]
