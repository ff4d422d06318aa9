"""Multi-GPU execution: batch data parallelism over RCCL (see dist.py)."""
from .dist import (BatchDataParallel, DistContext, all_gather_array, all_gather_object, all_reduce_max,  # noqa: F401
                   all_reduce_min, barrier, broadcast_object, init_distributed, shard, shutdown)
