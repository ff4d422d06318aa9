"""Multi-GPU execution: batch data parallelism over RCCL (see dist.py)."""
from .dist import (BatchDataParallel, DistContext, all_gather_array, all_reduce_max, barrier,  # noqa: F401
                   broadcast_object, init_distributed, shard, shutdown)
