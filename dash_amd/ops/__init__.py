"""Label-tensor level operations (host) and direct access to device primitives."""
from .labels import LabelTensor  # noqa: F401


def hip_aes_hash(blocks):
    """Fixed-key AES-128 of (n, 2) uint64 blocks on the GPU (the evaluator's T-table AES)."""
    from ..native import native

    return native().hip_aes_hash_array(blocks)


def hip_aes_throughput(blocks: int = 2048, iters: int = 2000):
    """(ms, AES/s) of the device AES implementation under full occupancy."""
    from ..native import native

    return native().hip_aes_bench(blocks, iters)
