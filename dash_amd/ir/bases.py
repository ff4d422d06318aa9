"""CRT and mixed-radix (MRS) bases.

Reference: misc/util.h:64-79 (prime table), garbled_circuit_interface.h:851-864
(compute_max_modulus), :888-930 (MRS lookup by CRT size and ReLU accuracy),
benchmarks/model_benchmarks/non_sgx/main.cpp:32-71 (optimized / CPM bases).
"""
from __future__ import annotations

from functools import reduce

PRIMES_100 = [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61, 67, 71, 73, 79, 83, 89, 97, 101,
              103, 107, 109, 113, 127, 131, 137, 139, 149, 151, 157, 163, 167, 173, 179, 181, 191, 193, 197, 199, 211,
              223, 227, 229, 233, 239, 241, 251, 257, 263, 269, 271, 277, 281, 283, 293, 307, 311, 313, 317, 331, 337,
              347, 349, 353, 359, 367, 373, 379, 383, 389, 397, 401, 409, 419, 421, 431, 433, 439, 443, 449, 457, 461,
              463, 467, 479, 487, 491, 499, 503, 509, 521, 523, 541]

# (k, accuracy%) -> MRS base (most significant digit first)
MRS_TABLE = {
    (4, 100.0): [26, 3], (4, 99.0): [18, 3],
    (5, 100.0): [54, 4, 3], (5, 99.9): [30, 5, 3], (5, 99.0): [36, 3],
    (6, 100.0): [60, 5, 5, 5], (6, 99.99): [42, 5, 5, 5], (6, 99.9): [48, 5, 4], (6, 99.0): [40, 3],
    (7, 100.0): [86, 7, 6, 6, 5], (7, 99.99): [88, 6, 5, 4], (7, 99.9): [60, 5, 4], (7, 99.0): [40, 3],
    (8, 100.0): [98, 9, 8, 8, 7, 5], (8, 99.999): [102, 7, 6, 5, 5], (8, 99.99): [78, 7, 5, 4],
    (8, 99.9): [78, 5, 3], (8, 99.0): [126],
    (9, 100.0): [76, 7, 7, 7, 7, 7, 5, 5], (9, 99.999): [114, 7, 6, 5, 5], (9, 99.99): [84, 6, 5, 5],
    (9, 99.9): [140, 9], (9, 99.0): [138],
    (10, 100.0): [202, 11, 11, 6, 6, 6, 6, 5, 5], (10, 99.999): [102, 7, 6, 6, 5], (10, 99.99): [112, 6, 5, 4],
    (10, 99.9): [190, 7], (10, 99.0): [140],
    (11, 100.0): [150, 8, 7, 7, 6, 6, 6, 5, 5, 5, 5, 5], (11, 99.999): [130, 7, 6, 5, 5], (11, 99.99): [174, 11, 7],
}

# ReDash optimized bases (benchmarks/model_benchmarks/non_sgx/main.cpp:39-50)
OPTIMIZED_BASES = {
    "MODEL_F_MINIONN_POOL_REPL": {"crt": [32, 97, 107], "mrs": [22, 19, 15, 13]},
    "MODEL_F_GNNP_POOL_REPL": {"crt": [32, 167, 173], "mrs": [26, 25, 21, 13]},
}
# ReDash CPM bases: first 7 primes with crt[0] replaced by the scale factor
CPM_MRS = [10, 9, 9, 8, 7, 7, 6]


def first_primes(k: int) -> list[int]:
    if not 0 < k <= 100:
        raise ValueError("k must be in [1, 100]")
    return PRIMES_100[:k]


def crt_modulus(base) -> int:
    return reduce(lambda a, b: a * b, base, 1)


def get_mrs_base(k: int, accuracy: float) -> list[int]:
    for (kk, acc), v in MRS_TABLE.items():
        if kk == k and abs(acc - accuracy) < 1e-9:
            return list(v)
    raise KeyError(f"no MRS base for k={k}, accuracy={accuracy}")


def compute_max_modulus(crt, mrs) -> int:
    """Largest modulus any gadget needs (the reference's formula, but using the
    largest CRT modulus rather than crt[0])."""
    m = max(crt)
    if mrs:
        m = max(m, max(mrs))
        k = len(crt)
        for d in range(1, len(mrs)):
            m = max(m, (k + 1) * mrs[d])
    return m
