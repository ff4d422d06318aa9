"""LabelTensor: a CRT-decomposed tensor of garbled labels (host side).

Reference: garbling/label_tensor.h (C15). One `Labels` block per CRT residue
p_j, each an int16 array [N, n_p] (label-major, the layout of the host
garbler/evaluator; the GPU uses the component-major transpose). Arithmetic
is component-wise mod p; compress/decompress/hash go through the native
codec and AES-NI code, so results are bit-identical with the evaluators.

    L = LabelTensor.from_labels(gc.garble_inputs(x), shape=(3, 32, 32))
    y = (L + L) * 3            # label arithmetic mod p
    C = y.compress()           # (k, N, 2) uint64, the 16-B wire form
    H = y.hash()               # fixed-key AES of every compressed label
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from ..native import native


class LabelTensor:
    def __init__(self, moduli: Sequence[int], blocks: Sequence[np.ndarray], shape: Sequence[int] = None):
        self.moduli = [int(p) for p in moduli]
        self.blocks = [np.ascontiguousarray(b, dtype=np.int16) for b in blocks]
        n = native()
        N = self.blocks[0].shape[0] if self.blocks else 0
        for p, b in zip(self.moduli, self.blocks):
            assert b.ndim == 2 and b.shape == (N, n.nr_comps(p)), "block shape must be (N, n_p)"
        self.shape = tuple(shape) if shape is not None else (N,)
        assert int(np.prod(self.shape)) == N, "shape does not match the number of labels"

    # ---------------------------------------------------------------- build
    @classmethod
    def from_labels(cls, labels, shape=None) -> "LabelTensor":
        return cls([p for p, _ in labels], [a for _, a in labels], shape)

    def to_labels(self) -> list:
        return [(p, b) for p, b in zip(self.moduli, self.blocks)]

    @classmethod
    def zeros(cls, moduli, shape) -> "LabelTensor":
        N = int(np.prod(shape))
        n = native()
        return cls(moduli, [np.zeros((N, n.nr_comps(p)), np.int16) for p in moduli], shape)

    @classmethod
    def random(cls, moduli, shape, rng=None) -> "LabelTensor":
        rng = rng or np.random.default_rng()
        N = int(np.prod(shape))
        n = native()
        return cls(moduli, [rng.integers(0, p, (N, n.nr_comps(p))).astype(np.int16) for p in moduli], shape)

    @property
    def size(self) -> int:
        return int(np.prod(self.shape))

    def __len__(self):
        return self.size

    def reshape(self, *shape) -> "LabelTensor":
        shape = shape[0] if len(shape) == 1 and isinstance(shape[0], (tuple, list)) else shape
        return LabelTensor(self.moduli, self.blocks, shape)

    def __getitem__(self, idx) -> "LabelTensor":
        flat = np.arange(self.size).reshape(self.shape)[idx].reshape(-1)
        return LabelTensor(self.moduli, [b[flat] for b in self.blocks], (flat.size,))

    # ----------------------------------------------------------- arithmetic
    def _binary(self, other, sign: int) -> "LabelTensor":
        assert isinstance(other, LabelTensor) and other.moduli == self.moduli
        o = other.blocks
        if other.size == 1 and self.size > 1:  # broadcast a single label (up/downshift)
            o = [np.broadcast_to(b, s.shape) for b, s in zip(o, self.blocks)]
        out = [((a.astype(np.int32) + sign * b.astype(np.int32)) % p).astype(np.int16)
               for a, b, p in zip(self.blocks, o, self.moduli)]
        return LabelTensor(self.moduli, out, self.shape)

    def __add__(self, other):
        return self._binary(other, 1)

    def __sub__(self, other):
        return self._binary(other, -1)

    def __neg__(self):
        return LabelTensor(self.moduli, [((-b.astype(np.int32)) % p).astype(np.int16)
                                         for b, p in zip(self.blocks, self.moduli)], self.shape)

    def __mul__(self, c):
        """Scalar or per-element integer multiple (reference operator*=)."""
        c = np.asarray(c, dtype=np.int64)
        out = []
        for b, p in zip(self.blocks, self.moduli):
            cc = (c % p).reshape(-1, 1) if c.ndim else np.int64(c % p)
            out.append(((b.astype(np.int64) * cc) % p).astype(np.int16))
        return LabelTensor(self.moduli, out, self.shape)

    __rmul__ = __mul__

    def matvecmul(self, W: np.ndarray) -> "LabelTensor":
        """out[o] = sum_i W[o, i] * L[i] (mod p), W public integers. Reference: label_tensor.h:783-818."""
        W = np.asarray(W, dtype=np.int64)
        assert W.shape[1] == self.size
        out = []
        for b, p in zip(self.blocks, self.moduli):
            out.append(((W % p) @ b.astype(np.int64) % p).astype(np.int16))
        return LabelTensor(self.moduli, out, (W.shape[0],))

    # ------------------------------------------------------------- codecs
    def compress(self) -> np.ndarray:
        """(k, N, 2) uint64 compressed labels C = sum_c L_c p^c."""
        return native().compress_labels(self.to_labels())

    @classmethod
    def decompress(cls, C: np.ndarray, moduli, shape=None) -> "LabelTensor":
        return cls.from_labels(native().decompress_labels(np.asarray(C, dtype=np.uint64), list(moduli)), shape)

    def hash(self) -> np.ndarray:
        """(k, N, 2) uint64 fixed-key AES-128 of every compressed label."""
        C = self.compress()
        k, N, _ = C.shape
        return native().aes_hash_array(C.reshape(k * N, 2)).reshape(k, N, 2)

    def colors(self) -> np.ndarray:
        """(k, N) point-and-permute colors (component 0)."""
        return np.stack([b[:, 0].astype(np.int64) for b in self.blocks])

    def __eq__(self, other) -> bool:  # type: ignore[override]
        return (isinstance(other, LabelTensor) and self.moduli == other.moduli
                and all(np.array_equal(a, b) for a, b in zip(self.blocks, other.blocks)))

    def __repr__(self) -> str:
        return f"LabelTensor(moduli={self.moduli}, shape={self.shape})"
