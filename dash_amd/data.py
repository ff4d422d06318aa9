"""Datasets: native MNIST / CIFAR-10 readers, normalization, quantization,
synthetic inputs. Reference: misc/dataloader.h (C14).

Images are float32 in [0, 1], layout [N][C][H][W] (the layout every layer
uses; the reference's ScalarTensor {W, H, C} with dims[0] fastest is the same
memory order). The raw files are the standard distribution formats
(`t10k-images-idx3-ubyte`, `test_batch.bin`, ...); there is no download step
on the target machines (no network), so paths must point at local copies.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from .ir.quant import QuantizationMethod, quantize_input
from .native import native

CIFAR10_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR10_STD = (0.2470, 0.2435, 0.2616)
MNIST_MEAN = (0.1307,)
MNIST_STD = (0.3081,)


@dataclass
class Dataset:
    train_images: np.ndarray  # float32 [N, C, H, W]
    train_labels: np.ndarray  # int64 [N]
    test_images: np.ndarray
    test_labels: np.ndarray


def _wrap(raw) -> Dataset:
    (trx, try_), (tex, tey) = raw
    f = lambda a: np.asarray(a, dtype=np.float32) / 255.0  # noqa: E731
    return Dataset(f(trx), np.asarray(try_, np.int64), f(tex), np.asarray(tey, np.int64))


def mnist(path: str) -> Dataset:
    """Reference: dataloader.h:48-77 (28x28x1, /255)."""
    return _wrap(native().load_mnist(str(path)))


def cifar10(path: str) -> Dataset:
    """Reference: dataloader.h:79-121 (32x32x3, /255)."""
    return _wrap(native().load_cifar10(str(path)))


def normalize(images: np.ndarray, mean: Sequence[float], std: Sequence[float]) -> np.ndarray:
    """Per-channel (x - mean) / std. Reference: dataloader.h:142-173."""
    x = np.asarray(images, dtype=np.float32)
    m = np.asarray(mean, np.float32).reshape(1, -1, 1, 1)
    s = np.asarray(std, np.float32).reshape(1, -1, 1, 1)
    assert x.ndim == 4 and x.shape[1] == m.shape[1], "mean/std size mismatch"
    return (x - m) / s


def normalize_dataset(d: Dataset, mean, std) -> Dataset:
    return Dataset(normalize(d.train_images, mean, std) if d.train_images.size else d.train_images, d.train_labels,
                   normalize(d.test_images, mean, std), d.test_labels)


def quantize(images: np.ndarray, q_method: QuantizationMethod = QuantizationMethod.SimpleQuant,
             q_parameter: int = -1, q_const: float = 1.0) -> np.ndarray:
    """Quantize a batch of float images to int64 circuit inputs (flattened per
    image). Reference: dataloader.h:123-140, 176-197."""
    x = np.asarray(images, dtype=np.float32)
    return np.stack([quantize_input(v.reshape(-1), QuantizationMethod(q_method), q_parameter, q_const) for v in x])


def synthetic(shape: Sequence[int], n: int, seed: int = 0, normalized: bool = True) -> np.ndarray:
    """Synthetic images of the given (C, H, W): uniform pixels in [0,1],
    optionally normalized with the CIFAR/MNIST statistics."""
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 256, size=(n, *shape)).astype(np.float32) / 255.0
    if normalized:
        if shape[0] == 3:
            x = normalize(x, CIFAR10_MEAN, CIFAR10_STD)
        elif shape[0] == 1:
            x = normalize(x, MNIST_MEAN, MNIST_STD)
    return x


def write_mnist(path: str, images: np.ndarray, labels: np.ndarray, prefix: str = "t10k") -> None:
    """Write uint8 images [N,1,28,28] / labels in the idx format (fixtures)."""
    import os

    os.makedirs(path, exist_ok=True)
    im = np.asarray(images, np.uint8)
    n, _, h, w = im.shape
    with open(f"{path}/{prefix}-images-idx3-ubyte", "wb") as f:
        f.write(np.array([0x803, n, h, w], dtype=">u4").tobytes())
        f.write(im.tobytes())
    with open(f"{path}/{prefix}-labels-idx1-ubyte", "wb") as f:
        f.write(np.array([0x801, n], dtype=">u4").tobytes())
        f.write(np.asarray(labels, np.uint8).tobytes())


def write_cifar10(path: str, images: np.ndarray, labels: np.ndarray, name: str = "test_batch.bin") -> None:
    """Write uint8 images [N,3,32,32] / labels as a CIFAR-10 binary batch."""
    import os

    os.makedirs(path, exist_ok=True)
    im = np.asarray(images, np.uint8).reshape(len(images), -1)
    rec = np.concatenate([np.asarray(labels, np.uint8).reshape(-1, 1), im], axis=1)
    with open(f"{path}/{name}", "wb") as f:
        f.write(rec.tobytes())


def accuracy(logits: np.ndarray, labels: np.ndarray) -> float:
    return float(np.mean(np.argmax(np.asarray(logits), axis=-1) == np.asarray(labels)))


def load(name: str, path: Optional[str] = None, normalized: bool = True) -> Dataset:
    """`mnist` / `cifar10` from `path`, normalized like the training pipeline."""
    if name == "mnist":
        d = mnist(path)
        return normalize_dataset(d, MNIST_MEAN, MNIST_STD) if normalized else d
    if name == "cifar10":
        d = cifar10(path)
        return normalize_dataset(d, CIFAR10_MEAN, CIFAR10_STD) if normalized else d
    raise ValueError(f"unknown dataset {name}")
