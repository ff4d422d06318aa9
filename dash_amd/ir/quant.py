"""Quantization schemes of Dash.

Reference: circuit/scalar_tensor.h:453-475 (quantize), :477-493 (rescale),
dense.h:41-58 / conv2d.h (scheme selection).

* SimpleQuant(q):       w_q = llround(w / q)
* ScaleQuant(l):        w_q = llround(w * 2^l),  b_q = llround(b * 2^(2l)),
                        followed by an auto-inserted Rescale(l)
* ScaleQuantPlus(s):    w_q = llround(w * s),    b_q = llround(b * s^2),
                        followed by Rescale({s})

Arithmetic is float32 like the reference (wandb_t = float) and rounding is
half-away-from-zero (std::llround), not numpy's half-to-even.
"""
from __future__ import annotations

import enum

import numpy as np


class QuantizationMethod(enum.IntEnum):
    SimpleQuant = 0
    ScaleQuant = 1
    ScaleQuantPlus = 2


def llround(v: np.ndarray) -> np.ndarray:
    v = np.asarray(v)
    return (np.sign(v) * np.floor(np.abs(v) + np.asarray(0.5, dtype=v.dtype))).astype(np.int64)


def quantize_simple(values: np.ndarray, q_const: float) -> np.ndarray:
    v = np.asarray(values, dtype=np.float32)
    return llround(v / np.float32(q_const))


def quantize_scale(values: np.ndarray, s: int) -> np.ndarray:
    v = np.asarray(values, dtype=np.float32)
    return llround(v * np.float32(s))


def quantize_params(w: np.ndarray, b: np.ndarray, method: QuantizationMethod, q_parameter: int, q_const: float):
    """Returns (w_q, b_q) as int64 arrays."""
    if method == QuantizationMethod.SimpleQuant:
        return quantize_simple(w, q_const), quantize_simple(b, q_const)
    if method == QuantizationMethod.ScaleQuant:
        return quantize_scale(w, 1 << q_parameter), quantize_scale(b, 1 << (2 * q_parameter))
    if method == QuantizationMethod.ScaleQuantPlus:
        return quantize_scale(w, q_parameter), quantize_scale(b, q_parameter * q_parameter)
    raise ValueError(f"unknown quantization method {method}")


def quantize_input(x: np.ndarray, method: QuantizationMethod, q_parameter: int, q_const: float) -> np.ndarray:
    """Input quantization used by the model benchmarks (scale like the weights)."""
    if method == QuantizationMethod.SimpleQuant:
        return quantize_simple(x, q_const)
    if method == QuantizationMethod.ScaleQuant:
        return quantize_scale(x, 1 << q_parameter)
    return quantize_scale(x, q_parameter)


def ceil_div(x: np.ndarray, s: int) -> np.ndarray:
    x = np.asarray(x, dtype=np.int64)
    return -((-x) // s)
