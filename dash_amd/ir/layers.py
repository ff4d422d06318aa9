"""Plaintext layer IR (float + quantized semantics, range tracking).

Reference: circuit/layer/*.h (C08-C11 in SURVEY §2.1). Tensors are numpy
arrays; images are laid out [C][H][W] (width fastest), which is the memory
order of the reference's dim_t {W, H, C} (dims[0] fastest).

Every layer knows how to describe itself to the native garbler
(`garble_spec`), which keeps the kind numbering of csrc/model.h.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import numpy as np

from .quant import QuantizationMethod, ceil_div, quantize_params

Q_MAX = np.iinfo(np.int64).max
Q_MIN = np.iinfo(np.int64).min


class Kind:
    DENSE = 0
    CONV = 1
    RELU = 2
    SIGN = 3
    RESCALE = 4
    MAXPOOL = 5
    FLATTEN = 6
    PROJ = 7
    MULT = 8
    MMULT = 9
    MAX = 10
    BASEEXT = 11
    ADD = 12
    SUMPOOL = 13


def _size(d: Sequence[int]) -> int:
    s = 1
    for v in d:
        s *= int(v)
    return s


class Layer:
    kind: int = -1
    name: str = "layer"

    # index of the layer whose output this layer reads (-1 = circuit input);
    # None = the previous layer (sequential). Used for projection shortcuts.
    in_src = None

    def __init__(self, in_dims: Sequence[int], out_dims: Sequence[int]):
        self.in_dims = tuple(int(d) for d in in_dims)
        self.out_dims = tuple(int(d) for d in out_dims)
        self.reset_ranges()

    # ---- geometry
    @property
    def in_size(self) -> int:
        return _size(self.in_dims)

    @property
    def out_size(self) -> int:
        return _size(self.out_dims)

    # ---- range tracking (reference layer.h:13-77)
    def reset_ranges(self):
        self.min_q = Q_MAX
        self.max_q = Q_MIN
        self.min_f = np.inf
        self.max_f = -np.inf

    def _track_q(self, *arrs):
        for a in arrs:
            a = np.asarray(a)
            if a.size:
                self.min_q = min(self.min_q, int(a.min()))
                self.max_q = max(self.max_q, int(a.max()))

    def _track_f(self, *arrs):
        for a in arrs:
            a = np.asarray(a)
            if a.size:
                self.min_f = min(self.min_f, float(a.min()))
                self.max_f = max(self.max_f, float(a.max()))

    def get_min_plain_q_val(self) -> int:
        return self.min_q

    def get_max_plain_q_val(self) -> int:
        return self.max_q

    # ---- semantics
    def plain_eval(self, x: np.ndarray, track: bool = True, ctx=None) -> np.ndarray:
        raise NotImplementedError

    def plain_q_eval(self, x: np.ndarray, track: bool = True, ctx=None, crt_modulus: Optional[int] = None) -> np.ndarray:
        raise NotImplementedError

    def quantize(self, q_const: float) -> None:  # SimpleQuant re-quantization
        pass

    def get_q_const(self) -> float:
        return 0.0

    def garble_spec(self) -> tuple[int, dict]:
        return self.kind, {}

    def __repr__(self) -> str:
        return f"{type(self).__name__}(in={self.in_dims}, out={self.out_dims})"


# ---------------------------------------------------------------------------
class Dense(Layer):
    """Fully connected layer, W [out][in]. Reference: circuit/layer/dense.h."""

    kind = Kind.DENSE
    name = "dense"

    def __init__(self, weights: np.ndarray, biases: np.ndarray, q_parameter: int = -1,
                 q_method: QuantizationMethod = QuantizationMethod.SimpleQuant, q_const: float = 10.0,
                 channel_tf: int = 0):
        w = np.asarray(weights, dtype=np.float32)
        b = np.asarray(biases, dtype=np.float32).reshape(-1)
        assert w.ndim == 2 and w.shape[0] == b.shape[0], "weights/biases shape mismatch"
        super().__init__((w.shape[1],), (w.shape[0],))
        self.weights, self.biases = w, b
        self.q_method, self.q_parameter, self.q_const = QuantizationMethod(q_method), q_parameter, q_const
        self.channel_tf = int(channel_tf)
        self.q_weights, self.q_biases = quantize_params(w, b, self.q_method, q_parameter, q_const)
        self._track_q(self.q_weights, self.q_biases)

    @classmethod
    def from_quantized(cls, q_weights: np.ndarray, q_biases: np.ndarray, channel_tf: int = 0) -> "Dense":
        d = cls(np.asarray(q_weights, dtype=np.float32), np.asarray(q_biases, dtype=np.float32), q_const=1.0,
                channel_tf=channel_tf)
        d.q_weights = np.asarray(q_weights, dtype=np.int64)
        d.q_biases = np.asarray(q_biases, dtype=np.int64).reshape(-1)
        d.reset_ranges()
        d._track_q(d.q_weights, d.q_biases)
        return d

    def _src(self, x):
        if self.channel_tf == 0:
            return x
        K, ch = x.shape[0], self.channel_tf
        i = np.arange(K)
        return x[i // ch + (i % ch) * (K // ch)]

    def quantize(self, q_const):
        self.q_const = q_const
        self.q_weights, self.q_biases = quantize_params(self.weights, self.biases, QuantizationMethod.SimpleQuant,
                                                        -1, q_const)
        self.reset_ranges()

    def get_q_const(self):
        return self.q_const

    def plain_eval(self, x, track=True, ctx=None):
        x = self._src(np.asarray(x, dtype=np.float32).reshape(-1))
        y = self.weights @ x + self.biases
        if track:
            self._track_f(x, y, self.weights, self.biases)
        return y

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        x = self._src(np.asarray(x, dtype=np.int64).reshape(-1))
        if track:
            self._track_q(x)
            # partial sums of every row, as the reference tracks them
            cs = np.cumsum(self.q_weights * x[None, :], axis=1)
            self._track_q(cs)
        y = self.q_weights @ x + self.q_biases
        if track:
            self._track_q(y)
        return y

    def get_min_plain_q_val(self):
        return min(self.min_q, int(self.q_weights.min()), int(self.q_biases.min()))

    def get_max_plain_q_val(self):
        return max(self.max_q, int(self.q_weights.max()), int(self.q_biases.max()))

    def garble_spec(self):
        return self.kind, {"in": self.in_size, "out": self.out_size, "w": self.q_weights.reshape(-1),
                           "b": self.q_biases.reshape(-1), "channel_tf": self.channel_tf}


def _im2col(x: np.ndarray, C, H, W, kh, kw, sh, sw, ph, pw):
    xp = np.pad(x.reshape(C, H, W), ((0, 0), (ph, ph), (pw, pw)))
    OH = (H + 2 * ph - kh) // sh + 1
    OW = (W + 2 * pw - kw) // sw + 1
    cols = np.empty((C, kh, kw, OH, OW), dtype=x.dtype)
    for dy in range(kh):
        for dx in range(kw):
            cols[:, dy, dx] = xp[:, dy:dy + sh * (OH - 1) + 1:sh, dx:dx + sw * (OW - 1) + 1:sw]
    return cols.reshape(C * kh * kw, OH * OW), OH, OW


class Conv2d(Layer):
    """2-D convolution, weights [F][C][kh][kw]; optional zero padding (an
    extension over the reference's 'valid'-only conv, needed by VGG/ResNet).
    Reference: circuit/layer/conv2d.h (index bug §2.7 #2 fixed)."""

    kind = Kind.CONV
    name = "conv2d"

    def __init__(self, weights: np.ndarray, biases: np.ndarray, input_width: int, input_height: int, channel: int,
                 filter: int, filter_width: int, filter_height: int, stride_width: int = 1, stride_height: int = 1,
                 q_parameter: int = -1, q_method: QuantizationMethod = QuantizationMethod.SimpleQuant,
                 q_const: float = 10.0, pad_width: int = 0, pad_height: int = 0):
        self.C, self.H, self.W, self.F = int(channel), int(input_height), int(input_width), int(filter)
        self.kh, self.kw, self.sh, self.sw = int(filter_height), int(filter_width), int(stride_height), int(stride_width)
        self.ph, self.pw = int(pad_height), int(pad_width)
        self.OH = (self.H + 2 * self.ph - self.kh) // self.sh + 1
        self.OW = (self.W + 2 * self.pw - self.kw) // self.sw + 1
        super().__init__((self.C, self.H, self.W), (self.F, self.OH, self.OW))
        w = np.asarray(weights, dtype=np.float32).reshape(self.F, self.C, self.kh, self.kw)
        b = np.asarray(biases, dtype=np.float32).reshape(self.F)
        self.weights, self.biases = w, b
        self.q_method, self.q_parameter, self.q_const = QuantizationMethod(q_method), q_parameter, q_const
        self.q_weights, self.q_biases = quantize_params(w, b, self.q_method, q_parameter, q_const)
        self._track_q(self.q_weights, self.q_biases)

    @classmethod
    def from_quantized(cls, q_weights, q_biases, input_width, input_height, channel, filter, filter_width,
                       filter_height, stride_width=1, stride_height=1, pad_width=0, pad_height=0):
        c = cls(np.zeros((filter, channel, filter_height, filter_width), np.float32), np.zeros(filter, np.float32),
                input_width, input_height, channel, filter, filter_width, filter_height, stride_width, stride_height,
                q_const=1.0, pad_width=pad_width, pad_height=pad_height)
        c.q_weights = np.asarray(q_weights, dtype=np.int64).reshape(filter, channel, filter_height, filter_width)
        c.q_biases = np.asarray(q_biases, dtype=np.int64).reshape(filter)
        c.weights = c.q_weights.astype(np.float32)
        c.biases = c.q_biases.astype(np.float32)
        c.reset_ranges()
        c._track_q(c.q_weights, c.q_biases)
        return c

    def quantize(self, q_const):
        self.q_const = q_const
        self.q_weights, self.q_biases = quantize_params(self.weights, self.biases, QuantizationMethod.SimpleQuant,
                                                        -1, q_const)
        self.reset_ranges()

    def get_q_const(self):
        return self.q_const

    def _conv(self, x, w, b):
        cols, OH, OW = _im2col(x, self.C, self.H, self.W, self.kh, self.kw, self.sh, self.sw, self.ph, self.pw)
        y = w.reshape(self.F, -1) @ cols + b[:, None]
        return y.reshape(-1), cols

    def plain_eval(self, x, track=True, ctx=None):
        y, _ = self._conv(np.asarray(x, dtype=np.float32).reshape(-1), self.weights, self.biases)
        if track:
            self._track_f(x, y, self.weights, self.biases)
        return y

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        x = np.asarray(x, dtype=np.int64).reshape(-1)
        y, cols = self._conv(x, self.q_weights, self.q_biases)
        if track:
            wf = self.q_weights.reshape(self.F, -1)
            # products and running partial sums (conv2d.h:85-140)
            for f in range(self.F):
                prod = wf[f][:, None] * cols
                self._track_q(prod, np.cumsum(prod, axis=0))
            self._track_q(y)
        return y

    def get_min_plain_q_val(self):
        return min(self.min_q, int(self.q_weights.min()), int(self.q_biases.min()))

    def get_max_plain_q_val(self):
        return max(self.max_q, int(self.q_weights.max()), int(self.q_biases.max()))

    def garble_spec(self):
        return self.kind, {"C": self.C, "H": self.H, "W": self.W, "F": self.F, "kh": self.kh, "kw": self.kw,
                           "sh": self.sh, "sw": self.sw, "ph": self.ph, "pw": self.pw,
                           "w": self.q_weights.reshape(-1), "b": self.q_biases.reshape(-1)}


class Relu(Layer):
    """ReLU via approximate sign (type approx_relu). Reference: relu.h."""

    kind = Kind.RELU
    name = "approx_relu"

    def __init__(self, dims):
        super().__init__(dims, dims)

    def plain_eval(self, x, track=True, ctx=None):
        y = np.maximum(np.asarray(x), 0)
        if track:
            self._track_f(y)
        return y

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        x = np.asarray(x, dtype=np.int64)
        y = np.maximum(x, 0)
        if track:
            self._track_q(x, y)
        return y

    def quantize(self, q_const):
        self.reset_ranges()


class Sign(Layer):
    """Sign activation x >= 0 ? 1 : -1 (Tanh replacement). Reference: sign.h."""

    kind = Kind.SIGN
    name = "sign"

    def __init__(self, dims):
        super().__init__(dims, dims)

    def plain_eval(self, x, track=True, ctx=None):
        y = np.where(np.asarray(x) >= 0, 1.0, -1.0).astype(np.float32)
        if track:
            self._track_f(y)
        return y

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        y = np.where(np.asarray(x) >= 0, 1, -1).astype(np.int64)
        if track:
            self._track_q(y)
        return y

    def quantize(self, q_const):
        self.reset_ranges()


class Rescale(Layer):
    """CRT scaling. Legacy DASH: `l` halvings (sign base extension); ReDash:
    division by CRT moduli `s` (base extension). Reference: rescale.h,
    rescale_gadget.h. With `crt_modulus` given, plain_q_eval reproduces the
    garbled semantics exactly: floor((x + (M/2 mod S)) / S) per step, which
    equals the reference's ceil(x/2) for the legacy mode."""

    kind = Kind.RESCALE
    name = "rescale"

    def __init__(self, l_or_s, dims):
        super().__init__(dims, dims)
        if isinstance(l_or_s, (list, tuple, np.ndarray)):
            self.l, self.s, self.use_sign_base_extension = -1, [int(v) for v in l_or_s], False
        else:
            self.l, self.s, self.use_sign_base_extension = int(l_or_s), [-1], True

    def _apply(self, x, crt_modulus):
        if self.use_sign_base_extension:
            if crt_modulus is None:
                return ceil_div(x, 1 << self.l)
            y = x
            for _ in range(self.l):
                y = (y + (crt_modulus // 2) % 2) // 2
            return y
        S = 1
        for f in self.s:
            S *= f
        if crt_modulus is None:
            y = x
            for f in self.s:
                y = ceil_div(y, f)
            return y
        return (x + (crt_modulus // 2) % S) // S

    def plain_eval(self, x, track=True, ctx=None):
        return np.asarray(x)

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        x = np.asarray(x, dtype=np.int64)
        y = self._apply(x, crt_modulus)
        if track:
            self._track_q(x, y)
            if x.size:
                self.in_min_q = min(self.in_min_q, int(x.min()))
                self.in_max_q = max(self.in_max_q, int(x.max()))
        return y

    def reset_ranges(self):
        super().reset_ranges()
        self.in_min_q = Q_MAX  # tracked range of the rescale's input (mixed-radix headroom check)
        self.in_max_q = Q_MIN

    @property
    def input_tracked(self) -> bool:
        return self.in_max_q >= self.in_min_q

    def mrs_limit(self, crt_modulus: int) -> int:
        """Exclusive upper bound of the inputs on which the single-shot mixed-radix rescale
        (gadgets.h RescaleMrsPlan) equals the reference's l-fold halving: x + U < M with
        U = M/2 rounded up to S - 1 mod S, S = 2^l (the top U - M/2 < S values wrap)."""
        M, S = int(crt_modulus), 1 << self.l
        h = M // 2
        U = h + (S - 1 - h % S) % S
        return M - U

    def garble_spec(self):
        if self.use_sign_base_extension:
            return self.kind, {"mode": 0, "l": self.l}
        return self.kind, {"mode": 1, "s": list(self.s)}


class Flatten(Layer):
    kind = Kind.FLATTEN
    name = "flatten"

    def __init__(self, dims):
        super().__init__(dims, (_size(dims),))

    def plain_eval(self, x, track=True, ctx=None):
        return np.asarray(x).reshape(-1)

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        if track:
            self.min_q, self.max_q = 0, 0
        return np.asarray(x).reshape(-1)


class MaxPool2d(Layer):
    """Max pooling as a pairwise tree of max(a,b) = a + relu(b - a).
    Reference: max_pool2d.h, garbled_maxpool2d.h (output dims use the stride,
    fixing §2.7 #8)."""

    kind = Kind.MAXPOOL
    name = "max_pool"

    def __init__(self, input_width, input_height, channel, kernel_width, kernel_height, stride_width=None,
                 stride_height=None):
        self.C, self.H, self.W = int(channel), int(input_height), int(input_width)
        self.kh, self.kw = int(kernel_height), int(kernel_width)
        self.sh = int(stride_height if stride_height is not None else kernel_height)
        self.sw = int(stride_width if stride_width is not None else kernel_width)
        self.OH = (self.H - self.kh) // self.sh + 1
        self.OW = (self.W - self.kw) // self.sw + 1
        super().__init__((self.C, self.H, self.W), (self.C, self.OH, self.OW))

    def _windows(self, x):
        x = np.asarray(x).reshape(self.C, self.H, self.W)
        out = []
        for dy in range(self.kh):
            for dx in range(self.kw):
                out.append(x[:, dy:dy + self.sh * (self.OH - 1) + 1:self.sh, dx:dx + self.sw * (self.OW - 1) + 1:self.sw])
        return out

    def plain_eval(self, x, track=True, ctx=None):
        y = np.max(np.stack(self._windows(x)), axis=0).reshape(-1)
        if track:
            self._track_f(y)
        return y

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        w = self._windows(np.asarray(x, dtype=np.int64))
        y = np.max(np.stack(w), axis=0).reshape(-1)
        if track:
            # differences b - a feed the ReLU gadgets
            self._track_q(y, *[a - b for a in w for b in w])
        return y

    def garble_spec(self):
        return self.kind, {"C": self.C, "H": self.H, "W": self.W, "kh": self.kh, "kw": self.kw, "sh": self.sh,
                           "sw": self.sw}


class SumPool2d(Layer):
    """Window sum (free in the label domain). Average pooling = SumPool2d + a
    rescale or a weight fold into the next linear layer."""

    kind = Kind.SUMPOOL
    name = "sum_pool"

    def __init__(self, input_width, input_height, channel, kernel_width, kernel_height, stride_width=None,
                 stride_height=None):
        self.C, self.H, self.W = int(channel), int(input_height), int(input_width)
        self.kh, self.kw = int(kernel_height), int(kernel_width)
        self.sh = int(stride_height if stride_height is not None else kernel_height)
        self.sw = int(stride_width if stride_width is not None else kernel_width)
        self.OH = (self.H - self.kh) // self.sh + 1
        self.OW = (self.W - self.kw) // self.sw + 1
        super().__init__((self.C, self.H, self.W), (self.C, self.OH, self.OW))

    def _sum(self, x):
        x = np.asarray(x).reshape(self.C, self.H, self.W)
        acc = 0
        for dy in range(self.kh):
            for dx in range(self.kw):
                acc = acc + x[:, dy:dy + self.sh * (self.OH - 1) + 1:self.sh, dx:dx + self.sw * (self.OW - 1) + 1:self.sw]
        return acc.reshape(-1)

    def plain_eval(self, x, track=True, ctx=None):
        return self._sum(np.asarray(x, dtype=np.float32))

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        y = self._sum(np.asarray(x, dtype=np.int64))
        if track:
            self._track_q(y)
        return y

    def garble_spec(self):
        return self.kind, {"C": self.C, "H": self.H, "W": self.W, "kh": self.kh, "kw": self.kw, "sh": self.sh,
                           "sw": self.sw}


class Add(Layer):
    """Residual addition of the current tensor and the output of layer `src`
    (-1 = circuit input). Free in the label domain."""

    kind = Kind.ADD
    name = "add"

    def __init__(self, dims, src: int):
        super().__init__(dims, dims)
        self.src = int(src)

    def plain_eval(self, x, track=True, ctx=None):
        return np.asarray(x) + ctx[self.src + 1]

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        y = np.asarray(x, dtype=np.int64) + np.asarray(ctx[self.src + 1], dtype=np.int64)
        if track:
            self._track_q(y)
        return y

    def garble_spec(self):
        return self.kind, {"src": self.src}


# ---- test-only layers (reference: projection.h, mult_layer.h, mixed_mod_mult_layer.h, max.h, base_extension.h)
class Projection(Layer):
    kind = Kind.PROJ
    name = "projection"

    def __init__(self, dims, in_moduli: Sequence[int], out_moduli: Sequence[int], functionality: Callable[[int], int]):
        super().__init__(dims, dims)
        self.in_moduli, self.out_moduli, self.functionality = list(in_moduli), list(out_moduli), functionality

    def plain_eval(self, x, track=True, ctx=None):
        return np.asarray(x)

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        return np.asarray(x)

    def garble_spec(self):
        p = {"in_mod": self.in_moduli, "out_mod": self.out_moduli}
        for j, m in enumerate(self.in_moduli):
            p[f"fn.{j}"] = [int(self.functionality(v)) for v in range(m)]
        return self.kind, p


class MultLayer(Layer):
    kind = Kind.MULT
    name = "mult_layer"

    def __init__(self, in_dims, out_dims=None):
        n = _size(in_dims)
        super().__init__(in_dims, out_dims or (n // 2,))

    def plain_eval(self, x, track=True, ctx=None):
        x = np.asarray(x).reshape(-1)
        return x[0::2] * x[1::2]

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        x = np.asarray(x, dtype=np.int64).reshape(-1)
        y = x[0::2] * x[1::2]
        if track:
            self._track_q(x, y)
        return y


class MixedModMultLayer(MultLayer):
    kind = Kind.MMULT
    name = "mixed_mod_mult_layer"

    def __init__(self, in_dims, out_dims=None, smaller_modulus: int = 2):
        super().__init__(in_dims, out_dims)
        self.smaller_modulus = int(smaller_modulus)

    def garble_spec(self):
        return self.kind, {"q": self.smaller_modulus}


class Max(Layer):
    kind = Kind.MAX
    name = "max"

    def __init__(self, in_dims=(2,)):
        super().__init__(in_dims, (1,))

    def plain_eval(self, x, track=True, ctx=None):
        return np.asarray([np.max(x)])

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        return np.asarray([np.max(np.asarray(x, dtype=np.int64))])


class BaseExtension(Layer):
    """Re-derives the residues of `extra_moduli` from the others (ReDash)."""

    kind = Kind.BASEEXT
    name = "base_extension"

    def __init__(self, dims, extra_moduli: Sequence[int]):
        super().__init__(dims, dims)
        self.extra_moduli = [int(v) for v in extra_moduli]

    def plain_eval(self, x, track=True, ctx=None):
        return np.asarray(x)

    def plain_q_eval(self, x, track=True, ctx=None, crt_modulus=None):
        return np.asarray(x)

    def garble_spec(self):
        return self.kind, {"extra": self.extra_moduli}
