"""Circuit container: plaintext / quantized evaluation, accuracy, CRT sizing and
quantization search. Reference: circuit/circuit.h (C12)."""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from .bases import crt_modulus, first_primes
from .layers import Layer
from .quant import quantize_simple


class Circuit:
    def __init__(self, layers: Sequence[Layer], q_parameter: int = -1):
        self.layers = list(layers)
        assert self.layers, "circuit needs at least one layer"
        self.q_parameter = q_parameter
        self.input_dims = self.layers[0].in_dims
        self.output_dims = self.layers[-1].out_dims

    @property
    def input_size(self) -> int:
        return self.layers[0].in_size

    @property
    def output_size(self) -> int:
        return self.layers[-1].out_size

    def __len__(self):
        return len(self.layers)

    def __iter__(self):
        return iter(self.layers)

    # ---------------------------------------------------------------- eval
    def plain_eval(self, x: np.ndarray, track: bool = True) -> np.ndarray:
        x = np.asarray(x, dtype=np.float32).reshape(-1)
        assert x.size == self.input_size, "input size does not match circuit input size"
        ctx = [x]
        for layer in self.layers:
            src = getattr(layer, "in_src", None)
            x = layer.plain_eval(ctx[src + 1] if src is not None else x, track, ctx)
            ctx.append(x)
        return x

    def plain_q_eval(self, x: np.ndarray, track: bool = True, crt_modulus: Optional[int] = None) -> np.ndarray:
        """Quantized evaluation. With `crt_modulus` the CRT-rescale semantics of
        the garbled circuit are reproduced exactly (see layers.Rescale)."""
        x = np.asarray(x, dtype=np.int64).reshape(-1)
        assert x.size == self.input_size, "input size does not match circuit input size"
        ctx = [x]
        for layer in self.layers:
            src = getattr(layer, "in_src", None)
            x = layer.plain_q_eval(ctx[src + 1] if src is not None else x, track, ctx, crt_modulus)
            ctx.append(x)
        return x

    def plain_test(self, inputs, labels) -> float:
        return float(np.mean([int(np.argmax(self.plain_eval(x, False)) == int(l)) for x, l in zip(inputs, labels)]))

    def plain_q_test(self, inputs, labels, crt_modulus: Optional[int] = None) -> float:
        return float(np.mean([int(np.argmax(self.plain_q_eval(x, False, crt_modulus)) == int(l))
                              for x, l in zip(inputs, labels)]))

    def compute_q_acc(self, x, q_x, q_constant: float, error_bound: float = 1.0) -> float:
        out = self.plain_eval(x)
        rec = self.plain_q_eval(q_x).astype(np.float32) * q_constant
        with np.errstate(divide="ignore", invalid="ignore"):
            rel = np.abs(out - rec) / np.abs(out)
        return float(np.mean(np.where(np.isfinite(rel), rel, np.where(out == rec, 0.0, np.inf)) < error_bound))

    # ---------------------------------------------------------- ranges / CRT
    def reset_ranges(self):
        for layer in self.layers:
            layer.reset_ranges()

    def calibrate(self, inputs, crt_modulus: Optional[int] = None, reset: bool = True) -> "Circuit":
        """Track every layer's quantized value range over `inputs` (the reference's
        range tracking, layer.h:13-77): feeds CRT sizing and the mixed-radix
        rescale guard (mrs_rescale_violations, garbling.resolve_constructions)."""
        if isinstance(inputs, np.ndarray) and inputs.ndim == 1:
            inputs = [inputs]
        if reset:
            self.reset_ranges()
        for x in inputs:
            self.plain_q_eval(x, True, crt_modulus)
        return self

    def get_min_plain_q_val(self) -> int:
        return min(l.get_min_plain_q_val() for l in self.layers)

    def get_max_plain_q_val(self) -> int:
        return max(l.get_max_plain_q_val() for l in self.layers)

    def required_crt_modulus(self, rescale_margin: bool = True) -> int:
        """2 * max |tracked value| (circuit.h:159-231). With `rescale_margin`, the
        input of every DASH rescale (divide by 2^l) also keeps 2^l below M/2, the
        band in which the single-shot mixed-radix rescale construction wraps
        (Rescale.mrs_limit): a base sized here is valid for every construction."""
        need = 2 * max(abs(self.get_min_plain_q_val()), abs(self.get_max_plain_q_val()))
        if rescale_margin:
            for l in self._dash_rescales():
                if l.input_tracked:
                    need = max(need, 2 * (max(abs(l.in_min_q), abs(l.in_max_q)) + (1 << l.l)))
        return need

    def _dash_rescales(self):
        return [l for l in self.layers if getattr(l, "use_sign_base_extension", False) and getattr(l, "l", -1) >= 1]

    def mrs_rescale_violations(self, crt_modulus: int, headroom: bool = False) -> list:
        """DASH rescale layers whose tracked input range reaches the mixed-radix wrap
        band [Rescale.mrs_limit(M), M/2): (layer index, tracked max, limit). Empty
        when no layer has been evaluated with range tracking (nothing to check)."""
        bad = []
        for i, l in enumerate(self.layers):
            if l in self._dash_rescales() and l.input_tracked:
                lim = l.mrs_limit(crt_modulus)
                # headroom: one further 2^l band above the tracked maximum must stay below the limit (the
                # tracked range comes from calibration samples; "auto" keeps a margin for unseen inputs)
                if l.in_max_q + ((1 << l.l) if headroom else 0) >= lim:
                    bad.append((i, int(l.in_max_q), int(lim)))
        return bad

    def infer_crt_base_size(self, inputs, max_k: int = 11, assert_bound: bool = True,
                            rescale_margin: bool = True) -> int:
        """Smallest k such that the product of the first k primes covers every
        tracked intermediate value (circuit.h:159-265), plus the mixed-radix
        rescale headroom (required_crt_modulus)."""
        if isinstance(inputs, np.ndarray) and inputs.ndim == 1:
            inputs = [inputs]
        for x in inputs:
            self.plain_q_eval(x, True)
        need = self.required_crt_modulus(rescale_margin)
        k = 0
        M = 0
        while M < need:
            k += 1
            if k > (max_k if assert_bound else 100):
                if assert_bound:
                    raise ValueError("inferred CRT base size too large; optimize the quantization constant")
                return -1
            M = crt_modulus(first_primes(k))
        return max(k, 1)

    def quantize(self, q_const: float):
        self._native_specs = None
        for layer in self.layers:
            layer.quantize(q_const)

    def get_q_const(self) -> float:
        for layer in self.layers:
            if layer.get_q_const() != 0:
                return layer.get_q_const()
        return 0.0

    def optimize_quantization(self, target_k: int, inputs, init_q: float = 0.2, init_step: float = 0.01,
                              final_step: float = 1e-5, nr_samples: int = -1) -> float:
        """Step search on the SimpleQuant constant until the inferred CRT size
        equals `target_k` with step <= final_step (circuit.h:273-311)."""
        step, k, q, last_q = init_step, -1, init_q, init_q
        self.quantize(q)
        eps = np.finfo(np.float64).eps
        samples = inputs if nr_samples < 0 else inputs[:nr_samples]
        for _ in range(100000):
            if k == target_k and step <= final_step:
                break
            assert q != 0, "q_val cannot be 0"
            self.reset_ranges()
            qin = [quantize_simple(x, q) for x in samples]
            k = self.infer_crt_base_size(qin, assert_bound=False)
            if k == -1:
                self.quantize(last_q)
                return last_q
            if k > target_k:
                if abs(last_q - (q + step)) < eps:
                    step /= 2
                last_q, q = q, q + step
            else:
                if abs(last_q - (q - step)) < eps or abs(q - step) < eps:
                    step /= 2
                last_q, q = q, q - step
            self.quantize(q)
        return q

    def __getstate__(self):
        # the cached native specs are process-local (circuits are pickled to other ranks / processes)
        st = dict(self.__dict__)
        st.pop("_native_specs", None)
        st.pop("_range_guards", None)  # device tensors / streams of the garbler's range guard
        return st

    def garble_specs_native(self):
        """The layer specs as a native GarbleSpecs, built once and reused while the layers' garbling parameters
        are unchanged: the garbler then reduces and hashes the public weights once, not per GC.

        The cache key is every scalar / list parameter of every layer spec plus the identity of its weight and
        bias arrays. Those arrays are made read-only when the specs are built, so an in-place edit
        (``l.q_weights[...] = v``) raises instead of silently garbling stale weights; assigning a new array (what
        quantize() does) changes the key. A writable array at call time (re-enabled by the caller) rebuilds."""
        from ..native import native

        specs = self.garble_specs()

        def norm(v):
            if isinstance(v, np.ndarray):
                return ("arr", id(v.base if v.base is not None else v), v.shape, str(v.dtype))
            if isinstance(v, (list, tuple)):
                return tuple(norm(x) for x in v)
            return v

        arrays = [a for l in self.layers for a in (getattr(l, "q_weights", None), getattr(l, "q_biases", None))
                  if isinstance(a, np.ndarray)]
        fp = tuple((int(k), tuple(sorted((n, norm(v)) for n, v in p.items()))) for k, p in specs)
        fp = (fp, tuple(id(a) for a in arrays))
        cache = getattr(self, "_native_specs", None)
        if cache is None or cache[0] != fp or any(a.flags.writeable for a in arrays):
            cache = (fp, native().GarbleSpecs(specs))
            self._native_specs = cache
            for a in arrays:
                try:
                    a.setflags(write=False)
                except ValueError:  # a view of memory we do not own: the identity key still covers reassignment
                    pass
        return cache[1]

    def garble_specs(self) -> list:
        specs = []
        for l in self.layers:
            kind, params = l.garble_spec()
            if getattr(l, "in_src", None) is not None:
                params = dict(params, in_src=int(l.in_src))
            specs.append((kind, params))
        return specs

    def __repr__(self) -> str:
        return "Circuit(\n  " + "\n  ".join(repr(l) for l in self.layers) + "\n)"
