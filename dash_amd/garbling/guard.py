"""Exact run-time range guard of the garbler's inputs (the mixed-radix rescale's wrap band, CRT overflow).

The garbled circuit computes every value modulo M = prod(CRT base) and its non-linear gadgets read them as
signed values in [-M/2, M/2). Two constructions are exact only on a narrower range:

* the mixed-radix rescale (gadgets.h RescaleMrsPlan) adds U = M/2 rounded up to S - 1 mod S (S = 2^l) before
  its single conversion, so its inputs must stay below ``Rescale.mrs_limit(M)``: the top < 2^l values below
  M/2 wrap and decode to a wrong but *valid* label (docs/SECURITY.md "mixed-radix wrap band");
* every gadget input outside [-M/2, M/2) has already wrapped modulo M (CRT overflow) — the reference's own
  failure mode, which it only guards statically through range calibration (circuit.h:159-265,
  rescale_gadget.h:115-242 is exact on the whole signed range but not beyond it).

The garbler knows its plaintext input and the public weights, so it can decide exactly, per input, whether
the garbled result will equal the plaintext one: it evaluates the quantized model and checks the input of
every non-linear gadget (ReLU, Sign, MaxPool, Rescale) and the outputs. An input that fails is refused with
``RangeGuardError`` before its result is released (never a silently wrong label).

Max pooling is a pairwise tree of max(a, b) = a + relu(b - a): besides its inputs, every difference b - a it
feeds a ReLU gadget must be a signed value. The guard bounds them all by the window's span: max - min <=
min(M/2, M - M/2 - 1) (a sufficient condition, exact for the tree's pairs).

Three implementations with one semantics (tests/test_range_guard.py pins them against each other):

* on a GPU, ``DevRangeGuard`` (csrc/hip/guard.hip): one HIP launch per layer over chunks of the batch,
  int64 activations and 32 x 32 -> 64-bit products, on its own high-priority stream beside the garbled
  evaluation; inputs whose activations exceed the int32 operand range are re-decided by the numpy model;
* the batched torch evaluation (float64 GEMMs, exact below 2^53), used on the CPU and as the bench's batched
  verification oracle (``outputs``);
* the per-input numpy model (``violations_np``), the exact reference of both and the path of layers without a
  batched form (test-only Mult / Max).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from ..ir import layers as L


class RangeGuardError(ValueError):
    """A garbler input whose garbled evaluation would leave a gadget's exact range (wrap band / overflow)."""


def _half(M: int) -> int:
    return M // 2


class RangeGuard:
    """Per-circuit exact range check. ``mrs=True``: DASH Rescale(l) inputs must stay below the mixed-radix
    wrap band; every gadget input and output must be a signed CRT value in [-M/2, M/2)."""

    CHUNK = 16  # inputs per GPU pass (im2col working set ~60 MB on the MiniONN CNN)

    def __init__(self, circuit, crt_modulus: int, mrs: bool = True, device: Optional[int] = None):
        self.circuit, self.M, self.mrs = circuit, int(crt_modulus), bool(mrs)
        self.device = device
        self.batched = all(isinstance(l, (L.Conv2d, L.Dense, L.Rescale, L.Relu, L.Sign, L.Flatten, L.MaxPool2d,
                                          L.SumPool2d, L.Add, L.Projection, L.BaseExtension)) for l in circuit.layers)
        self._w = None
        self._stream = None
        self._dev = None  # DevRangeGuard (GPU), built on first use

    # ------------------------------------------------------------------ limits
    def _limits(self, layer) -> Optional[tuple]:
        """(lo, hi_exclusive) the layer's input must satisfy, or None (linear / free layers)."""
        h = _half(self.M)
        lo, hi = -h, self.M - h
        if isinstance(layer, L.Rescale):
            if self.mrs and layer.use_sign_base_extension and layer.l >= 1:
                hi = min(hi, layer.mrs_limit(self.M))
            return lo, hi
        if isinstance(layer, (L.Relu, L.Sign, L.MaxPool2d, L.Max)):
            return lo, hi
        return None

    def span_max(self) -> int:
        """Largest max - min of a max-pooling window whose pairwise differences are all signed CRT values."""
        h = _half(self.M)
        return min(h, self.M - h - 1)

    # ------------------------------------------------------------------ exact per-input reference (numpy)
    def violations_np(self, x) -> list:
        """[(layer index or 'out', min, max, lo, hi)] of one input, by the numpy plaintext evaluation."""
        c, M = self.circuit, self.M
        x = np.asarray(x, dtype=np.int64).reshape(-1)
        ctx, cur, bad = [x], x, []
        for i, l in enumerate(c.layers):
            src = getattr(l, "in_src", None)
            inp = ctx[src + 1] if src is not None else cur
            lim = self._limits(l)
            if lim is not None and inp.size:
                mn, mx = int(inp.min()), int(inp.max())
                if mn < lim[0] or mx >= lim[1]:
                    bad.append((i, mn, mx, lim[0], lim[1]))
            if isinstance(l, L.MaxPool2d) and inp.size:
                w = np.stack(l._windows(inp))
                span = int((w.max(axis=0) - w.min(axis=0)).max())
                if span > self.span_max():
                    bad.append((i, "span", span, 0, self.span_max()))
            cur = l.plain_q_eval(inp, False, ctx, M)
            ctx.append(cur)
        h = _half(M)
        if cur.size and (int(cur.min()) < -h or int(cur.max()) >= M - h):
            bad.append(("out", int(cur.min()), int(cur.max()), -h, M - h))
        return bad

    # ------------------------------------------------------------------ batched torch path
    def _tdev(self):
        import torch

        if self.device is not None and torch.cuda.is_available():
            return torch.device("cuda", int(self.device))
        return torch.device("cpu")

    def _weights(self, dev):
        import torch

        if self._w is None or self._w[0] != dev:
            ws = []
            for l in self.circuit.layers:
                if isinstance(l, L.Conv2d):
                    ws.append((torch.tensor(np.array(l.q_weights.reshape(l.F, -1)), dtype=torch.float64, device=dev),
                               torch.tensor(np.array(l.q_biases), dtype=torch.float64, device=dev)))
                elif isinstance(l, L.Dense):
                    perm = None
                    if l.channel_tf:
                        K, ch = l.in_size, l.channel_tf
                        i = np.arange(K)
                        perm = torch.as_tensor(i // ch + (i % ch) * (K // ch), device=dev)
                    ws.append((torch.tensor(np.array(l.q_weights), dtype=torch.float64, device=dev),
                               torch.tensor(np.array(l.q_biases), dtype=torch.float64, device=dev), perm))
                else:
                    ws.append(None)
            self._w = (dev, ws)
        return self._w[1]

    def _bad_batch(self, X, want_out: bool = False):
        """X: (B, N) int64 tensor -> (B,) bool tensor, True where a gadget input leaves its exact range (and the
        outputs, with want_out)."""
        import torch
        import torch.nn.functional as F

        M, h = self.M, _half(self.M)
        ws = self._weights(X.device)
        B = X.shape[0]
        bad = torch.zeros(B, dtype=torch.bool, device=X.device)
        ctx, cur = [X], X
        for i, l in enumerate(self.circuit.layers):
            src = getattr(l, "in_src", None)
            inp = ctx[src + 1] if src is not None else cur
            lim = self._limits(l)
            if lim is not None:
                bad |= (inp < lim[0]).any(dim=1) | (inp >= lim[1]).any(dim=1)
            if isinstance(l, L.Conv2d):
                W, b = ws[i]
                cols = F.unfold(inp.to(torch.float64).view(B, l.C, l.H, l.W), (l.kh, l.kw), padding=(l.ph, l.pw),
                                stride=(l.sh, l.sw))
                y = torch.matmul(W, cols) + b[:, None]
                out = y.reshape(B, -1).to(torch.int64)
            elif isinstance(l, L.Dense):
                W, b, perm = ws[i]
                xin = inp if perm is None else inp[:, perm]
                out = (xin.to(torch.float64) @ W.t() + b).to(torch.int64)
            elif isinstance(l, L.Rescale):
                if l.use_sign_base_extension:
                    out = inp
                    for _ in range(l.l):
                        out = torch.div(out + h % 2, 2, rounding_mode="floor")
                else:
                    S = int(np.prod(l.s))
                    out = torch.div(inp + h % S, S, rounding_mode="floor")
            elif isinstance(l, L.Relu):
                out = torch.clamp_min(inp, 0)
            elif isinstance(l, L.Sign):
                out = torch.where(inp >= 0, 1, -1).to(torch.int64)
            elif isinstance(l, L.MaxPool2d):
                v = inp.view(B, l.C, l.H, l.W)
                out = mn = None
                for dy in range(l.kh):
                    for dx in range(l.kw):
                        w = v[:, :, dy:dy + l.sh * (l.OH - 1) + 1:l.sh, dx:dx + l.sw * (l.OW - 1) + 1:l.sw]
                        out = w if out is None else torch.maximum(out, w)
                        mn = w if mn is None else torch.minimum(mn, w)
                bad |= ((out - mn).reshape(B, -1) > self.span_max()).any(dim=1)
                out = out.reshape(B, -1)
            elif isinstance(l, L.SumPool2d):
                v = inp.view(B, l.C, l.H, l.W)
                out = 0
                for dy in range(l.kh):
                    for dx in range(l.kw):
                        out = out + v[:, :, dy:dy + l.sh * (l.OH - 1) + 1:l.sh, dx:dx + l.sw * (l.OW - 1) + 1:l.sw]
                out = out.reshape(B, -1)
            elif isinstance(l, L.Add):
                out = inp + ctx[l.src + 1]
            else:  # Flatten, Projection, BaseExtension: value-preserving
                out = inp.reshape(B, -1)
            ctx.append(out)
            cur = out
        bad |= (cur < -h).any(dim=1) | (cur >= M - h).any(dim=1)
        return (bad, cur) if want_out else bad

    def outputs(self, xs) -> np.ndarray:
        """The exact quantized plaintext outputs (Circuit.plain_q_eval with the CRT modulus) of a batch, by the
        same batched evaluation: the bench's verification oracle for many inputs."""
        xs = np.asarray(np.stack([np.asarray(x, dtype=np.int64).reshape(-1) for x in xs]))
        if not self.batched:
            return np.stack([self.circuit.plain_q_eval(x, False, self.M) for x in xs])
        import torch

        dev = self._tdev()
        with torch.no_grad():
            X = torch.as_tensor(xs).to(dev)
            outs = [self._bad_batch(X[k:k + self.CHUNK], True)[1] for k in range(0, len(xs), self.CHUNK)]
            return torch.cat(outs).cpu().numpy()

    # ------------------------------------------------------------------ native GPU path
    def native_spec(self) -> dict:
        """The DevRangeGuard description of the circuit. Elementwise layers (rescale, ReLU, sign, value-preserving)
        whose input is read by no other layer are fused into the epilogue of the layer before them ("post": each
        checks its input range, then applies its function); every remaining group is one launch. Activation
        buffers are shared by values whose lifetimes do not overlap."""
        c, M, h = self.circuit, self.M, _half(self.M)
        lay = c.layers
        n = len(lay)
        srcs = []
        for i, l in enumerate(lay):
            src = getattr(l, "in_src", None)
            srcs.append(src + 1 if src is not None else i)
        readers: dict = {}
        for i, l in enumerate(lay):
            readers.setdefault(srcs[i], []).append(i)
            if isinstance(l, L.Add):
                readers.setdefault(l.src + 1, []).append(i)
        elem = (L.Rescale, L.Relu, L.Sign, L.Flatten, L.Projection, L.BaseExtension)

        def op_of(i):
            l, d = lay[i], {}
            lim = self._limits(l)
            if lim is not None:
                d.update(check=True, lo=int(lim[0]), hi=int(lim[1]))
            if isinstance(l, L.Rescale):
                if l.use_sign_base_extension:
                    d.update(kind=2, l=int(l.l), c=int(h % 2))
                else:
                    S = int(np.prod(l.s))
                    d.update(kind=3, S=S, c=int(h % S))
            elif isinstance(l, L.Relu):
                d.update(kind=4)
            elif isinstance(l, L.Sign):
                d.update(kind=5)
            else:
                d.update(kind=9)
            return d

        # groups: a head layer and the elementwise layers fused after it
        groups, i = [], 0
        while i < n:
            g, j = [i], i + 1
            while (j < n and isinstance(lay[j], elem) and srcs[j] == j and readers.get(j) == [j]
                   and len(g) - (0 if isinstance(lay[i], elem) else 1) < 6):
                g.append(j)
                j += 1
            groups.append(g)
            i = j
        # buffers: the output of group k (context index g[-1] + 1) lives until the last group that reads it
        group_of_ctx = {g[-1] + 1: k for k, g in enumerate(groups)}
        last_use = {n: len(groups)}
        for k, g in enumerate(groups):
            ins = [srcs[g[0]]] + ([lay[g[0]].src + 1] if isinstance(lay[g[0]], L.Add) else [])
            for ci in ins:
                assert ci == 0 or ci in group_of_ctx, "range guard: a fused value is read by a later layer"
                last_use[ci] = max(last_use.get(ci, -1), k)
        ctx_buf, buf_elems, holder, layers = [0] * (n + 1), [], [], []
        for k, g in enumerate(groups):
            head = lay[g[0]]
            out_ctx = g[-1] + 1
            out_size = int(lay[g[-1]].out_size)
            free = [b for b, cj in enumerate(holder) if last_use.get(cj, -1) < k]
            if free:
                b = free[0]
                buf_elems[b] = max(buf_elems[b], out_size)
                holder[b] = out_ctx
            else:
                b = len(holder)
                holder.append(out_ctx)
                buf_elems.append(out_size)
            for j in g:
                ctx_buf[j + 1] = b
            d = dict(src=srcs[g[0]], buf=b, in_size=int(head.in_size), out_size=out_size)
            post = [op_of(j) for j in g[1:]]
            if isinstance(head, L.Conv2d):
                d.update(kind=0, C=head.C, H=head.H, W=head.W, F=head.F, kh=head.kh, kw=head.kw, sh=head.sh,
                         sw=head.sw, ph=head.ph, pw=head.pw, OH=head.OH, OW=head.OW,
                         w=_i32(head.q_weights.reshape(head.F, -1)), b=np.asarray(head.q_biases, np.int64))
            elif isinstance(head, L.Dense):
                perm = None
                if head.channel_tf:
                    K, ch = head.in_size, head.channel_tf
                    kk = np.arange(K)
                    perm = (kk // ch + (kk % ch) * (K // ch)).astype(np.int32)
                d.update(kind=1, w=_i32(head.q_weights), b=np.asarray(head.q_biases, np.int64).reshape(-1), perm=perm)
            elif isinstance(head, (L.MaxPool2d, L.SumPool2d)):
                d.update(kind=6 if isinstance(head, L.MaxPool2d) else 7, C=head.C, H=head.H, W=head.W, kh=head.kh,
                         kw=head.kw, sh=head.sh, sw=head.sw, OH=head.OH, OW=head.OW, span_max=int(self.span_max()))
                lim = self._limits(head)
                if lim is not None:
                    d.update(check=True, lo=int(lim[0]), hi=int(lim[1]))
            elif isinstance(head, L.Add):
                d.update(kind=8, add_src=int(head.src + 1))
            else:  # an elementwise head: its own op first
                d.update(kind=9)
                post = [op_of(g[0])] + post
            d["post"] = post
            layers.append(d)
        return dict(layers=layers, input_size=int(c.input_size), ctx_buf=ctx_buf, buf_elems=buf_elems,
                    out_lo=-h, out_hi=M - h)

    def _native(self):
        if self._dev is None:
            from ..native import native

            spec = self.native_spec()
            per_input = 8 * sum(spec["buf_elems"])
            chunk = int(max(1, min(64, (256 << 20) // max(1, per_input))))
            self._dev = native().DevRangeGuard(int(self.device), spec["layers"], spec["input_size"], spec["ctx_buf"],
                                               spec["buf_elems"], spec["out_lo"], spec["out_hi"], chunk)
        return self._dev

    def _native_ok(self) -> bool:
        if self.device is None or not self.batched:
            return False
        try:
            import torch

            return torch.cuda.is_available()
        except ImportError:  # pragma: no cover
            return False

    # ------------------------------------------------------------------ public API
    def submit(self, xs) -> "PendingCheck":
        """Start the check of a batch of inputs; on a GPU it runs on its own stream (DevRangeGuard),
        overlapping the garbled evaluation launched before. ``PendingCheck.raise_if_bad()`` before releasing
        the results."""
        xs = np.asarray(np.stack([np.asarray(x, dtype=np.int64).reshape(-1) for x in xs]))
        if not self.batched:
            return PendingCheck(self, xs, None, None)
        if self._native_ok():
            g = self._native()
            return PendingCheck(self, xs, None, None, native=(g, g.submit(xs)))
        import torch

        dev = self._tdev()
        if dev.type == "cuda":
            if self._stream is None:
                self._stream = torch.cuda.Stream(device=dev)
            st = self._stream
            st.wait_stream(torch.cuda.current_stream(dev))  # staging of an earlier submit is free again
            with torch.cuda.stream(st):
                X = torch.as_tensor(xs).pin_memory().to(dev, non_blocking=True)
                flags = torch.cat([self._bad_batch(X[k:k + self.CHUNK]) for k in range(0, len(xs), self.CHUNK)])
                host = flags.to("cpu", non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
            return PendingCheck(self, xs, host, ev)
        with torch.no_grad():
            X = torch.as_tensor(xs)
            flags = torch.cat([self._bad_batch(X[k:k + self.CHUNK]) for k in range(0, len(xs), self.CHUNK)])
        return PendingCheck(self, xs, flags, None)

    def check(self, xs) -> None:
        self.submit(xs).raise_if_bad()


class PendingCheck:
    def __init__(self, guard: RangeGuard, xs: np.ndarray, flags, event, native=None):
        self.guard, self.xs, self.flags, self.event = guard, xs, flags, event
        self.native = native
        self._bad = None

    def bad_indices(self) -> List[int]:
        if self._bad is not None:
            return self._bad
        if self.native is not None:  # DevRangeGuard: bit 0 violation, bit 1 activations beyond int32 operands
            g, ticket = self.native
            f = np.asarray(g.wait(ticket))
            self.native = None
            self._bad = [int(i) for i in np.nonzero(f & 1)[0]]
            self._bad += [int(i) for i in np.nonzero(f == 2)[0] if self.guard.violations_np(self.xs[i])]
            self._bad.sort()
            return self._bad
        if self.flags is None:  # per-input numpy path
            return [i for i, x in enumerate(self.xs) if self.guard.violations_np(x)]
        if self.event is not None:
            self.event.synchronize()
        return [int(i) for i in np.nonzero(self.flags.numpy())[0]]

    def raise_if_bad(self) -> None:
        bad = self.bad_indices()
        if bad:
            i = bad[0]
            v = self.guard.violations_np(self.xs[i])
            raise RangeGuardError(
                f"range guard: {len(bad)} of {len(self.xs)} input(s) would leave an exact gadget range (first: "
                f"input {i}, layer/lo/hi violations {v}); the garbled result would be a valid but wrong label. "
                f"Refused: use rescale='legacy' or a larger CRT base for such inputs")


def _i32(a) -> np.ndarray:
    a = np.asarray(a, dtype=np.int64)
    if a.size and (a.min() < -(1 << 31) or a.max() >= (1 << 31)):
        raise ValueError("range guard: weights beyond int32")
    return a.astype(np.int32)


def guard_for(circuit, crt_modulus: int, mrs: bool, device: Optional[int] = None) -> RangeGuard:
    """The circuit's cached guard (weights staged once per device)."""
    cache = circuit.__dict__.setdefault("_range_guards", {})
    key = (int(crt_modulus), bool(mrs), device)
    g = cache.get(key)
    if g is None:
        g = cache[key] = RangeGuard(circuit, crt_modulus, mrs, device)
    return g
