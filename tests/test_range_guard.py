"""The garbler's exact run-time range guard (dash_amd/garbling/guard.py).

The mixed-radix rescale (gadgets.h RescaleMrsPlan) is exact below Rescale.mrs_limit(M); an input in the band
[mrs_limit, M/2) decodes to a valid but wrong label. The guard must refuse such an input loudly (before its
result is released) while passing every in-range input; its batched torch evaluation must agree exactly with
the numpy plaintext model (Circuit.plain_q_eval). Reference semantics: rescale_gadget.h:115-242 (exact on the
whole signed range).
"""
from __future__ import annotations

import numpy as np
import pytest

import dash_amd as d
from dash_amd.garbling import GarbledCircuit, RangeGuard, RangeGuardError
from dash_amd.ir.bases import crt_modulus, first_primes

K = 6
M = crt_modulus(first_primes(K))
SEED = bytes(range(16))


def _identity_rescale(n=4, l=5):
    """x -> Dense(I, 0) -> Rescale(l) -> ReLU: the rescale sees the plaintext input itself."""
    c = d.Circuit([d.Dense.from_quantized(np.eye(n, dtype=np.int64), np.zeros(n, np.int64)), d.Rescale(l, (n,)),
                   d.Relu((n,))])
    rng = np.random.default_rng(0)
    c.calibrate([rng.integers(-50, 51, size=n) for _ in range(8)], M)
    return c


def test_band_is_real_and_guard_refuses_it():
    c = _identity_rescale()
    lim = c.layers[1].mrs_limit(M)
    assert lim < M // 2  # the band is not empty for this M and l
    x_band = np.array([3, lim, -7, 1], dtype=np.int64)  # one element at the band's first value
    x_ok = np.array([3, lim - 1, -7, 1], dtype=np.int64)

    # without the guard the mixed-radix GC decodes the band input to a wrong (but valid) label
    off = GarbledCircuit(c, K, 100.0, seed=SEED, rescale="mrs", range_guard="off")
    assert off.rescale == "mrs"
    y = off.decode_outputs(off.cpu_evaluate(off.garble_inputs(x_band)))
    assert not np.array_equal(y, off.plain_q_eval(x_band))

    # with it (the default for mixed-radix GCs) the garbler refuses to encode it
    gc = GarbledCircuit(c, K, 100.0, seed=SEED, rescale="mrs")
    assert gc.guard_enabled
    with pytest.raises(RangeGuardError):
        gc.garble_inputs(x_band)
    with pytest.raises(RangeGuardError):
        gc.garble_inputs_compressed(x_band)
    # the last in-range value is exact and passes
    y = gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x_ok)))
    assert np.array_equal(y, gc.plain_q_eval(x_ok))


def test_legacy_gc_is_exact_in_the_band_and_not_guarded_by_default():
    c = _identity_rescale()
    lim = c.layers[1].mrs_limit(M)
    x = np.array([0, lim, lim + 2, -5], dtype=np.int64)
    gc = GarbledCircuit(c, K, 100.0, seed=SEED, rescale="legacy", hardened=False)
    assert not gc.guard_enabled
    assert np.array_equal(gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x))), gc.plain_q_eval(x))
    # "on": the guard also checks CRT overflow for the reference constructions (this input is in range)
    gc_on = GarbledCircuit(c, K, 100.0, seed=SEED, rescale="legacy", hardened=False, range_guard="on")
    gc_on.garble_inputs(x)
    with pytest.raises(RangeGuardError):  # beyond M/2: wrapped modulo M before the rescale
        gc_on.garble_inputs(np.array([0, M // 2 + 1, 0, 0], dtype=np.int64))


def test_batched_guard_matches_numpy_model():
    """The batched torch evaluation flags exactly the inputs the numpy plaintext model flags (MiniONN CNN,
    calibrated inputs plus scaled-up ones that push the rescale inputs over the limit)."""
    from dash_amd.ir.quant import QuantizationMethod
    from dash_amd.models import BENCH_CONFIGS, build_circuit, quantized_inputs

    cfg = BENCH_CONFIGS["MODEL_F_MINIONN_POOL_REPL/DASH"]
    qm = QuantizationMethod(cfg["q_method"])
    c = build_circuit("MODEL_F_MINIONN_POOL_REPL", qm, cfg["q_parameter"], seed=0)
    MM = crt_modulus(first_primes(cfg["crt"]))
    xs = list(quantized_inputs("MODEL_F_MINIONN_POOL_REPL", 3, qm, cfg["q_parameter"], seed=1))
    xs += [x * 40 for x in xs[:2]] + [x * 2000 for x in xs[:1]]
    g = RangeGuard(c, MM, mrs=True)
    flags = sorted(g.submit(xs).bad_indices())
    ref = [i for i, x in enumerate(xs) if g.violations_np(x)]
    assert flags == ref
    assert 0 not in flags and 5 in flags  # calibrated-range inputs pass, a far-out one is refused


@pytest.mark.gpu
def test_guard_on_gpu_matches_numpy_and_refuses_band_on_device_encode_path():
    """Bench / serving shape: device-encoded batch, guard submitted on a side stream after the launch and
    checked before the results are released."""
    import torch

    from dash_amd.runtime import HipEvaluator

    c = _identity_rescale()
    lim = c.layers[1].mrs_limit(M)
    gcs = [GarbledCircuit(c, K, 100.0, seed=bytes([i]) * 16, rescale="mrs", device=0) for i in range(2)]
    ev = HipEvaluator(template=gcs[0].model, batch=2, device=0)
    enc = gcs[0].device_input_encoder(0, 2, slot=0)
    for b, gc in enumerate(gcs):
        ev.load(b, gc.model)
        if b:
            enc.load(gc.garbler, b)
    xs = np.array([[3, lim - 1, -7, 1], [1, 2, lim, 4]], dtype=np.int64)
    ev.encode_device_into(0, enc, xs)
    ev.run()
    pend = gcs[0].guard.submit(xs)
    ev.fetch_outputs()
    assert pend.bad_indices() == [1]
    with pytest.raises(RangeGuardError):
        pend.raise_if_bad()
    y0 = ev.decode(0, gcs[0])
    assert np.array_equal(y0, gcs[0].plain_q_eval(xs[0]))
    # the GPU batched path agrees with numpy on the MiniONN CNN too
    from dash_amd.ir.quant import QuantizationMethod
    from dash_amd.models import BENCH_CONFIGS, build_circuit, quantized_inputs

    cfg = BENCH_CONFIGS["MODEL_F_MINIONN_POOL_REPL/DASH"]
    qm = QuantizationMethod(cfg["q_method"])
    cm = build_circuit("MODEL_F_MINIONN_POOL_REPL", qm, cfg["q_parameter"], seed=0)
    MM = crt_modulus(first_primes(cfg["crt"]))
    xm = list(quantized_inputs("MODEL_F_MINIONN_POOL_REPL", 20, qm, cfg["q_parameter"], seed=2))
    xm[7] = xm[7] * 2000
    g = RangeGuard(cm, MM, mrs=True, device=0)
    assert g.submit(xm).bad_indices() == [7]
    torch.cuda.synchronize()


def test_batched_outputs_equal_plain_q_eval():
    from dash_amd.ir.quant import QuantizationMethod
    from dash_amd.models import BENCH_CONFIGS, build_circuit, quantized_inputs

    for name in ("MODEL_F_MINIONN_POOL_REPL", "MODEL_F_GNNP_POOL_REPL"):
        cfg = BENCH_CONFIGS[f"{name}/DASH"]
        qm = QuantizationMethod(cfg["q_method"])
        c = build_circuit(name, qm, cfg["q_parameter"], seed=0)
        MM = crt_modulus(first_primes(cfg["crt"]))
        xs = quantized_inputs(name, 3, qm, cfg["q_parameter"], seed=4)
        got = RangeGuard(c, MM).outputs(xs)
        assert np.array_equal(got, np.stack([c.plain_q_eval(x, False, MM) for x in xs]))


# ---------------------------------------------------------------- the native (DevRangeGuard) description
def _simulate_spec(spec, xs):
    """Numpy interpreter of RangeGuard.native_spec with the kernels' semantics (csrc/hip/guard.hip), buffers
    shared exactly as the spec assigns them: a CPU check of the description the GPU guard runs."""
    X = np.asarray(xs, dtype=np.int64)
    B = X.shape[0]
    bufs = [np.full((B, e), 7777777, dtype=np.int64) for e in spec["buf_elems"]]
    flags = np.zeros(B, dtype=bool)

    def ctx(i):
        return X if i == 0 else bufs[spec["ctx_buf"][i]]

    def post(ops, y):
        nonlocal flags
        for o in ops:
            if o.get("check"):
                flags |= ((y < o["lo"]) | (y >= o["hi"])).any(axis=1)
            k = o["kind"]
            if k == 2:
                for _ in range(o["l"]):
                    y = (y + o["c"]) >> 1
            elif k == 3:
                y = (y + o["c"]) // o["S"]
            elif k == 4:
                y = np.maximum(y, 0)
            elif k == 5:
                y = np.where(y >= 0, 1, -1)
        return y

    for d in spec["layers"]:
        x = ctx(d["src"])[:, :d["in_size"]].copy()
        k = d["kind"]
        if k == 0:
            C, H, W = d["C"], d["H"], d["W"]
            xp = np.pad(x.reshape(B, C, H, W), ((0, 0), (0, 0), (d["ph"], d["ph"]), (d["pw"], d["pw"])))
            w = d["w"].astype(np.int64).reshape(d["F"], C, d["kh"], d["kw"])
            y = np.zeros((B, d["F"], d["OH"], d["OW"]), np.int64)
            for dy in range(d["kh"]):
                for dx in range(d["kw"]):
                    win = xp[:, :, dy:dy + d["sh"] * (d["OH"] - 1) + 1:d["sh"], dx:dx + d["sw"] * (d["OW"] - 1) + 1:d["sw"]]
                    y += np.einsum("bchw,fc->bfhw", win, w[:, :, dy, dx])
            y = (y + d["b"][None, :, None, None]).reshape(B, -1)
        elif k == 1:
            xin = x if d.get("perm") is None else x[:, d["perm"]]
            y = xin @ d["w"].astype(np.int64).T + d["b"]
        elif k in (6, 7):
            v = x.reshape(B, d["C"], d["H"], d["W"])
            ws = [v[:, :, dy:dy + d["sh"] * (d["OH"] - 1) + 1:d["sh"], dx:dx + d["sw"] * (d["OW"] - 1) + 1:d["sw"]]
                  for dy in range(d["kh"]) for dx in range(d["kw"])]
            st = np.stack(ws)
            if d.get("check"):
                flags |= ((x < d["lo"]) | (x >= d["hi"])).any(axis=1)
            if k == 6:
                y = st.max(axis=0)
                if d.get("check"):
                    flags |= ((st.max(axis=0) - st.min(axis=0)).reshape(B, -1) > d["span_max"]).any(axis=1)
            else:
                y = st.sum(axis=0)
            y = y.reshape(B, -1)
        elif k == 8:
            y = x + ctx(d["add_src"])[:, :d["in_size"]]
        else:
            y = x
        bufs[d["buf"]][:, :d["out_size"]] = post(d.get("post", []), y)
    out = bufs[spec["layers"][-1]["buf"]][:, :spec["layers"][-1]["out_size"]]
    flags |= ((out < spec["out_lo"]) | (out >= spec["out_hi"])).any(axis=1)
    return [int(i) for i in np.nonzero(flags)[0]], out


def _residual_circuit():
    """conv -> rescale -> relu -> conv -> add(residual of the relu) -> maxpool -> flatten -> dense: a live
    value held across layers (buffer sharing) and a max-pooling span check."""
    rng = np.random.default_rng(3)
    c1 = d.Conv2d.from_quantized(rng.integers(-4, 5, (4, 2, 3, 3)), rng.integers(-4, 5, 4), 6, 6, 2, 4, 3, 3,
                                 pad_width=1, pad_height=1)
    c2 = d.Conv2d.from_quantized(rng.integers(-4, 5, (4, 4, 3, 3)), rng.integers(-4, 5, 4), 6, 6, 4, 4, 3, 3,
                                 pad_width=1, pad_height=1)
    mp = d.MaxPool2d(6, 6, 4, 2, 2)
    dn = d.Dense.from_quantized(rng.integers(-3, 4, (5, 36)), rng.integers(-3, 4, 5), channel_tf=4)
    return d.Circuit([c1, d.Rescale(2, (144,)), d.Relu((144,)), c2, d.Add((144,), 2), mp, d.Flatten((4, 3, 3)), dn])


def test_native_spec_matches_numpy_model():
    """The GPU guard's description (buffer sharing, kinds, limits, permutation) flags exactly the inputs the numpy
    model flags and computes the plaintext outputs (MiniONN CNN and a residual circuit)."""
    from dash_amd.ir.quant import QuantizationMethod
    from dash_amd.models import BENCH_CONFIGS, build_circuit, quantized_inputs

    cfg = BENCH_CONFIGS["MODEL_F_MINIONN_POOL_REPL/DASH"]
    qm = QuantizationMethod(cfg["q_method"])
    cm = build_circuit("MODEL_F_MINIONN_POOL_REPL", qm, cfg["q_parameter"], seed=0)
    MM = crt_modulus(first_primes(cfg["crt"]))
    xs = list(quantized_inputs("MODEL_F_MINIONN_POOL_REPL", 3, qm, cfg["q_parameter"], seed=1))
    xs += [xs[0] * 40, xs[1] * 2000]
    for circ, M_, X in ((cm, MM, xs), (_residual_circuit(), crt_modulus(first_primes(4)), None)):
        g = RangeGuard(circ, M_, mrs=True)
        if X is None:
            rng = np.random.default_rng(0)
            X = [rng.integers(-20, 21, circ.input_size) for _ in range(6)] + [rng.integers(-900, 900, circ.input_size)]
        spec = g.native_spec()
        assert len(spec["buf_elems"]) < len(spec["layers"])  # values whose lifetimes end share buffers
        assert len(spec["layers"]) < len(circ.layers)  # elementwise layers fused into the layer before them
        bad, out = _simulate_spec(spec, X)
        assert bad == [i for i, x in enumerate(X) if g.violations_np(x)]
        for i, x in enumerate(X):
            if i not in bad:
                assert np.array_equal(out[i], circ.plain_q_eval(x, False, M_))


def test_maxpool_span_check():
    """A max-pooling window whose inputs are signed values but whose difference b - a is not (it would wrap in
    the pairwise max tree's ReLU gadget) is refused by every guard implementation."""
    Mm = crt_modulus(first_primes(3))  # 30: signed range [-15, 15)
    mp = d.MaxPool2d(2, 1, 1, 2, 1)
    c = d.Circuit([mp])
    g = RangeGuard(c, Mm, mrs=True)
    ok, wide = np.array([-7, 7]), np.array([-14, 14])
    assert not g.violations_np(ok) and g.violations_np(wide)
    assert g.submit([ok, wide]).bad_indices() == [1]
    assert _simulate_spec(g.native_spec(), [ok, wide])[0] == [1]


@pytest.mark.gpu
def test_native_guard_matches_numpy_on_gpu():
    """DevRangeGuard (csrc/hip/guard.hip) on the device: the flags of MiniONN and residual-circuit batches equal
    the numpy model's, across chunk boundaries, including an activation beyond the int32 operand range."""
    from dash_amd.ir.quant import QuantizationMethod
    from dash_amd.models import BENCH_CONFIGS, build_circuit, quantized_inputs

    cfg = BENCH_CONFIGS["MODEL_F_MINIONN_POOL_REPL/DASH"]
    qm = QuantizationMethod(cfg["q_method"])
    cm = build_circuit("MODEL_F_MINIONN_POOL_REPL", qm, cfg["q_parameter"], seed=0)
    MM = crt_modulus(first_primes(cfg["crt"]))
    xs = list(quantized_inputs("MODEL_F_MINIONN_POOL_REPL", 70, qm, cfg["q_parameter"], seed=3))
    xs[5] = xs[5] * 2000
    xs[66] = xs[66] * 2000
    xs[40] = xs[40] * (1 << 33)  # beyond the int32 operands: decided by the exact host model
    g = RangeGuard(cm, MM, mrs=True, device=0)
    assert g._native_ok()
    got = g.submit(xs).bad_indices()
    assert got == [i for i, x in enumerate(xs) if g.violations_np(x)]
    assert 5 in got and 66 in got and 40 in got and 0 not in got
    rc = _residual_circuit()
    Mr = crt_modulus(first_primes(4))
    rng = np.random.default_rng(1)
    X = [rng.integers(-20, 21, rc.input_size) for _ in range(9)] + [rng.integers(-900, 900, rc.input_size)]
    gr = RangeGuard(rc, Mr, mrs=True, device=0)
    assert gr.submit(X).bad_indices() == [i for i, x in enumerate(X) if gr.violations_np(x)]
    # two tickets in flight, waited out of order
    p1, p2 = g.submit(xs[:8]), g.submit(xs[60:70])
    assert p2.bad_indices() == [6] and p1.bad_indices() == [5]
    # a replayed check (same ticket and batch size) starts from clear flags and reads the new inputs
    for rep in range(3):
        assert g.submit(xs[8:16]).bad_indices() == []
        assert g.submit(xs[:8]).bad_indices() == [5]
