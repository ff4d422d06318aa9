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
