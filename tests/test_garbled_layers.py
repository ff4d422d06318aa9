"""End-to-end garbling tests (garble -> encode -> host evaluate -> decode vs the
plaintext reference), ported from the reference's gtest suite
(dash/test/test_dense.h, test_conv2d.h, test_sign.h, test_relu.h,
test_rescale.h, test_maxpool2d.h, test_projection.h, test_mult.h,
test_mixed_mod_mult.h) plus cases the reference never ran."""
import numpy as np
import pytest

import dash_amd as d
from dash_amd.garbling import GarbledCircuit

SEED = bytes(range(16))


def run(circuit, crt, mrs, x, seed=SEED, threads=0, fused=True):
    gc = GarbledCircuit(circuit, crt, mrs, seed=seed, nthreads=threads, fused_sign=fused)
    assert gc.model.sign_fused == fused
    return gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x))), gc


# ---------------------------------------------------------------- dense
DENSE_PARAMS = [
    (np.array([[1]]), np.array([0]), [5]),
    (np.array([[2, 3]]), np.array([1]), [4, -3]),
    (np.array([[1, 0], [0, 1]]), np.array([0, 0]), [7, -9]),
    (np.array([[1, -1, 2], [0, 0, 0]]), np.array([5, -5]), [3, 4, 5]),
    (np.array([[-3, 2], [4, -1], [0, 7]]), np.array([1, 2, 3]), [-2, 6]),
]


@pytest.mark.parametrize("W,b,x", DENSE_PARAMS)
def test_single_dense(W, b, x):
    c = d.Circuit([d.Dense.from_quantized(W, b)])
    out, _ = run(c, 8, None, x)
    np.testing.assert_array_equal(out, W @ np.array(x) + b)


def test_dense_random_100_50_and_two_layers():
    rng = np.random.default_rng(0)
    W1 = rng.integers(-20, 21, (50, 100)); b1 = rng.integers(-20, 21, 50)
    W2 = rng.integers(-20, 21, (10, 50)); b2 = rng.integers(-20, 21, 10)
    x = rng.integers(-20, 21, 100)
    c = d.Circuit([d.Dense.from_quantized(W1, b1), d.Dense.from_quantized(W2, b2)])
    out, _ = run(c, 8, None, x)
    np.testing.assert_array_equal(out, W2 @ (W1 @ x + b1) + b2)


def test_dense_channel_tf():
    rng = np.random.default_rng(1)
    W = rng.integers(-5, 6, (4, 12)); b = rng.integers(-5, 6, 4)
    x = rng.integers(-5, 6, 12)
    dn = d.Dense.from_quantized(W, b, channel_tf=3)
    out, gc = run(d.Circuit([dn]), 8, None, x)
    np.testing.assert_array_equal(out, gc.plain_q_eval(x))


# ----------------------------------------------------------------- conv
def naive_conv(x, W, b, C, H, Wd, s=(1, 1), p=(0, 0)):
    F, _, kh, kw = W.shape
    xp = np.pad(x.reshape(C, H, Wd), ((0, 0), (p[0], p[0]), (p[1], p[1])))
    OH = (H + 2 * p[0] - kh) // s[0] + 1
    OW = (Wd + 2 * p[1] - kw) // s[1] + 1
    out = np.zeros((F, OH, OW), np.int64)
    for f in range(F):
        for y in range(OH):
            for xx in range(OW):
                out[f, y, xx] = np.sum(W[f] * xp[:, y * s[0]:y * s[0] + kh, xx * s[1]:xx * s[1] + kw]) + b[f]
    return out.reshape(-1)


CONV_PARAMS = [  # (C, H, W, F, kh, kw, sh, sw, ph, pw)
    (1, 3, 3, 1, 1, 1, 1, 1, 0, 0),   # identity
    (1, 4, 4, 1, 2, 2, 1, 1, 0, 0),   # 2x2
    (3, 5, 5, 1, 3, 3, 1, 1, 0, 0),   # multi channel
    (2, 5, 5, 4, 3, 3, 1, 1, 0, 0),   # multi filter
    (2, 6, 6, 3, 2, 2, 2, 2, 0, 0),   # stride 2
    (2, 6, 7, 3, 2, 3, 1, 2, 0, 0),   # non-square kernel (reference bug §2.7 #2)
    (3, 5, 5, 2, 3, 3, 1, 1, 1, 1),   # same padding
]


@pytest.mark.parametrize("p", CONV_PARAMS)
def test_conv(p):
    C, H, W_, F, kh, kw, sh, sw, ph, pw = p
    rng = np.random.default_rng(sum(p))
    W = rng.integers(-6, 7, (F, C, kh, kw)); b = rng.integers(-6, 7, F)
    x = rng.integers(-8, 9, C * H * W_)
    conv = d.Conv2d.from_quantized(W, b, W_, H, C, F, kw, kh, sw, sh, pad_width=pw, pad_height=ph)
    out, _ = run(d.Circuit([conv]), 8, None, x)
    np.testing.assert_array_equal(out, naive_conv(x, W, b, C, H, W_, (sh, sw), (ph, pw)))


def test_two_conv_random():
    rng = np.random.default_rng(3)
    W1 = rng.integers(-3, 4, (4, 3, 4, 4)); b1 = rng.integers(-3, 4, 4)
    W2 = rng.integers(-3, 4, (2, 4, 3, 3)); b2 = rng.integers(-3, 4, 2)
    c1 = d.Conv2d.from_quantized(W1, b1, 16, 16, 3, 4, 4, 4, 2, 2)
    c2 = d.Conv2d.from_quantized(W2, b2, 7, 7, 4, 2, 3, 3)
    x = rng.integers(-4, 5, 3 * 16 * 16)
    out, gc = run(d.Circuit([c1, c2]), 8, None, x)
    np.testing.assert_array_equal(out, gc.plain_q_eval(x))


# ------------------------------------------------------ sign / relu edges
SIGN_PARAMS = [
    ([2, 3, 5], [26, 6, 3, 2], [0, 1, -1, 7, -7, 14, -15]),
    (9, [76, 7, 7, 7, 7, 7, 5, 5], [0, 1, -1, 7, -7, 55773217, -55773217, 111546434, -111546435]),
]


# both sign constructions: fused casts (default) and the reference's explicit casts
FUSED = pytest.mark.parametrize("fused", [True, False], ids=["fused", "refcasts"])


@FUSED
@pytest.mark.parametrize("crt,mrs,vals", SIGN_PARAMS)
def test_sign(crt, mrs, vals, fused):
    out, _ = run(d.Circuit([d.Sign((len(vals),))]), crt, mrs, vals, fused=fused)
    np.testing.assert_array_equal(out, np.where(np.array(vals) >= 0, 1, -1))


@FUSED
@pytest.mark.parametrize("crt,mrs,vals", SIGN_PARAMS)
def test_relu(crt, mrs, vals, fused):
    out, _ = run(d.Circuit([d.Relu((len(vals),))]), crt, mrs, vals, fused=fused)
    np.testing.assert_array_equal(out, np.maximum(vals, 0))


@pytest.mark.parametrize("k,acc", [(4, 100.0), (5, 100.0), (6, 100.0), (7, 100.0), (8, 100.0), (9, 100.0), (7, 99.99)])
@FUSED
def test_relu_mrs_table(k, acc, fused):
    from dash_amd.ir.bases import crt_modulus, first_primes

    M = crt_modulus(first_primes(k))
    rng = np.random.default_rng(k)
    vals = rng.integers(-M // 2, M // 2, 40)
    out, _ = run(d.Circuit([d.Relu((40,))]), k, acc, vals, fused=fused)
    if acc == 100.0:
        np.testing.assert_array_equal(out, np.maximum(vals, 0))
    else:  # approximate: wrong only very close to 0 / M/2
        assert np.mean(out == np.maximum(vals, 0)) > 0.9


# -------------------------------------------------------------- rescale
RESCALE_VALS = [0, 1, -1, 7, -7, 14, -15, 55773217, -55773217, 111546434, -111546435]


@FUSED
def test_rescale_legacy_reference_case(fused):
    c = d.Circuit([d.Rescale(2, (len(RESCALE_VALS),))])
    out, _ = run(c, 9, 100.0, RESCALE_VALS, fused=fused)
    expected = -((-np.array(RESCALE_VALS)) // 4)  # ceil(ceil(x/2)/2)
    np.testing.assert_array_equal(out, expected)


@pytest.mark.parametrize("crt,mrs,s", [([32, 97, 107], [22, 19, 15, 13], [32]),
                                       ([32, 167, 173], [26, 25, 21, 13], [32]),
                                       ([2, 3, 5, 7, 11, 13, 17], [86, 7, 6, 6, 5], [2, 3]),
                                       ([32, 3, 5, 7, 11, 13, 17], [10, 9, 9, 8, 7, 7, 6], [32])])
def test_rescale_redash(crt, mrs, s):
    rng = np.random.default_rng(len(crt))
    x = rng.integers(-100000, 100000, 64)
    c = d.Circuit([d.Rescale(s, (64,))])
    out, gc = run(c, crt, mrs, x)
    np.testing.assert_array_equal(out, c.plain_q_eval(x, False, gc.crt_modulus))


def test_base_extension():
    rng = np.random.default_rng(9)
    x = rng.integers(0, 97 * 107, 30)
    out, _ = run(d.Circuit([d.BaseExtension((30,), [32])]), [32, 97, 107], [22, 19, 15, 13], x)
    np.testing.assert_array_equal(out, x)


# -------------------------------------------------------------- pooling
@pytest.mark.parametrize("C,H,W,k,s", [(1, 2, 2, 2, 2), (2, 4, 4, 2, 2), (1, 3, 3, 1, 1), (3, 6, 6, 3, 3), (2, 5, 5, 2, 1)])
@FUSED
def test_maxpool(C, H, W, k, s, fused):
    rng = np.random.default_rng(C * H + k)
    x = rng.integers(-1000, 1000, C * H * W)
    mp = d.MaxPool2d(W, H, C, k, k, s, s)
    out, _ = run(d.Circuit([mp]), 7, 100.0, x, fused=fused)
    np.testing.assert_array_equal(out, mp.plain_q_eval(x))


def test_max_and_sumpool_and_residual():
    x = [5, -3, 12, 7]
    out, _ = run(d.Circuit([d.Max((4,))]), 6, 100.0, x)
    assert out[0] == 12
    rng = np.random.default_rng(4)
    x = rng.integers(-30, 30, 2 * 4 * 4)
    c = d.Circuit([d.SumPool2d(4, 4, 2, 2, 2), d.Add((2, 2, 2), 0), d.Relu((2, 2, 2))])
    out, gc = run(c, 7, 100.0, x)
    np.testing.assert_array_equal(out, gc.plain_q_eval(x))


# --------------------------------------------------------- gate layers
def test_projection_up_and_down():
    c = d.Circuit([d.Projection((3,), [19], [91], lambda v: v), d.Projection((3,), [91], [19], lambda v: v % 19)])
    gc = GarbledCircuit(c, [19], None, seed=SEED)
    res = gc.decoder.decode_residues(gc.cpu_evaluate(gc.garble_inputs([0, 5, 18])))
    np.testing.assert_array_equal(res[0], [0, 5, 18])
    c = d.Circuit([d.Projection((3,), [19], [10], lambda v: v % 10), d.Projection((3,), [10], [19], lambda v: v)])
    gc = GarbledCircuit(c, [19], None, seed=SEED)
    res = gc.decoder.decode_residues(gc.cpu_evaluate(gc.garble_inputs([3, 9, 12])))
    np.testing.assert_array_equal(res[0], [3, 9, 2])


MULT = [[0, 0], [0, 2], [0, -2], [2, 1], [2, 2], [2, 4], [-2, 1], [-2, 2], [-2, 4], [-1, -1], [-1, -2], [-1, -4]]


@pytest.mark.parametrize("v", MULT)
def test_mult(v):
    out, _ = run(d.Circuit([d.MultLayer((2,))]), [19], None, v)
    assert out[0] == v[0] * v[1]


def test_mult_multi_residue():
    out, _ = run(d.Circuit([d.MultLayer((4,))]), 5, None, [23, -45, -7, 9])
    np.testing.assert_array_equal(out, [23 * -45, -63])


@pytest.mark.parametrize("v", [[5, 1], [5, 0], [-3, 1], [0, 1], [8, 1]])
def test_mixed_mod_mult(v):
    out, _ = run(d.Circuit([d.MixedModMultLayer((2,), smaller_modulus=2)]), [19], None, v)
    assert out[0] == v[0] * v[1]


def test_sign_dense_model_e():
    rng = np.random.default_rng(11)
    W1 = rng.integers(-3, 4, (10, 20)); b1 = rng.integers(-3, 4, 10)
    W2 = rng.integers(-3, 4, (4, 10)); b2 = rng.integers(-3, 4, 4)
    c = d.Circuit([d.Dense.from_quantized(W1, b1), d.Sign((10,)), d.Dense.from_quantized(W2, b2)])
    x = rng.integers(-5, 6, 20)
    out, gc = run(c, 5, 100.0, x)
    np.testing.assert_array_equal(out, gc.plain_q_eval(x))


def test_encode_cm_matches_encode():
    from dash_amd.models import build_circuit, quantized_inputs

    c = build_circuit("MODEL_A")
    x = quantized_inputs("MODEL_A", 1)[0]
    gc = GarbledCircuit(c, 7, 100.0, seed=SEED)
    lab = gc.garble_inputs(x)
    cm = gc.garble_inputs_cm(x)
    assert len(cm) == len(lab)
    for (p, a), b in zip(lab, cm):
        np.testing.assert_array_equal(a.T, b)


def _shortcut_block(seed=0):
    """conv -> relu -> [main: strided conv, relu, conv] + [shortcut: 1x1 strided conv on the block input] -> relu"""
    from dash_amd.ir.circuit import Circuit
    from dash_amd.ir.layers import Add, Conv2d, Relu

    rng = np.random.default_rng(seed)
    c0 = Conv2d(rng.integers(-3, 4, (4, 2, 3, 3)), rng.integers(-5, 5, 4), 6, 6, 2, 4, 3, 3, 1, 1, pad_width=1,
                pad_height=1, q_const=1.0)
    ca = Conv2d(rng.integers(-3, 4, (8, 4, 3, 3)), rng.integers(-5, 5, 8), 6, 6, 4, 8, 3, 3, 2, 2, pad_width=1,
                pad_height=1, q_const=1.0)
    cb = Conv2d(rng.integers(-3, 4, (8, 8, 3, 3)), rng.integers(-5, 5, 8), 3, 3, 8, 8, 3, 3, 1, 1, pad_width=1,
                pad_height=1, q_const=1.0)
    cs = Conv2d(rng.integers(-3, 4, (8, 4, 1, 1)), rng.integers(-5, 5, 8), 6, 6, 4, 8, 1, 1, 2, 2, q_const=1.0)
    cs.in_src = 1  # reads the block input (output of layer 1)
    c = Circuit([c0, Relu(c0.out_dims), ca, Relu(ca.out_dims), cb, cs, Add(cb.out_dims, 4), Relu(cb.out_dims)])
    xs = [rng.integers(-4, 5, c.input_size) for _ in range(3)]
    return c, xs


def test_projection_shortcut_in_src():
    c, xs = _shortcut_block()
    k = c.infer_crt_base_size(xs)
    for x in xs:
        out, _ = run(c, k, 100.0, x)
        ref = GarbledCircuit(c, k, 100.0, garble_me=False).plain_q_eval(x)
        np.testing.assert_array_equal(out, ref)


def test_resnet18_zoo_has_projection_shortcuts():
    from dash_amd.models import build_circuit

    c = build_circuit("RESNET18")
    srcs = [l.in_src for l in c.layers if l.in_src is not None]
    assert len(srcs) == 3  # stages 2-4 change width / stride
    specs = c.garble_specs()
    assert sum("in_src" in p for _, p in specs) == 3


def test_fused_sign_drops_cast_tables_and_roundtrips():
    """The fused construction stores no cast1 tables (k (t-1) + (t-1) fewer projections per sign gadget) and
    survives serialization with its construction flag."""
    vals = [0, 1, -1, 7, -7, 14, -15]
    c = d.Circuit([d.Relu((len(vals),))])
    gf = GarbledCircuit(c, [2, 3, 5], [26, 6, 3, 2], seed=SEED, fused_sign=True)
    gr = GarbledCircuit(c, [2, 3, 5], [26, 6, 3, 2], seed=SEED, fused_sign=False)
    assert "s.cast1" not in gf.model.layer_arrays(0) and "s.cast1" in gr.model.layer_arrays(0)
    assert gf.model.table_bytes() < gr.model.table_bytes()
    m2 = type(gf.model).deserialize(gf.model.serialize())
    assert m2.sign_fused
    gf.model = m2
    np.testing.assert_array_equal(gf.decode_outputs(gf.cpu_evaluate(gf.garble_inputs(vals))), np.maximum(vals, 0))


# ------------------------------------------- mixed-radix rescale (construction of the legacy function)
def _mrs_shift(M, S):
    """(U, q) of gadgets.h RescaleMrsPlan: x_u = (x + U) mod M, y = floor(x_u / S) - q."""
    h = M // 2
    U = h + (S - 1 - h % S) % S
    return U, (U - (S - 1)) // S


@pytest.mark.parametrize("k,l", [(7, 5), (7, 1), (8, 3), (9, 2), (4, 4)])
def test_rescale_mrs_equals_legacy_function(k, l):
    """ceil(x / 2^l) on the whole signed range except the top U - M/2 values (which wrap)."""
    c0 = d.Circuit([d.Rescale(l, (1,))])
    M = GarbledCircuit(c0, k, 100.0, seed=SEED, garble_me=False).crt_modulus
    S = 1 << l
    U, q = _mrs_shift(M, S)
    top = M // 2 - (U - M // 2)  # first wrapping value
    rng = np.random.default_rng(k * 100 + l)
    vals = [v for v in RESCALE_VALS if -M // 2 <= v < top]
    vals += [-M // 2, -M // 2 + 1, top - 1, top - 2, 0, S, -S, S - 1, 1 - S]
    vals += list(rng.integers(-M // 2, top, 48))
    x = np.array(vals, dtype=np.int64)
    c = d.Circuit([d.Rescale(l, (len(x),))])
    gc = GarbledCircuit(c, k, 100.0, seed=SEED, rescale="mrs")
    out = gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x)))
    np.testing.assert_array_equal(out, -((-x) // S))
    # == the legacy gadget's plaintext semantics (l halvings) on this domain
    np.testing.assert_array_equal(out, c.plain_q_eval(x, False, M))
    # the wrapping top values follow floor(((x + U) mod M) / S) - q
    xt = np.arange(top, M // 2, dtype=np.int64)
    if xt.size:
        ct = d.Circuit([d.Rescale(l, (xt.size,))])
        # the garbler's exact range guard refuses the band; with it off, the wrapped values are what decode
        from dash_amd.garbling.guard import RangeGuardError

        with pytest.raises(RangeGuardError):
            GarbledCircuit(ct, k, 100.0, seed=SEED, rescale="mrs").garble_inputs(xt)
        gt = GarbledCircuit(ct, k, 100.0, seed=SEED, rescale="mrs", range_guard="off")
        ot = gt.decode_outputs(gt.cpu_evaluate(gt.garble_inputs(xt)))
        exp = ((xt + U) % M) // S - q
        exp = np.where(exp >= M // 2, exp - M, exp)
        np.testing.assert_array_equal(ot, exp)


def test_rescale_mrs_tables_and_model():
    """One table per rescale layer (no sign gadget), far smaller than the legacy l iterations; a conv ->
    rescale -> relu -> dense model garbled with it decodes to the plaintext quantized output."""
    from dash_amd.ir.quant import QuantizationMethod as Q
    from dash_amd.models import build_circuit, quantized_inputs

    c = build_circuit("MODEL_B_POOL_REPL", Q.ScaleQuant, 3, seed=1)
    xs = quantized_inputs("MODEL_B_POOL_REPL", 3, Q.ScaleQuant, 3, seed=5)
    new = GarbledCircuit(c, 8, 100.0, seed=SEED, rescale="mrs")
    old = GarbledCircuit(c, 8, 100.0, seed=SEED, rescale="legacy")
    assert new.table_bytes < old.table_bytes / 2
    for x in xs:
        y = new.decode_outputs(new.cpu_evaluate(new.garble_inputs(x)))
        np.testing.assert_array_equal(y, new.plain_q_eval(x))
    from dash_amd.native import native

    blob = new.model.serialize()
    m2 = native().GarbledModel.deserialize(blob)
    assert m2.serialize() == blob
    y = new.decode_outputs(native().cpu_evaluate(m2, new.garble_inputs(xs[0]), 0))
    np.testing.assert_array_equal(y, new.plain_q_eval(xs[0]))


# ---------------------------------------------- exact mixed-radix sign for the ReLU
@pytest.mark.parametrize("k", [2, 3, 4, 7, 9])
def test_relu_mrs_sign_exact(k):
    """ReLU with the exact mixed-radix sign: max(x, 0) on the whole signed range, edges included."""
    c0 = d.Circuit([d.Relu((1,))])
    M = GarbledCircuit(c0, k, None, seed=SEED, garble_me=False).crt_modulus
    h = M // 2
    rng = np.random.default_rng(k)
    vals = [0, 1, -1, h - 1, -h, -h + 1, h - 2, 2, -2] + list(rng.integers(-h, h, 40))
    x = np.array(vals, dtype=np.int64)
    c = d.Circuit([d.Relu((len(x),))])
    gc = GarbledCircuit(c, k, None, seed=SEED, relu="mrs")  # no approximate-sign MRS base needed
    out = gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x)))
    np.testing.assert_array_equal(out, np.maximum(x, 0))


def test_relu_mrs_tables_and_model():
    """MODEL_B with both mixed-radix constructions decodes to the plaintext output; ReLU tables shrink."""
    from dash_amd.ir.quant import QuantizationMethod as Q
    from dash_amd.models import build_circuit, quantized_inputs

    c = build_circuit("MODEL_B_POOL_REPL", Q.ScaleQuant, 3, seed=1)
    xs = quantized_inputs("MODEL_B_POOL_REPL", 3, Q.ScaleQuant, 3, seed=6)
    both = GarbledCircuit(c, 8, 100.0, seed=SEED, rescale="mrs", relu="mrs")
    resc = GarbledCircuit(c, 8, 100.0, seed=SEED, rescale="mrs", relu="approx")
    assert both.table_bytes < resc.table_bytes
    for x in xs:
        y = both.decode_outputs(both.cpu_evaluate(both.garble_inputs(x)))
        np.testing.assert_array_equal(y, both.plain_q_eval(x))


# -------------------------------- joint rescale + ReLU: the rescale's conversion yields the ReLU's sign
@pytest.mark.parametrize("k,l", [(7, 5), (7, 1), (8, 3), (4, 4), (2, 1)])
def test_rescale_relu_joint_exact(k, l):
    """relu(ceil(x / 2^l)) with the sign taken from the rescale's mixed-radix digit of residue 2 (converted
    last): exact on the rescale's domain, values around 0 (where the sign threshold sits) included."""
    mrs = 100.0 if k >= 4 else None
    c0 = d.Circuit([d.Rescale(l, (1,))])
    M = GarbledCircuit(c0, k, mrs, seed=SEED, garble_me=False).crt_modulus
    S = 1 << l
    U, q = _mrs_shift(M, S)
    top = M // 2 - (U - M // 2)
    rng = np.random.default_rng(k * 31 + l)
    vals = [-M // 2, -M // 2 + 1, top - 1, top - 2, 0, 1, -1, 2, S, -S, S - 1, 1 - S, S + 1, -S - 1]
    vals += list(range(-2 * S - 2, 2 * S + 3))
    vals += list(rng.integers(-M // 2, top, 48))
    x = np.array([v for v in vals if -M // 2 <= v < top], dtype=np.int64)
    n = len(x)
    c = d.Circuit([d.Rescale(l, (n,)), d.Relu((n,))])
    gc = GarbledCircuit(c, k, mrs, seed=SEED, rescale="mrs", relu="joint")
    assert list(gc.model.layer_params(1)["smode"]) == [2]
    assert list(gc.model.layer_params(0)["sign_out"]) == [1]
    out = gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x)))
    np.testing.assert_array_equal(out, np.maximum(-((-x) // S), 0))


def test_rescale_relu_joint_model():
    """MODEL_B with joint rescale + ReLU decodes to the plaintext output; the joint ReLUs carry only the
    mixed-modulus half-gate tables, and the model survives serialization."""
    from dash_amd.ir.quant import QuantizationMethod as Q
    from dash_amd.models import build_circuit, quantized_inputs
    from dash_amd.native import native

    c = build_circuit("MODEL_B_POOL_REPL", Q.ScaleQuant, 3, seed=1)
    xs = quantized_inputs("MODEL_B_POOL_REPL", 3, Q.ScaleQuant, 3, seed=7)
    joint = GarbledCircuit(c, 8, 100.0, seed=SEED, rescale="mrs", relu="joint")
    resc = GarbledCircuit(c, 8, 100.0, seed=SEED, rescale="mrs", relu="approx")
    assert joint.table_bytes < resc.table_bytes
    nj = sum(1 for i in range(joint.model.num_layers) if list(joint.model.layer_params(i).get("smode", [])) == [2])
    assert nj >= 1
    for x in xs:
        y = joint.decode_outputs(joint.cpu_evaluate(joint.garble_inputs(x)))
        np.testing.assert_array_equal(y, joint.plain_q_eval(x))
    blob = joint.model.serialize()
    m2 = native().GarbledModel.deserialize(blob)
    y = joint.decode_outputs(native().cpu_evaluate(m2, joint.garble_inputs(xs[0]), 0))
    np.testing.assert_array_equal(y, joint.plain_q_eval(xs[0]))


def test_rescale_mrs_wrap_band_guard():
    """The mixed-radix rescale wraps on the top U - M/2 values below M/2. M = 2*3*5*7 = 210, l = 2: U = 107, so
    inputs 103, 104 wrap. A calibrated circuit whose tracked rescale input reaches the band is refused with
    rescale="mrs", "auto" falls back to the reference construction (exact there), and infer_crt_base_size
    reserves the band."""
    crt, l, M = [2, 3, 5, 7], 2, 210
    band = np.arange(M // 2 - (1 << l), M // 2, dtype=np.int64)  # M/2 - 2^l ... M/2 - 1 = 101..104
    c = d.Circuit([d.Rescale(l, (band.size,))])
    assert c.layers[0].mrs_limit(M) == 103
    # unguarded (never calibrated, run-time guard off): the mixed-radix construction really does differ on 103, 104
    raw = GarbledCircuit(c, crt, 100.0, seed=SEED, rescale="mrs", range_guard="off")
    out = raw.decode_outputs(raw.cpu_evaluate(raw.garble_inputs(band)))
    ref = c.plain_q_eval(band, False, M)
    assert np.array_equal(out[:2], ref[:2]) and not np.array_equal(out[2:], ref[2:])
    # calibrated on the band: refused / auto -> legacy, which matches the reference semantics
    c.calibrate([band])
    assert c.mrs_rescale_violations(M) == [(0, 104, 103)]
    with pytest.raises(ValueError, match="wrap band"):
        GarbledCircuit(c, crt, 100.0, seed=SEED, rescale="mrs")
    auto = GarbledCircuit(c, crt, 100.0, seed=SEED)
    assert auto.rescale == "legacy" and auto.relu == "approx"
    np.testing.assert_array_equal(auto.decode_outputs(auto.cpu_evaluate(auto.garble_inputs(band))), ref)
    # CRT sizing reserves 2^l below M/2 for every rescale input: 104 + 4 > 105 -> one more prime than 2*104 needs
    assert c.required_crt_modulus(rescale_margin=False) == 2 * 104
    assert c.required_crt_modulus() == 2 * (104 + 4)
    assert c.infer_crt_base_size([band], rescale_margin=False) == 4
    assert c.infer_crt_base_size([band]) == 5
    # just below the band without a further 2^l of headroom: explicit "mrs" is exact, "auto" stays legacy
    near = np.arange(99, 103, dtype=np.int64)
    c1 = d.Circuit([d.Rescale(l, (near.size,))]).calibrate([near])
    assert GarbledCircuit(c1, crt, 100.0, seed=SEED, garble_me=False).rescale == "legacy"
    g1 = GarbledCircuit(c1, crt, 100.0, seed=SEED, rescale="mrs")
    np.testing.assert_array_equal(g1.decode_outputs(g1.cpu_evaluate(g1.garble_inputs(near))),
                                  c1.plain_q_eval(near, False, M))
    # well below the band: calibrated auto picks the mixed-radix construction and it is exact
    ok = np.arange(90, 99, dtype=np.int64)
    c2 = d.Circuit([d.Rescale(l, (ok.size,))]).calibrate([ok])
    g2 = GarbledCircuit(c2, crt, 100.0, seed=SEED)
    assert g2.rescale == "mrs" and g2.relu == "joint"
    np.testing.assert_array_equal(g2.decode_outputs(g2.cpu_evaluate(g2.garble_inputs(ok))), c2.plain_q_eval(ok, False, M))
