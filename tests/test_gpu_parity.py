"""HIP evaluator vs host oracle: bit-exact labels for every layer type."""
import numpy as np
import pytest

import dash_amd as d
from dash_amd.garbling import GarbledCircuit

pytestmark = pytest.mark.gpu


def _hip(models, mfma=True):
    from dash_amd.runtime import HipEvaluator

    return HipEvaluator(models, mfma=mfma)


def _same(a: bytes, b: bytes) -> bool:
    """Byte identity of two serialized blobs (digests: pytest's diff of two multi-MB byte strings on a failure
    takes minutes)."""
    import hashlib

    return len(a) == len(b) and hashlib.sha256(a).digest() == hashlib.sha256(b).digest()


FUSED = pytest.mark.parametrize("fused", [True, False], ids=["fused", "refcasts"])


def _check(circuit, crt, mrs, xs, mfma=True, plain=True, fused=True, rescale="legacy", relu="approx", hardened=None):
    gcs = [GarbledCircuit(circuit, crt, mrs, seed=bytes([i + 1]) * 16, fused_sign=fused, rescale=rescale, relu=relu,
                          hardened=hardened)
           for i in range(len(xs))]
    enc = [g.garble_inputs(x) for g, x in zip(gcs, xs)]
    cpu = [g.cpu_evaluate(e) for g, e in zip(gcs, enc)]
    ev = _hip([g.model for g in gcs], mfma=mfma)
    gpu = ev.evaluate(enc)
    for c, g in zip(cpu, gpu):
        assert len(c) == len(g)
        for (pc, ac), (pg, ag) in zip(c, g):
            assert pc == pg
            np.testing.assert_array_equal(ac, ag)
    outs = [g.decode_outputs(o) for g, o in zip(gcs, gpu)]
    if plain:
        for g, x, o in zip(gcs, xs, outs):
            np.testing.assert_array_equal(o, g.plain_q_eval(x))
    return outs


def test_aes_parity(native):
    rng = np.random.default_rng(0)
    a = rng.integers(0, 2**63, size=(1000, 2), dtype=np.uint64)
    np.testing.assert_array_equal(native.hip_aes_hash_array(a), native.aes_hash_array(a))


def test_hard_pad_parity(native):
    """Hardened-encoding pads: the GPU's ChaCha12 (dev.h hard_block) == the host's (core.h), every word."""
    rng = np.random.default_rng(7)
    n = 600
    keys = rng.integers(0, 2**63, size=(n, 2), dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    gates = rng.integers(0, 2**62, size=n, dtype=np.uint64)
    subs = rng.integers(0, 2**31, size=n, dtype=np.uint64).astype(np.uint32)
    blks = rng.integers(0, 4, size=n, dtype=np.uint64).astype(np.uint32)
    dev = native.hip_hard_pads(keys, gates, subs, blks)
    for i in range(0, n, 37):
        K = int(keys[i, 0]) | (int(keys[i, 1]) << 64)
        host = native.hard_pads(K, int(gates[i]), int(subs[i]), int(blks[i]))
        for q in range(4):
            assert (int(dev[i, q, 0]) | (int(dev[i, q, 1]) << 64)) == host[q]


@pytest.mark.parametrize("hardened", [True, False], ids=["hardened", "reference"])
def test_dense_relu_encodings(hardened):
    """Both offline-message encodings through the HIP evaluator: labels bit-exact vs the host oracle."""
    rng = np.random.default_rng(11)
    W1 = rng.integers(-8, 9, (24, 30)); b1 = rng.integers(-8, 9, 24)
    c = d.Circuit([d.Dense.from_quantized(W1, b1), d.Relu((24,)), d.Dense.from_quantized(W1[:6, :24], b1[:6])])
    xs = [rng.integers(-20, 20, 30) for _ in range(3)]
    _check(c, 7, 100.0, xs, hardened=hardened)


@pytest.mark.parametrize("q", [2, 3, 5, 7, 11, 13, 17, 19, 23, 32, 56, 86, 97, 107, 167, 173])
def test_codec_parity(native, q):
    rng = np.random.default_rng(q)
    n = native.nr_comps(q)
    L = rng.integers(0, q, size=(500, n)).astype(np.int16)
    comp, dec = native.hip_codec(L, q)
    np.testing.assert_array_equal(dec, L)
    for i in range(0, 500, 97):
        c = int(comp[i, 0]) | (int(comp[i, 1]) << 64)
        assert c == native.compress(L[i], q)


def test_dense_relu():
    rng = np.random.default_rng(1)
    W1 = rng.integers(-8, 9, (20, 30)); b1 = rng.integers(-8, 9, 20)
    W2 = rng.integers(-8, 9, (5, 20)); b2 = rng.integers(-8, 9, 5)
    c = d.Circuit([d.Dense.from_quantized(W1, b1), d.Relu((20,)), d.Dense.from_quantized(W2, b2)])
    xs = [rng.integers(-20, 20, 30) for _ in range(3)]
    _check(c, 8, 100.0, xs)


@pytest.mark.parametrize("mfma", [False, True])
def test_conv(mfma):
    rng = np.random.default_rng(2)
    W = rng.integers(-5, 6, (8, 3, 3, 3)); b = rng.integers(-5, 6, 8)
    W2 = rng.integers(-5, 6, (4, 8, 2, 2)); b2 = rng.integers(-5, 6, 4)
    c = d.Circuit([d.Conv2d.from_quantized(W, b, 9, 9, 3, 8, 3, 3, 1, 1, pad_width=1, pad_height=1),
                   d.Conv2d.from_quantized(W2, b2, 9, 9, 8, 4, 2, 2, 2, 2)])
    xs = [rng.integers(-5, 6, 3 * 81) for _ in range(2)]
    _check(c, 9, None, xs, mfma=mfma)


@pytest.mark.parametrize("W,H,C,k,sw,sh,pad", [(30, 6, 5, 3, 1, 1, 0), (13, 5, 5, 3, 1, 1, 1), (8, 4, 5, 3, 1, 1, 0),
                                               (16, 6, 5, 5, 1, 1, 2), (21, 7, 5, 2, 2, 2, 0), (11, 5, 5, 3, 2, 2, 1),
                                               (12, 9, 3, 3, 1, 2, 1), (10, 6, 70, 3, 1, 1, 1)])
def test_conv_band_edges(W, H, C, k, sw, sh, pad):
    """Band staging of the MFMA conv: rows whose width is not a multiple of 8 (edge items as clamped loads),
    left/right padding, strides; few input channels take the tap-unrolled image (C * k * k <= 64 patch bytes as
    the channels of one 1x1 k-step), C = 70 the channel-chunked image. Labels bit-exact against the host."""
    rng = np.random.default_rng(W * 100 + H)
    F = 6
    Wt = rng.integers(-5, 6, (F, C, k, k)); b = rng.integers(-5, 6, F)
    c = d.Circuit([d.Conv2d.from_quantized(Wt, b, W, H, C, F, k, k, sw, sh, pad_width=pad, pad_height=pad)])
    xs = [rng.integers(-6, 7, C * H * W) for _ in range(2)]
    _check(c, 7, None, xs)


@pytest.mark.parametrize("crt", [7, [5, 7, 131]], ids=["base7", "p131_centered"])
def test_conv_many_images(crt):
    """Band conv over many images (3 GCs x every component of every residue) with the exact 24-bit epilogue
    reduction (small accumulator bound) and, for p = 131, the centered-operand path and the 32-bit reduction
    where the bound is too large; a 2x2 stride-2 conv follows. Labels bit-exact against the host."""
    rng = np.random.default_rng(31)
    C, F, H, W = 16, 32, 7, 7
    Wt = rng.integers(-5, 6, (F, C, 3, 3)); b = rng.integers(-5, 6, F)
    c = d.Circuit([d.Conv2d.from_quantized(Wt, b, W, H, C, F, 3, 3, 1, 1),
                   d.Conv2d.from_quantized(rng.integers(-5, 6, (16, F, 2, 2)), rng.integers(-5, 6, 16), 5, 5, F, 16,
                                           2, 2, 2, 2)])
    xs = [rng.integers(-6, 7, C * H * W) for _ in range(3)]
    # labels bit-exact vs the host always; the plaintext check only where the CRT range holds the values
    _check(c, crt, None, xs, plain=crt == 7)


@FUSED
def test_sign_edges(fused):
    vals = [0, 1, -1, 55773217, -55773217, 111546434, -111546435]
    c = d.Circuit([d.Sign((len(vals),))])
    _check(c, 9, [76, 7, 7, 7, 7, 7, 5, 5], [vals, vals[::-1]], fused=fused)


@FUSED
def test_relu_edges(fused):
    vals = [0, 1, -1, 7, -7, 14, -15]
    c = d.Circuit([d.Relu((len(vals),))])
    _check(c, [2, 3, 5], [26, 6, 3, 2], [vals], fused=fused)


@FUSED
@pytest.mark.parametrize("layer", ["relu", "sign"])
def test_single_digit_mrs(layer, fused):
    """ReLU/Sign accuracy 99 % with k = 8 selects a one-digit MRS base ([126]): no casts, no carry chain."""
    rng = np.random.default_rng(5)
    xs = [rng.integers(-1000, 1000, 64) for _ in range(2)]
    c = d.Circuit([d.Relu((64,)) if layer == "relu" else d.Sign((64,))])
    _check(c, 8, 99.0, xs, plain=False, fused=fused)  # approximate (99 %): GPU == host labels bit for bit


@FUSED
def test_rescale_legacy(fused):
    rng = np.random.default_rng(3)
    xs = [rng.integers(-100000, 100000, 300) for _ in range(2)]
    c = d.Circuit([d.Rescale(2, (300,))])
    _check(c, 9, 100.0, xs, fused=fused)


@pytest.mark.parametrize("k,l", [(7, 5), (9, 2), (4, 1), (11, 3)])
def test_rescale_mrs(k, l):
    """Single-shot mixed-radix rescale (chain + output kernels) == host oracle, bit for bit."""
    rng = np.random.default_rng(k + l)
    c = d.Circuit([d.Rescale(l, (300,))])
    h = GarbledCircuit(c, k, 100.0, garble_me=False).crt_modulus // 2
    xs = [rng.integers(-h, h - (1 << l), 300) for _ in range(2)]
    _check(c, k, 100.0, xs, rescale="mrs")


@pytest.mark.parametrize("relu", ["approx", "mrs", "joint"])
def test_minionn_head_mrs_rescale(relu):
    """MiniONN conv -> rescale(l=5) -> relu at full size with the mixed-radix rescale (and sign)."""
    from dash_amd.ir.quant import QuantizationMethod as Q
    from dash_amd.models import build_circuit, quantized_inputs

    full = build_circuit("MODEL_F_MINIONN_POOL_REPL", Q.ScaleQuant, 5, seed=0)
    c = d.Circuit(full.layers[:3])
    xs = quantized_inputs("MODEL_F_MINIONN_POOL_REPL", 2, Q.ScaleQuant, 5, seed=3)
    _check(c, 7, 100.0, xs, rescale="mrs", relu=relu)


@pytest.mark.parametrize("k", [2, 3, 7, 9])
def test_relu_mrs_sign(k):
    """Exact mixed-radix-sign ReLU (label hash + chain + mixed multiply kernels) == host oracle, edges included."""
    c0 = d.Circuit([d.Relu((1,))])
    h = GarbledCircuit(c0, k, None, garble_me=False).crt_modulus // 2
    rng = np.random.default_rng(k)
    vals = np.array([0, 1, -1, h - 1, -h, -h + 1, 2, -2] + list(rng.integers(-h, h, 120)), dtype=np.int64)
    c = d.Circuit([d.Relu((len(vals),))])
    _check(c, k, None, [vals, vals[::-1].copy()], relu="mrs")


@pytest.mark.parametrize("crt,mrs", [([32, 97, 107], [22, 19, 15, 13]), ([32, 3, 5, 7, 11, 13, 17], [10, 9, 9, 8, 7, 7, 6])])
def test_rescale_redash(crt, mrs):
    rng = np.random.default_rng(4)
    xs = [rng.integers(-100000, 100000, 200) for _ in range(2)]
    c = d.Circuit([d.Rescale([32], (200,))])
    _check(c, crt, mrs, xs)


@FUSED
def test_maxpool_sumpool_add(fused):
    rng = np.random.default_rng(5)
    c = d.Circuit([d.MaxPool2d(6, 6, 2, 2, 2), d.Add((2, 3, 3), 0), d.SumPool2d(3, 3, 2, 3, 3)])
    xs = [rng.integers(-50, 50, 72) for _ in range(2)]
    _check(c, 7, 100.0, xs, fused=fused)


def test_projection_mult_mixed():
    c = d.Circuit([d.Projection((4,), [19], [91], lambda v: v), d.Projection((4,), [91], [19], lambda v: v % 19)])
    _check(c, [19], None, [[0, 1, 5, 18]], plain=False)
    c = d.Circuit([d.MultLayer((4,))])
    _check(c, [19], None, [[2, -4, -1, -2]])
    c = d.Circuit([d.MixedModMultLayer((4,), smaller_modulus=2)])
    _check(c, [19], None, [[5, 1, -3, 0]])


def test_base_extension():
    rng = np.random.default_rng(6)
    c = d.Circuit([d.BaseExtension((20,), [32])])
    xs = [rng.integers(0, 97 * 107, 20)]
    gcs = GarbledCircuit(c, [32, 97, 107], [22, 19, 15, 13], seed=bytes(16))
    enc = gcs.garble_inputs(xs[0])
    ev = _hip([gcs.model])
    out = gcs.decode_outputs(ev.evaluate([enc])[0])
    np.testing.assert_array_equal(out, xs[0])


def test_model_a_batch():
    from dash_amd.models import build_circuit, quantized_inputs

    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 3)
    _check(c, 7, 100.0, xs)


def test_staged_input_paths():
    """encode_into / set_input_cm + upload_inputs == the label-list path."""
    from dash_amd.models import build_circuit, quantized_inputs

    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 2)
    gcs = [GarbledCircuit(c, 7, 100.0, seed=bytes([i + 9]) * 16) for i in range(2)]
    ev = _hip([g.model for g in gcs])
    ref = ev.evaluate([g.garble_inputs(x) for g, x in zip(gcs, xs)])
    ev.encode_into(0, gcs[0], xs[0])
    ev.set_input_cm(1, gcs[1].garble_inputs_cm(xs[1]))
    ev.upload_inputs()
    ev.run()
    got = ev.get_outputs()
    for r, g in zip(ref, got):
        for (pr, ar), (pg, ag) in zip(r, g):
            assert pr == pg
            np.testing.assert_array_equal(ar, ag)
    for g, x, o in zip(gcs, xs, got):
        np.testing.assert_array_equal(g.decode_outputs(o), g.plain_q_eval(x))


def test_compressed_wire_paths():
    """Compressed online messages (16 B per label) through the HIP evaluator."""
    from dash_amd.models import build_circuit, quantized_inputs

    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 3)
    gcs = [GarbledCircuit(c, 7, 100.0, seed=bytes([i + 20]) * 16) for i in range(3)]
    ev = _hip([g.model for g in gcs])
    ev.encode_compressed_into(0, gcs[0], xs[0])
    for b in (1, 2):
        ev.set_input_compressed(b, gcs[b].garble_inputs_compressed(xs[b]))
    ev.upload_inputs_compressed()
    ev.run()
    ev.fetch_outputs()
    for b, (g, x) in enumerate(zip(gcs, xs)):
        ref = g.plain_q_eval(x)
        np.testing.assert_array_equal(ev.decode(b, g), ref)
        np.testing.assert_array_equal(g.decode_compressed(ev.outputs_compressed(b)), ref)
    # a tampered output label must not decode
    bad = ev.outputs_compressed(0).copy()
    bad[0, 0, 0] ^= 1
    with pytest.raises(d.IntegrityError):
        gcs[0].decode_compressed(bad)


def test_graph_replay_matches_eager():
    """Runs 2+ replay the captured hipGraph; results must equal the eager run."""
    import torch

    from dash_amd.models import build_circuit, quantized_inputs
    from dash_amd.ir.quant import QuantizationMethod as Q

    c = build_circuit("MODEL_B_POOL_REPL", Q.ScaleQuant, 3, seed=4)
    xs = quantized_inputs("MODEL_B_POOL_REPL", 6, Q.ScaleQuant, 3)
    gcs = [GarbledCircuit(c, 8, 100.0, seed=bytes([i + 40]) * 16) for i in range(2)]
    ev = _hip([g.model for g in gcs])
    st = torch.cuda.Stream()
    for r in range(3):
        for b, g in enumerate(gcs):
            ev.encode_compressed_into(b, g, xs[2 * r + b])
        ev.upload_inputs_compressed(st)
        ev.run(st)
        ev.fetch_outputs(st)
        for b, g in enumerate(gcs):
            np.testing.assert_array_equal(ev.decode(b, g), g.plain_q_eval(xs[2 * r + b]))


def test_device_input_encoder():
    """Online message #1 written on the device by the garbler's encoder (k_encode_in) decodes like the host-encoded
    wire form, across graph replays on a side stream, for a host- and a GPU-garbled GC."""
    import torch

    from dash_amd.models import build_circuit, quantized_inputs
    from dash_amd.ir.quant import QuantizationMethod as Q

    c = build_circuit("MODEL_B_POOL_REPL", Q.ScaleQuant, 3, seed=4)
    xs = quantized_inputs("MODEL_B_POOL_REPL", 6, Q.ScaleQuant, 3)
    gcs = [GarbledCircuit(c, 8, 100.0, seed=bytes([50]) * 16),
           GarbledCircuit(c, 8, 100.0, seed=bytes([51]) * 16, device=0)]
    ev = _hip([g.model for g in gcs])
    encs = [g.device_input_encoder(0) for g in gcs]
    assert encs[0].input_size() == c.input_size
    st = torch.cuda.Stream()
    for r in range(3):
        for b, enc in enumerate(encs):
            ev.encode_device_into(b, enc, xs[2 * r + b], st)
        ev.run(st)
        ev.fetch_outputs(st)
        for b, g in enumerate(gcs):
            np.testing.assert_array_equal(ev.decode(b, g), g.plain_q_eval(xs[2 * r + b]))
    # the host wire path on the same slots still agrees (the encoder left no state in the evaluator)
    for b, g in enumerate(gcs):
        ev.encode_compressed_into(b, g, xs[b])
    ev.upload_inputs_compressed(st)
    ev.run(st)
    ev.fetch_outputs(st)
    for b, g in enumerate(gcs):
        np.testing.assert_array_equal(ev.decode(b, g), g.plain_q_eval(xs[b]))
    with pytest.raises(Exception, match="size"):
        ev.encode_device_into(0, encs[0], xs[0][:-1], st)
    # one two-slot encoder (a group's): both slots with one launch; a slot never armed is refused
    enc2 = gcs[0].device_input_encoder(0, 2)
    with pytest.raises(Exception, match="no GC"):
        ev.encode_device_into(0, enc2, np.stack([xs[2], xs[3]]), st)
    enc2.load(gcs[1].garbler, 1)
    for r in range(2):
        ev.encode_device_into(0, enc2, np.stack([xs[2 * r], xs[2 * r + 1]]), st)
        ev.run(st)
        ev.fetch_outputs(st)
        for b, g in enumerate(gcs):
            np.testing.assert_array_equal(ev.decode(b, g), g.plain_q_eval(xs[2 * r + b]))


def test_projection_shortcut_in_src():
    from tests.test_garbled_layers import _shortcut_block

    c, xs = _shortcut_block()
    k = c.infer_crt_base_size(xs)
    _check(c, k, 100.0, xs)


@FUSED
@pytest.mark.parametrize("name", ["relu", "sign", "rescale", "model_b", "minionn_head"])
def test_gpu_garbler_bit_identical(name, fused):
    """GPU garbler (ReLU / Sign / legacy rescale on the device) == CPU garbler, byte for byte."""
    from dash_amd.ir.circuit import Circuit
    from dash_amd.ir.layers import Relu, Rescale, Sign
    from dash_amd.ir.quant import QuantizationMethod as Q
    from dash_amd.models import build_circuit

    if name == "relu":
        c, k = Circuit([Relu((300,))]), 8
    elif name == "sign":
        c, k = Circuit([Sign((300,))]), 7
    elif name == "rescale":
        c, k = Circuit([Rescale(2, (300,))]), 7
    elif name == "model_b":
        c, k = build_circuit("MODEL_B_POOL_REPL", Q.ScaleQuant, 3, seed=1), 8
    else:
        full = build_circuit("MODEL_F_MINIONN_POOL_REPL", Q.ScaleQuant, 5, seed=0)
        c, k = Circuit(full.layers[:3]), 7  # conv, rescale(l=5), relu at full size
    seed = bytes(range(16))
    cpu = GarbledCircuit(c, k, 100.0, seed=seed, fused_sign=fused)
    gpu = GarbledCircuit(c, k, 100.0, seed=seed, device=0, fused_sign=fused)
    assert _same(gpu.model.serialize(), cpu.model.serialize())
    assert _same(gpu.decoder.serialize(), cpu.decoder.serialize())


@pytest.mark.parametrize("name", ["rescale", "minionn_head"])
def test_gpu_garbler_bit_identical_mrs_rescale(name):
    """GPU garbler of the mixed-radix rescale == host garbler, byte for byte."""
    from dash_amd.ir.circuit import Circuit
    from dash_amd.ir.layers import Rescale
    from dash_amd.ir.quant import QuantizationMethod as Q
    from dash_amd.models import build_circuit

    if name == "rescale":
        c, k = Circuit([Rescale(5, (300,))]), 7
    else:
        full = build_circuit("MODEL_F_MINIONN_POOL_REPL", Q.ScaleQuant, 5, seed=0)
        c, k = Circuit(full.layers[:4]), 7  # conv, rescale(l=5), relu, conv
    seed = bytes(range(16))
    cpu = GarbledCircuit(c, k, 100.0, seed=seed, rescale="mrs", relu="approx")
    gpu = GarbledCircuit(c, k, 100.0, seed=seed, device=0, rescale="mrs", relu="approx")
    assert _same(gpu.model.serialize(), cpu.model.serialize())
    assert _same(gpu.decoder.serialize(), cpu.decoder.serialize())


@pytest.mark.parametrize("name", ["relu", "minionn_head"])
def test_gpu_garbler_bit_identical_mrs_relu(name):
    """GPU garbler of the mixed-radix-sign ReLU == host garbler, byte for byte."""
    from dash_amd.ir.circuit import Circuit
    from dash_amd.ir.layers import Relu
    from dash_amd.ir.quant import QuantizationMethod as Q
    from dash_amd.models import build_circuit

    if name == "relu":
        c, k = Circuit([Relu((300,))]), 7
    else:
        full = build_circuit("MODEL_F_MINIONN_POOL_REPL", Q.ScaleQuant, 5, seed=0)
        c, k = Circuit(full.layers[:5]), 7  # conv, rescale, relu, conv, rescale
    seed = bytes(range(16))
    cpu = GarbledCircuit(c, k, 100.0, seed=seed, rescale="mrs", relu="mrs")
    gpu = GarbledCircuit(c, k, 100.0, seed=seed, device=0, rescale="mrs", relu="mrs")
    assert _same(gpu.model.serialize(), cpu.model.serialize())
    assert _same(gpu.decoder.serialize(), cpu.decoder.serialize())


@pytest.mark.parametrize("nb", [2, 3], ids=["b2_one_pass", "b3_two_kernels"])
@pytest.mark.parametrize("k,l", [(7, 5), (8, 3), (2, 1)])
def test_rescale_relu_joint(k, l, nb):
    """Joint rescale + ReLU (chain mode 2 writes the sign hash/color; batch <= 2: k_rescale_relu_out, else
    k_rescale_mrs_out_hash + k_relu_mult) == host oracle == relu(ceil(x / 2^l)), values around the sign
    threshold included."""
    mrs = 100.0 if k >= 4 else None
    c0 = d.Circuit([d.Relu((1,))])
    M = GarbledCircuit(c0, k, mrs, garble_me=False).crt_modulus
    S, h = 1 << l, M // 2
    rng = np.random.default_rng(k + l)
    vals = list(range(-2 * S - 2, 2 * S + 3)) + [-h, -h + 1] + list(rng.integers(-h, h - S, 100))
    x = np.array([v for v in vals if -h <= v < h - S], dtype=np.int64)  # the rescale's non-wrapping domain
    c = d.Circuit([d.Rescale(l, (len(x),)), d.Relu((len(x),))])
    xs = [x, x[::-1].copy(), np.roll(x, 7)][:nb]
    outs = _check(c, k, mrs, xs, rescale="mrs", relu="joint")
    np.testing.assert_array_equal(outs[0], np.maximum(-((-x) // S), 0))


@pytest.mark.parametrize("name", ["pair", "minionn_head"])
def test_gpu_garbler_bit_identical_joint_relu(name):
    """GPU garbler of the joint rescale + ReLU (sign_last rescale, relu_mult) == host garbler, byte for byte."""
    from dash_amd.ir.circuit import Circuit
    from dash_amd.ir.quant import QuantizationMethod as Q
    from dash_amd.models import build_circuit

    if name == "pair":
        c, k = d.Circuit([d.Rescale(3, (300,)), d.Relu((300,))]), 7
    else:
        full = build_circuit("MODEL_F_MINIONN_POOL_REPL", Q.ScaleQuant, 5, seed=0)
        c, k = Circuit(full.layers[:7]), 7  # conv, rescale, relu, conv, rescale, relu, conv
    seed = bytes(range(16))
    cpu = GarbledCircuit(c, k, 100.0, seed=seed, rescale="mrs", relu="joint")
    gpu = GarbledCircuit(c, k, 100.0, seed=seed, device=0, rescale="mrs", relu="joint")
    assert _same(gpu.model.serialize(), cpu.model.serialize())
    assert _same(gpu.decoder.serialize(), cpu.decoder.serialize())


@pytest.mark.parametrize("rescale,relu", [("mrs", "joint"), ("legacy", "approx")])
def test_gpu_garble_into_evaluator_slot(rescale, relu):
    """Zero-copy offline phase: the GPU garbler writes a GC's tables straight into an evaluator slot
    (HipEvaluator.sink). The slot then holds exactly the host garbler's tables (same seed), load() only adds the
    per-GC constants, and both slots decode to the plaintext outputs."""
    from dash_amd.ir.circuit import Circuit
    from dash_amd.ir.quant import QuantizationMethod as Q
    from dash_amd.models import build_circuit, quantized_inputs
    from dash_amd.runtime import HipEvaluator

    full = build_circuit("MODEL_F_MINIONN_POOL_REPL", Q.ScaleQuant, 5, seed=0)
    c, k = Circuit(full.layers[:5]), 7  # conv, rescale(l=5), relu, conv, rescale
    xs = quantized_inputs("MODEL_F_MINIONN_POOL_REPL", 2, Q.ScaleQuant, 5, seed=3)
    kw = dict(rescale=rescale, relu=relu)
    first = GarbledCircuit(c, k, 100.0, seed=bytes([7]) * 16, device=0, **kw)
    ev = HipEvaluator(template=first.model, batch=2, device=0)
    ev.load(0, first.model)
    seed = bytes(range(16))
    into = GarbledCircuit(c, k, 100.0, seed=seed, device=0, sink=ev.sink(1), **kw)
    host = GarbledCircuit(c, k, 100.0, seed=seed, **kw)
    assert _same(into.model.serialize(), host.model.serialize())  # the host copy is fetched from the slot itself
    ev.load(1, into.model)
    for b, gc in enumerate((first, into)):
        ev.encode_compressed_into(b, gc, xs[b])
    ev.upload_inputs_compressed()
    ev.run()
    ev.fetch_outputs()
    for b, gc in enumerate((first, into)):
        np.testing.assert_array_equal(ev.decode(b, gc), gc.plain_q_eval(xs[b]))


def _dense_layer(rng, fin, fout, channel_tf=0):
    return d.Dense(rng.integers(-4, 5, (fout, fin)), rng.integers(-6, 6, fout), q_const=1.0, channel_tf=channel_tf)


def _gpu_vs_host(c, crt, mrs, **kw):
    seed = bytes(range(16))
    cpu = GarbledCircuit(c, crt, mrs, seed=seed, **kw)
    gpu = GarbledCircuit(c, crt, mrs, seed=seed, device=0, **kw)
    assert _same(gpu.model.serialize(), cpu.model.serialize())
    assert _same(gpu.decoder.serialize(), cpu.decoder.serialize())
    return gpu


@pytest.mark.parametrize("name", ["dense", "dense_tf", "dense_zero_weights", "model_a", "lenet5", "sumpool",
                                  "maxpool_odd", "max", "shortcut", "redash_head", "redash_rescale2",
                                  "base_ext"])
def test_gpu_garbler_bit_identical_all_kinds(name):
    """Round 4: dense, sum / max pooling, residual add + in_src, the ReDash rescale (trans projections + base
    extension) and the base-extension layer garble on the device, byte-identical to the host garbler."""
    from dash_amd.ir.quant import QuantizationMethod as Q
    from dash_amd.models import BENCH_CONFIGS, build_circuit

    rng = np.random.default_rng(11)
    crt, mrs, kw = 8, 100.0, {}
    xs = [np.random.default_rng(5 + i).integers(-20, 20, 1) for i in range(2)]  # replaced per circuit below
    if name == "dense":
        c = d.Circuit([_dense_layer(rng, 300, 70)])
    elif name == "dense_tf":
        c = d.Circuit([_dense_layer(rng, 96, 33, channel_tf=3)])
    elif name == "dense_zero_weights":
        lay = _dense_layer(rng, 64, 20)
        lay.q_weights[:, ::3] = 0  # zero (and multiple-of-p) weights take the Z-label quirk
        lay.q_weights[:, 1::7] = 2 * 3 * 5
        c = d.Circuit([lay])
    elif name == "model_a":
        c = build_circuit("MODEL_A")
    elif name == "lenet5":
        c, crt = build_circuit("LENET5", Q.ScaleQuant, 3, seed=1), 8
    elif name == "sumpool":
        c = d.Circuit([d.SumPool2d(8, 8, 3, 4, 4), d.Relu((3, 2, 2))])
    elif name == "maxpool_odd":
        c = d.Circuit([d.MaxPool2d(9, 9, 2, 3, 3)])  # 9-value windows: levels with an odd carry
    elif name == "max":
        c = d.Circuit([d.Max((7,))])
    elif name == "shortcut":
        from tests.test_garbled_layers import _shortcut_block

        c, xs = _shortcut_block()
        crt = c.infer_crt_base_size(xs)  # sized for these inputs
    elif name == "redash_head":
        from dash_amd.models import quantized_inputs

        cfg = BENCH_CONFIGS["MODEL_F_MINIONN_POOL_REPL/REDASH_OPT"]
        full = build_circuit("MODEL_F_MINIONN_POOL_REPL", cfg["q_method"], cfg["q_parameter"], seed=0)
        c, crt, mrs = d.Circuit(full.layers[:4]), cfg["crt"], cfg["mrs"]  # conv, rescale({32}), relu, conv
        xs = quantized_inputs("MODEL_F_MINIONN_POOL_REPL", 2, cfg["q_method"], cfg["q_parameter"], seed=3)
    elif name == "redash_rescale2":
        c, crt, mrs = d.Circuit([d.Rescale([32], (200,))]), [32, 3, 5, 7, 11, 13, 17], [10, 9, 9, 8, 7, 7, 6]
    else:
        c, crt, mrs = d.Circuit([d.BaseExtension((50,), [32])]), [32, 97, 107], [22, 19, 15, 13]
    g = _gpu_vs_host(c, crt, mrs, **kw)
    if name in ("dense", "model_a", "maxpool_odd", "shortcut", "redash_head"):
        from dash_amd.runtime import HipEvaluator

        if xs[0].size != c.input_size:
            xs = [np.random.default_rng(5 + i).integers(-20, 20, c.input_size) for i in range(2)]
        ev = HipEvaluator(template=g.model, batch=1, device=0)
        ev.load(0, g.model)
        ev.encode_compressed_into(0, g, xs[0])
        ev.upload_inputs_compressed()
        ev.run()
        ev.fetch_outputs()
        np.testing.assert_array_equal(ev.decode(0, g), g.plain_q_eval(xs[0]))
