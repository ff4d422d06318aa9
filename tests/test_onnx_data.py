"""ONNX import/export and dataset readers.

Reference coverage: dash/test/test_onnx_modelloader.h (fixture
dash/test/fixtures/model_dense.onnx, read here in place — it is a data file,
decoded by our own protobuf reader; expected weights copied from the test).
"""
import os

import numpy as np
import pytest

from dash_amd import data
from dash_amd.garbling import GarbledCircuit
from dash_amd.ir.layers import Conv2d, Dense, Flatten, MaxPool2d, Relu, Rescale
from dash_amd.ir.circuit import Circuit
from dash_amd.ir.onnx import load_onnx_model, parse_onnx, save_onnx_model
from dash_amd.ir.quant import QuantizationMethod as Q

FIXTURE = "/root/reference/dash/test/fixtures/model_dense.onnx"


@pytest.mark.skipif(not os.path.exists(FIXTURE), reason="reference fixture not mounted")
def test_reference_dense_fixture():
    c = load_onnx_model(FIXTURE, Q.SimpleQuant, 10)
    assert c.input_dims == (1, 28, 28)
    assert c.output_dims == (10,)
    assert isinstance(c.layers[0], Flatten) and isinstance(c.layers[1], Dense)
    w = c.layers[1].weights.reshape(-1)
    b = c.layers[1].biases
    assert w[0] == np.float32(-0.02056167833507061004638671875)
    assert w[9] == np.float32(0.00375685538165271282196044921875)
    assert w[-1] == np.float32(0.018187098205089569091796875)
    assert b[0] == np.float32(-0.02799860946834087371826171875)
    assert b[4] == np.float32(-0.0069468836300075054168701171875)
    assert b[-1] == np.float32(-0.02649968676269054412841796875)


@pytest.mark.skipif(not os.path.exists(FIXTURE), reason="reference fixture not mounted")
def test_reference_fixture_scalequant_inserts_rescale():
    c = load_onnx_model(FIXTURE, Q.ScaleQuant, 3)
    assert [type(l).__name__ for l in c.layers] == ["Flatten", "Dense", "Rescale"]
    c = load_onnx_model(FIXTURE, Q.ScaleQuantPlus, 7)
    assert c.layers[2].s == [7]


def _small_cnn(seed=0):
    rng = np.random.default_rng(seed)
    conv = Conv2d(rng.normal(0, 0.3, (4, 1, 3, 3)), rng.normal(0, 0.1, 4), 8, 8, 1, 4, 3, 3, 1, 1, pad_width=1,
                  pad_height=1, q_const=0.05)
    pool = MaxPool2d(8, 8, 4, 2, 2)
    dense = Dense(rng.normal(0, 0.3, (5, 64)), rng.normal(0, 0.1, 5), q_const=0.05)
    return Circuit([conv, Relu(conv.out_dims), pool, Flatten(pool.out_dims), dense])


def test_export_import_roundtrip(tmp_path):
    c = _small_cnn()
    p = tmp_path / "m.onnx"
    save_onnx_model(p, c)
    m = parse_onnx(p)
    assert m["producer_name"] == "dash_amd"
    assert [n["op_type"] for n in m["nodes"]] == ["Conv", "Relu", "MaxPool", "Flatten", "Gemm"]
    assert m["nodes"][0]["attrs"]["pads"] == [1, 1, 1, 1]
    c2 = load_onnx_model(p, Q.SimpleQuant, -1, q_const=0.05)
    assert [type(l).__name__ for l in c2.layers] == [type(l).__name__ for l in c.layers]
    np.testing.assert_array_equal(c2.layers[0].weights, c.layers[0].weights)
    np.testing.assert_array_equal(c2.layers[4].weights, c.layers[4].weights)
    x = np.random.default_rng(1).normal(0, 1, 64).astype(np.float32)
    np.testing.assert_allclose(c2.plain_eval(x), c.plain_eval(x), rtol=1e-6)


def test_onnx_model_garbles(tmp_path):
    c = _small_cnn(3)
    p = tmp_path / "m.onnx"
    save_onnx_model(p, c)
    c2 = load_onnx_model(p, Q.SimpleQuant, -1, q_const=0.05)
    x = np.random.default_rng(2).integers(-20, 20, 64)
    k = c2.infer_crt_base_size([x])
    gc = GarbledCircuit(c2, k, 100.0, seed=bytes(16))
    out = gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x)))
    np.testing.assert_array_equal(out, gc.plain_q_eval(x))


def test_gemm_without_transb_and_batchnorm(tmp_path):
    """Hand-built graph: Gemm(transB=0) + BatchNormalization folded into a Conv."""
    from dash_amd.ir import onnx as ox

    rng = np.random.default_rng(5)
    W = rng.normal(0, 1, (2, 1, 3, 3)).astype(np.float32)
    B = rng.normal(0, 1, 2).astype(np.float32)
    gamma, beta = np.array([1.5, 0.5], np.float32), np.array([0.1, -0.2], np.float32)
    mean, var = np.array([0.3, -0.1], np.float32), np.array([2.0, 0.5], np.float32)
    G = rng.normal(0, 1, (8, 3)).astype(np.float32)  # [in][out], transB = 0
    nodes = (ox._node("Conv", ["x", "W", "B"], ["c"], "conv", ox._attr_ints("kernel_shape", [3, 3]))
             + ox._node("BatchNormalization", ["c", "g", "b", "m", "v"], ["bn"], "bn", ox._attr_float("epsilon", 1e-5))
             + ox._node("Flatten", ["bn"], ["f"], "flat", ox._attr_int("axis", 1))
             + ox._node("Gemm", ["f", "G"], ["y"], "fc"))
    inits = b"".join(ox._ld(5, ox._tensor(n, a)) for n, a in
                     [("W", W), ("B", B), ("g", gamma), ("b", beta), ("m", mean), ("v", var), ("G", G)])
    graph = nodes + inits + ox._ld(11, ox._value_info("x", (1, 1, 4, 4))) + ox._ld(12, ox._value_info("y", (1, 3)))
    blob = ox._i(1, 7) + ox._s(2, "pytorch") + ox._ld(7, graph)
    c = ox.create_circuit_from_onnx(ox.parse_onnx(blob), Q.SimpleQuant, 0.01)
    conv, dense = c.layers[0], c.layers[2]
    g = gamma / np.sqrt(var + 1e-5)
    np.testing.assert_allclose(conv.weights, W * g.reshape(-1, 1, 1, 1), rtol=1e-6)
    np.testing.assert_allclose(conv.biases, (B - mean) * g + beta, rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(dense.weights, G.T)


def test_mnist_cifar_readers(tmp_path):
    rng = np.random.default_rng(0)
    im = rng.integers(0, 256, (5, 1, 28, 28), dtype=np.uint8)
    lab = rng.integers(0, 10, 5)
    data.write_mnist(str(tmp_path / "mnist"), im, lab)
    d = data.mnist(str(tmp_path / "mnist"))
    assert d.test_images.shape == (5, 1, 28, 28) and d.train_images.shape[0] == 0
    np.testing.assert_allclose(d.test_images, im / 255.0, rtol=1e-6)
    np.testing.assert_array_equal(d.test_labels, lab)
    ci = rng.integers(0, 256, (3, 3, 32, 32), dtype=np.uint8)
    cl = rng.integers(0, 10, 3)
    data.write_cifar10(str(tmp_path / "cifar"), ci, cl)
    data.write_cifar10(str(tmp_path / "cifar"), ci[:2], cl[:2], name="data_batch_1.bin")
    d = data.cifar10(str(tmp_path / "cifar"))
    assert d.test_images.shape == (3, 3, 32, 32) and d.train_images.shape == (2, 3, 32, 32)
    np.testing.assert_allclose(d.test_images, ci / 255.0, rtol=1e-6)
    np.testing.assert_array_equal(d.test_labels, cl)
    n = data.normalize(d.test_images, data.CIFAR10_MEAN, data.CIFAR10_STD)
    np.testing.assert_allclose(n[:, 1], (ci[:, 1] / 255.0 - 0.4822) / 0.2435, rtol=1e-5, atol=1e-6)
    q = data.quantize(n, Q.ScaleQuant, 5)
    assert q.shape == (3, 3072) and q.dtype == np.int64


def test_reader_errors(tmp_path):
    from dash_amd.native import native

    with pytest.raises(RuntimeError):
        data.mnist(str(tmp_path / "missing"))
    with pytest.raises(RuntimeError):
        native().onnx_parse(b"\x0a\xff\xff")  # truncated
