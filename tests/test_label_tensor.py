"""LabelTensor algebra and codecs (reference dash/test/test_label.h)."""
import numpy as np

from dash_amd.garbling import GarbledCircuit
from dash_amd.models import build_circuit, quantized_inputs
from dash_amd.ops import LabelTensor
from tests.aes_ref import dash_hash


def test_algebra_matches_label_semantics():
    c = build_circuit("MODEL_A")
    x = quantized_inputs("MODEL_A", 1)[0]
    gc = GarbledCircuit(c, 5, 100.0, seed=bytes(16))
    L = LabelTensor.from_labels(gc.garble_inputs(x), shape=(1, 28, 28))
    assert L.shape == (1, 28, 28) and L.size == 784
    Z = LabelTensor.zeros(L.moduli, L.shape)
    assert L + Z == L and L - L == Z and -(-L) == L
    assert (L * 3) == L + L + L
    assert L * 0 == Z
    # matvecmul with identity keeps labels; with 2*I doubles them
    sub = L[0, 0, :4]
    assert sub.size == 4
    assert sub.matvecmul(np.eye(4, dtype=np.int64)) == sub
    assert sub.matvecmul(2 * np.eye(4, dtype=np.int64)) == sub + sub


def test_compress_decompress_hash():
    rng = np.random.default_rng(3)
    L = LabelTensor.random([2, 3, 5, 7, 11, 13, 17, 19], (10,), rng)
    C = L.compress()
    assert C.shape == (8, 10, 2)
    assert LabelTensor.decompress(C, L.moduli) == L
    H = L.hash()
    for j in (0, 5):
        for e in (0, 9):
            c = int(C[j, e, 0]) | (int(C[j, e, 1]) << 64)
            h = int(H[j, e, 0]) | (int(H[j, e, 1]) << 64)
            assert dash_hash(c) == h
    assert np.array_equal(L.colors()[1], L.blocks[1][:, 0])
