"""Trusted-garbler process split (reference SGX flow, C40/C41), CPU evaluator."""
import numpy as np
import pytest

from dash_amd.garbling import GarbledCircuit
from dash_amd.models import build_circuit, quantized_inputs
from dash_amd.sgx import GarblerEnclave


def test_enclave_ann_infer_cpu():
    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 4)
    with GarblerEnclave(c, 7, 100.0, batch=2, backend="cpu") as enc:
        out = enc.ann_infer(xs)
        assert enc.last_stats["online_bytes"] > 0
    ref = GarbledCircuit(c, 7, 100.0, garble_me=False)
    np.testing.assert_array_equal(out, np.stack([ref.plain_q_eval(x) for x in xs]))

