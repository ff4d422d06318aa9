"""Training pipeline -> Circuit -> ONNX -> garbled inference (C48 end to end)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from dash_amd.garbling import GarbledCircuit  # noqa: E402
from dash_amd.ir.onnx import load_onnx_model, save_onnx_model  # noqa: E402
from dash_amd.ir.quant import QuantizationMethod as Q, quantize_input  # noqa: E402
from dash_amd.models.train import evaluate, to_circuit, train  # noqa: E402


def test_train_export_garble(tmp_path):
    model, (xte, yte) = train("MODEL_A", epochs=3, n_synthetic=4096, fake_quant=0.01, device="cpu", log=lambda *_: None)
    acc = evaluate(model, xte, yte)
    assert acc > 0.3  # learnable synthetic task, well above chance
    model.fq.c = 0.0  # compare the float networks
    c = to_circuit(model, "MODEL_A", Q.ScaleQuant, 4)
    x = xte[0].reshape(-1)
    with torch.no_grad():
        ref = model(torch.from_numpy(xte[:1])).numpy()[0]
    np.testing.assert_allclose(c.plain_eval(x), ref, rtol=1e-4, atol=1e-4)
    p = tmp_path / "a.onnx"
    save_onnx_model(p, c, producer="pytorch")
    c2 = load_onnx_model(p, Q.ScaleQuant, 4)
    xq = quantize_input(x, Q.ScaleQuant, 4, 0.0)
    k = c2.infer_crt_base_size([xq])
    gc = GarbledCircuit(c2, max(k, 7), 100.0)
    out = gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(xq)))
    np.testing.assert_array_equal(out, gc.plain_q_eval(xq))
