"""Whole models on the GPU: full VGG-16 / ResNet-18 / MiniONN circuits garbled by the GPU garbler and
evaluated by the HIP evaluator at batch 1, against the plaintext quantized evaluation; and the streamed-table
evaluator mode (tables in pinned host memory, three rotating HBM layer windows) against the same oracle."""
import numpy as np
import pytest

from dash_amd.garbling import GarbledCircuit
from dash_amd.ir.quant import QuantizationMethod as Q
from dash_amd.models import build_circuit, quantized_inputs

pytestmark = pytest.mark.gpu


def _run(ev, gcs, xs, runs=1):
    outs = None
    for _ in range(runs):
        for b, (gc, x) in enumerate(zip(gcs, xs)):
            ev.encode_compressed_into(b, gc, x)
        ev.upload_inputs_compressed()
        ev.run()
        ev.fetch_outputs()
        outs = [ev.decode(b, gc) for b, gc in enumerate(gcs)]
    return outs


@pytest.mark.parametrize("name", ["VGG16", "RESNET18", "MODEL_F_MINIONN_POOL_REPL"])
def test_full_model_batch1(name):
    """The whole circuit (every conv, rescale, ReLU, pool, residual add, dense) at batch 1 with the flagship
    constructions, GPU-garbled, decoded outputs == plain_q_eval."""
    from dash_amd.runtime import HipEvaluator

    c = build_circuit(name, Q.ScaleQuant, 5, seed=0)
    x = quantized_inputs(name, 1, Q.ScaleQuant, 5, seed=11)[0]
    gc = GarbledCircuit(c, 7, 100.0, seed=bytes([3]) * 16, device=0, rescale="mrs", relu="joint")
    ev = HipEvaluator(template=gc.model, batch=1, device=0)
    ev.load(0, gc.model)
    (y,) = _run(ev, [gc], [x])
    np.testing.assert_array_equal(y, gc.plain_q_eval(x))


@pytest.mark.parametrize("rescale,relu", [("mrs", "joint"), ("legacy", "approx")])
def test_streamed_tables(rescale, relu):
    """stream_tables=True: the same GCs decode to the plaintext outputs, over two runs (the second run's
    layer-0..2 uploads wait for the first run's end), and the device holds only the three layer windows."""
    from dash_amd.runtime import HipEvaluator

    name = "MODEL_F_MINIONN_POOL_REPL"
    c = build_circuit(name, Q.ScaleQuant, 5, seed=0)
    xs = quantized_inputs(name, 2, Q.ScaleQuant, 5, seed=5)
    gcs = [GarbledCircuit(c, 7, 100.0, seed=bytes([b + 1]) * 16, device=0, rescale=rescale, relu=relu)
           for b in range(2)]
    ev = HipEvaluator(template=gcs[0].model, batch=2, device=0, stream_tables=True)
    assert ev.streams_tables
    for b, gc in enumerate(gcs):
        ev.load(b, gc.model)
    outs = _run(ev, gcs, xs, runs=2)
    for gc, x, y in zip(gcs, xs, outs):
        np.testing.assert_array_equal(y, gc.plain_q_eval(x))
    assert ev.table_bytes() > 0  # counted as pinned host bytes
