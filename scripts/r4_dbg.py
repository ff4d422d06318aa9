"""Debug: GPU-garble one circuit with per-layer tracing (DASH_GG_TRACE=1, DASH_GG_SYNC=1) and compare to the host."""
import sys  # noqa
import time

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import dash_amd as d
from dash_amd.garbling import GarbledCircuit
from dash_amd.ir.quant import QuantizationMethod as Q
from dash_amd.models import build_circuit

name = sys.argv[1]
rng = np.random.default_rng(11)
if name == "dense":
    c, k = d.Circuit([d.Dense(rng.integers(-4, 5, (70, 300)), rng.integers(-6, 6, 70), q_const=1.0)]), 8
elif name == "dense_relu":
    c, k = d.Circuit([d.Dense(rng.integers(-4, 5, (70, 300)), rng.integers(-6, 6, 70), q_const=1.0), d.Relu((70,))]), 8
else:
    c, k = build_circuit("MODEL_B_POOL_REPL", Q.ScaleQuant, 3, seed=1), 8
print("layers", [l.kind for l in c.layers], flush=True)
t = time.time()
gpu = GarbledCircuit(c, k, 100.0, seed=bytes(range(16)), device=0)
print("gpu garbled", round(time.time() - t, 3), flush=True)
cpu = GarbledCircuit(c, k, 100.0, seed=bytes(range(16)))
print("identical", gpu.model.serialize() == cpu.model.serialize(), flush=True)
