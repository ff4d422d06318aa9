import time, sys, os
sys.path.insert(0, os.getcwd())
from dash_amd.garbling import GarbledCircuit
from dash_amd.ir.quant import QuantizationMethod as Q
from dash_amd.models import build_circuit
c = build_circuit("MODEL_F_MINIONN_POOL_REPL", Q.ScaleQuant, 5, seed=0)
for i in range(4):
    t = time.perf_counter(); g = GarbledCircuit(c, 7, 100.0, seed=bytes([i]) * 16, device=0, rescale="mrs"); dt = time.perf_counter() - t
    print("garble s", round(dt, 4), "layers ms", [round(x, 1) for x in g.garbling_layer_ms()], "sum", round(sum(g.garbling_layer_ms()), 1))
    t = time.perf_counter(); g.model = None; g = None; print("free s", round(time.perf_counter() - t, 4))
