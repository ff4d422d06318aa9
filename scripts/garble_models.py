#!/usr/bin/env python
"""Per-model GPU garbling time (offline phase): seconds per GC (min over reps after one warm-up) and the per-layer
wall milliseconds of the last GC, for the zoo configurations of the round-4 GPU garbler coverage."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dash_amd.garbling import GarbledCircuit  # noqa: E402
from dash_amd.models import BENCH_CONFIGS, build_circuit, quantized_inputs  # noqa: E402
from dash_amd.ir.quant import QuantizationMethod as Q  # noqa: E402

CASES = [("VGG16", "MODEL_F_MINIONN_POOL_REPL/DASH"), ("RESNET18", "MODEL_F_MINIONN_POOL_REPL/DASH"),
         ("MODEL_F_MINIONN_POOL_REPL", "MODEL_F_MINIONN_POOL_REPL/REDASH_OPT"),
         ("MODEL_F_MINIONN_POOL_REPL", "MODEL_F_MINIONN_POOL_REPL/REDASH_CPM"),
         ("MODEL_F_MINIONN_POOL_REPL", "MODEL_F_MINIONN_POOL_REPL/DASH"), ("LENET5", "MODEL_F_MINIONN_POOL_REPL/DASH")]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
for model, cfgname in CASES:
    cfg = BENCH_CONFIGS[cfgname]
    qm = Q(cfg["q_method"])
    c = build_circuit(model, qm, cfg["q_parameter"], seed=0)
    c.calibrate(quantized_inputs(model, 16, qm, cfg["q_parameter"], seed=0))
    kw = dict(rescale="mrs", relu="joint") if cfgname.endswith("/DASH") else {}
    ts = []
    for r in range(reps + 1):
        t = time.perf_counter()
        gc = GarbledCircuit(c, cfg["crt"], cfg["mrs"], seed=bytes([r]) * 16, device=0, **kw)
        ts.append(time.perf_counter() - t)
        gc.model = None
    names = [f"{i}:{l.name}" for i, l in enumerate(c.layers)]
    ms = gc.garbling_layer_ms()
    top = sorted(zip(ms, names), reverse=True)[:6]
    print(json.dumps({"model": model, "scheme": cfgname.split("/")[1], "s_per_gc": round(min(ts[1:]), 4),
                      "first_s": round(ts[0], 3), "layers": len(names),
                      "top_layers_ms": [[n, round(v, 2)] for v, n in top]}), flush=True)
