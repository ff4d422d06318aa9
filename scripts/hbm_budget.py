#!/usr/bin/env python
"""HBM accounting of one evaluator group: tables vs activations/scratch vs garbler cache (MiniONN DASH)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dash_amd.garbling import GarbledCircuit  # noqa: E402
from dash_amd.ir.quant import QuantizationMethod  # noqa: E402
from dash_amd.models import BENCH_CONFIGS, build_circuit  # noqa: E402
from dash_amd.native import native  # noqa: E402
from dash_amd.runtime import HipEvaluator  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 6
cfg = BENCH_CONFIGS["MODEL_F_MINIONN_POOL_REPL/DASH"]
c = build_circuit("MODEL_F_MINIONN_POOL_REPL", QuantizationMethod(cfg["q_method"]), cfg["q_parameter"], seed=0)
torch.cuda.init()
f0, tot = torch.cuda.mem_get_info(0)
ev = None
for b in range(B):
    gc = GarbledCircuit(c, cfg["crt"], cfg["mrs"], seed=bytes([b]) * 16, device=0)
    if ev is None:
        ev = HipEvaluator(template=gc.model, batch=B, device=0)
        f1, _ = torch.cuda.mem_get_info(0)
    ev.load(b, gc.model)
    gc = None
f2, _ = torch.cuda.mem_get_info(0)
cache = native().gpu_table_cache_bytes()
native().gpu_table_cache_trim()
f3, _ = torch.cuda.mem_get_info(0)
print(json.dumps({"B": B, "evaluator_device_bytes_GB": ev.device_bytes() / 1e9, "tables_GB": ev.table_bytes() / 1e9,
                  "after_ctor_used_GB": (f0 - f1) / 1e9, "after_loads_used_GB": (f0 - f2) / 1e9,
                  "garbler_cache_GB": cache / 1e9, "after_trim_used_GB": (f0 - f3) / 1e9, "total_GB": tot / 1e9}))
