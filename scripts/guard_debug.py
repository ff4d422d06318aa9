"""Native range guard vs the numpy model on the bench's inputs (A/B knobs DASH_GUARD_I24 / DASH_GUARD_GRAPH)."""
import sys
import time

import numpy as np

from dash_amd.garbling.guard import RangeGuard
from dash_amd.ir.bases import crt_modulus, first_primes
from dash_amd.ir.quant import QuantizationMethod
from dash_amd.models import BENCH_CONFIGS, build_circuit, quantized_inputs

cfg = BENCH_CONFIGS["MODEL_F_MINIONN_POOL_REPL/DASH"]
qm = QuantizationMethod(cfg["q_method"])
c = build_circuit("MODEL_F_MINIONN_POOL_REPL", qm, cfg["q_parameter"], seed=0)
M = crt_modulus(first_primes(cfg["crt"]))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 160
xs = quantized_inputs("MODEL_F_MINIONN_POOL_REPL", B, qm, cfg["q_parameter"], seed=1000)
g = RangeGuard(c, M, mrs=True, device=0)
ref = [i for i, x in enumerate(xs) if g.violations_np(x)]
for rep in range(3):
    t = time.perf_counter()
    p = g.submit(xs)
    got = p.bad_indices()
    dt = time.perf_counter() - t
    print(f"rep {rep}: native {len(got)} flagged {got[:10]} numpy {ref[:10]} ({1000 * dt:.2f} ms)", flush=True)
spec = g.native_spec()
print("buf_elems", spec["buf_elems"], "ctx_buf", spec["ctx_buf"])
