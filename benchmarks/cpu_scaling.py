#!/usr/bin/env python
"""Host-evaluator strong scaling over worker threads (1..16).

Mirrors benchmarks/micro_benchmarks/non_sgx_scaling/main.cpp (thread sweep
:70-311; rescale with crt_base[0] = 2^l :266-311). CSV columns:
  type, nr_threads, crt_base_size, dimensions, run, runtime, q_acc
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dash_amd.garbling import GarbledCircuit  # noqa: E402
from dash_amd.ir.circuit import Circuit  # noqa: E402
from dash_amd.ir.layers import Conv2d, Dense, Relu, Rescale  # noqa: E402
from dash_amd.ir.quant import QuantizationMethod  # noqa: E402
from dash_amd.utils.bench_util import csv_path, date_string  # noqa: E402

Q_CONST = 0.0001


def make(layer, dim, rng):
    x = rng.integers(0, 256, size=dim if layer != "conv2d" else dim * dim * 3).astype(np.int64)
    if layer == "dense":
        b = np.sqrt(1.0 / dim)
        c = Circuit([Dense(rng.uniform(-b, b, (dim, dim)), rng.uniform(-b, b, dim), -1,
                           QuantizationMethod.SimpleQuant, Q_CONST)])
        return c, x, c.infer_crt_base_size([x]), None
    if layer == "conv2d":
        b = np.sqrt(1.0 / (3 * 16))
        c = Circuit([Conv2d(rng.uniform(-b, b, (16, 3, 4, 4)), rng.uniform(-b, b, 16), dim, dim, 3, 16, 4, 4, 2, 2,
                            -1, QuantizationMethod.SimpleQuant, Q_CONST)])
        return c, x, c.infer_crt_base_size([x]), None
    if layer == "approx_relu":
        return Circuit([Relu((dim,))]), x, 8, 100.0
    # rescaling by 2^l with crt_base[0] = 2^l (ReDash factor), l = 1
    return Circuit([Rescale([2], (dim,))]), x, 8, 100.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="dense,conv2d,approx_relu,rescaling")
    ap.add_argument("--dims", default="")
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--out", default="data")
    args = ap.parse_args()
    default_dims = {"dense": [1024], "conv2d": [128], "approx_relu": [16384], "rescaling": [16384]}
    date = date_string()
    rng = np.random.default_rng(42)
    for layer in args.layers.split(","):
        dims = [int(d) for d in args.dims.split(",")] if args.dims else default_dims[layer]
        path = csv_path(args.out, date, f"{layer}_scaling")
        with open(path, "w") as f:
            f.write("type, nr_threads, crt_base_size, dimensions, run, runtime, q_acc\n")
            for dim in dims:
                c, x, k, mrs = make(layer, dim, rng)
                q_acc = c.compute_q_acc(x.astype(np.float32), x, Q_CONST) if layer in ("dense", "conv2d") else -1.0
                gc = GarbledCircuit(c, k, mrs)
                g = gc.garble_inputs(x)
                ref = None
                for nt in [int(t) for t in args.threads.split(",")]:
                    for run in range(args.runs):
                        t = time.perf_counter()
                        out = gc.cpu_evaluate(g, nt)
                        ms = 1000 * (time.perf_counter() - t)
                        y = gc.decode_outputs(out)
                        if ref is None:
                            ref = y
                        assert np.array_equal(ref, y), "thread count changed the result"
                        f.write(f"CPU, {nt}, {k}, {dim}, {run}, {ms:f}, {q_acc:f}\n")
                        print(f"{layer:12s} dim={dim} threads={nt:2d} run={run} {ms:9.2f} ms", flush=True)
        print("wrote", path)


if __name__ == "__main__":
    main()
