#!/usr/bin/env python
"""Per-layer micro-benchmarks: CPU (host oracle) vs GPU (HIP evaluator).

Mirrors benchmarks/micro_benchmarks/non_sgx/main.cpp of the reference
(sweeps :577-685; PyTorch-like init :20-55; inputs uniform in [0, 255]
:58-65; GPU memory via the device's free-memory delta :67-75) and writes the
same CSV columns:

  dense / conv2d:      type, dimensions, crt_base_size, run, runtime, gpu_mem_usage, q_acc
  approx_relu / sign:  ..., q_acc, relu_acc|sign_acc
  rescaling:           type, dimensions, crt_base_size, run, runtime, gpu_mem_usage, use_legacy_scaling

Timed region: evaluation only (cpu_evaluate / HIP run), like the reference.
GPU runs additionally take `--batch` garbled circuits per launch and report
per-circuit time (runtime / batch) so batching gains are visible.

Usage:
  python benchmarks/micro.py --layers dense,conv2d,approx_relu,sign,rescaling --targets cpu,gpu --runs 3
  python benchmarks/micro.py --layers dense --targets gpu,gpu_valu --batch 16   # MFMA vs VALU dense
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
from dash_amd.ir.layers import Conv2d, Dense, Relu, Rescale, Sign  # noqa: E402
from dash_amd.ir.quant import QuantizationMethod  # noqa: E402
from dash_amd.utils.bench_util import csv_path, date_string  # noqa: E402

Q_CONST = 0.0001
DENSE_DIMS = [128, 256, 512, 1024, 2048]
CONV_DIMS = [(64, 64, 3), (128, 128, 3), (256, 256, 3)]
ACT_DIMS = [128, 256, 512, 1024, 2048, 4096, 8192, 16384]


def init_wb(shape, in_features, rng):
    bound = np.sqrt(1.0 / in_features)
    return rng.uniform(-bound, bound, size=shape).astype(np.float32)


def init_inputs(n, rng):
    return rng.integers(0, 256, size=n).astype(np.int64)


def gpu_mem_used() -> float:
    try:
        import torch

        free, total = torch.cuda.mem_get_info()
        return float(total - free)
    except Exception:
        return -1.0


def run_cpu(circuit, k, mrs, x):
    gc = GarbledCircuit(circuit, k, mrs)
    g = gc.garble_inputs(x)
    t = time.perf_counter()
    out = gc.cpu_evaluate(g)
    ms = 1000 * (time.perf_counter() - t)
    gc.decode_outputs(out)
    return ms, -1.0


def run_gpu(circuit, k, mrs, x, batch, mfma=True, reps=10):
    """Per-GC evaluation time: one untimed run (lazy setup), then the mean of `reps` runs (the same
    evaluation repeated on the staged inputs; outputs are decoded and checked after the last)."""
    import torch

    from dash_amd.runtime import HipEvaluator

    m1 = gpu_mem_used()
    gcs = [GarbledCircuit(circuit, k, mrs) for _ in range(batch)]
    ev = HipEvaluator([g.model for g in gcs], mfma=mfma)
    for b, g in enumerate(gcs):
        ev.encode_compressed_into(b, g, x)
    ev.upload_inputs_compressed()
    torch.cuda.synchronize()
    m2 = gpu_mem_used()
    ev.run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        ev.run()
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t) / reps
    ev.fetch_outputs()
    for b, g in enumerate(gcs):
        np.testing.assert_array_equal(ev.decode(b, g), g.plain_q_eval(x))
    del ev
    return ms / batch, (m2 - m1) / batch


def bench(layer, targets, runs, batch, rng, out_dir, date):
    extra = {"approx_relu": "relu_acc", "sign": "sign_acc"}.get(layer)
    cols = "type, dimensions, crt_base_size, run, runtime, gpu_mem_usage, " + (
        "use_legacy_scaling" if layer == "rescaling" else "q_acc" + (f", {extra}" if extra else ""))
    path = csv_path(out_dir, date, layer)
    with open(path, "w") as f:
        f.write(cols + "\n")
        if layer == "dense":
            cases = [(d, None) for d in DENSE_DIMS]
        elif layer == "conv2d":
            cases = [(d, None) for d in CONV_DIMS]
        elif layer in ("approx_relu", "sign"):
            cases = [(d, acc) for d in ACT_DIMS for acc in (99.0, 100.0)]
        else:
            cases = [(d, legacy) for d in ACT_DIMS for legacy in (True, False)]
        for dim, opt in cases:
            for target in targets:
                for run in range(runs):
                    if layer == "dense":
                        w = init_wb((dim, dim), dim, rng)
                        b = init_wb((dim,), dim, rng)
                        x = init_inputs(dim, rng)
                        c = Circuit([Dense(w, b, -1, QuantizationMethod.SimpleQuant, Q_CONST)])
                        q_acc = c.compute_q_acc(x.astype(np.float32), x, Q_CONST)
                        k, mrs = c.infer_crt_base_size([x]), None
                    elif layer == "conv2d":
                        W, H, C = dim
                        F, fs, st = 16, 4, 2
                        w = init_wb((F, C, fs, fs), C * fs * fs, rng)
                        b = init_wb((F,), C * fs * fs, rng)
                        x = init_inputs(W * H * C, rng)
                        c = Circuit([Conv2d(w, b, W, H, C, F, fs, fs, st, st, -1, QuantizationMethod.SimpleQuant,
                                            Q_CONST)])
                        q_acc = c.compute_q_acc(x.astype(np.float32), x, Q_CONST)
                        k, mrs = c.infer_crt_base_size([x]), None
                    elif layer in ("approx_relu", "sign"):
                        x = init_inputs(dim, rng)
                        c = Circuit([Relu((dim,)) if layer == "approx_relu" else Sign((dim,))])
                        q_acc = c.compute_q_acc(x.astype(np.float32), x, Q_CONST)
                        k, mrs = 8, opt
                    else:
                        x = init_inputs(dim, rng)
                        c = Circuit([Rescale(1, (dim,)) if opt else Rescale([2], (dim,))])
                        q_acc = None
                        k, mrs = 8, 100.0
                    if target == "cpu":
                        ms, mem = run_cpu(c, k, mrs, x)
                    else:  # gpu: MFMA kernels where they exist; gpu_valu: the VALU kernels (A/B)
                        ms, mem = run_gpu(c, k, mrs, x, batch, mfma=target != "gpu_valu")
                    dims_s = "x".join(map(str, dim)) if isinstance(dim, tuple) else str(dim)
                    row = [target.upper(), dims_s, str(k), str(run), f"{ms:f}", f"{mem:f}"]
                    if layer == "rescaling":
                        row.append(str(int(opt)))
                    else:
                        row.append(f"{q_acc:f}")
                        if extra:
                            row.append(f"{opt:f}")
                    f.write(", ".join(row) + "\n")
                    f.flush()
                    print(f"{layer:12s} {target} dim={dims_s:>12s} k={k} run={run} {ms:10.3f} ms", flush=True)
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="dense,conv2d,approx_relu,sign,rescaling")
    ap.add_argument("--targets", default="cpu,gpu")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1, help="GCs per GPU launch")
    ap.add_argument("--out", default="data")
    ap.add_argument("--max-dim", type=int, default=0, help="skip sweep points above this size (quick runs)")
    args = ap.parse_args()
    global DENSE_DIMS, ACT_DIMS, CONV_DIMS
    if args.max_dim:
        DENSE_DIMS = [d for d in DENSE_DIMS if d <= args.max_dim]
        ACT_DIMS = [d for d in ACT_DIMS if d <= args.max_dim]
        CONV_DIMS = [d for d in CONV_DIMS if d[0] <= args.max_dim]
    targets = args.targets.split(",")
    if any(t.startswith("gpu") for t in targets):
        from dash_amd.runtime import hip_available

        if not hip_available():
            print("no GPU visible: running cpu only", file=sys.stderr)
            targets = [t for t in targets if not t.startswith("gpu")]
    rng = np.random.default_rng(42)
    date = date_string()
    for layer in args.layers.split(","):
        print("wrote", bench(layer, targets, args.runs, args.batch, rng, args.out, date))


if __name__ == "__main__":
    main()
