#!/usr/bin/env python
"""Offline-phase timing: garble one GC on the host vs with the GPU sign-gadget garbler.

  python scripts/garble_bench.py --model MODEL_F_MINIONN_POOL_REPL --reps 2
Prints one JSON line per mode with seconds per GC and per-layer milliseconds, and checks
that the device-garbled model is byte-identical to the host-garbled one.
"""
import argparse
import json
import os
import sys
import time

# DASH_PKG_ROOT: import dash_amd from another tree (A/B builds, scripts/ab_variant.sh)
sys.path.insert(0, os.environ.get("DASH_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dash_amd.garbling import GarbledCircuit  # noqa: E402
from dash_amd.ir.quant import QuantizationMethod as Q  # noqa: E402
from dash_amd.models import build_circuit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="MODEL_F_MINIONN_POOL_REPL")
    ap.add_argument("--k", type=int, default=7)
    ap.add_argument("--l", type=int, default=5)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--gpu-only", action="store_true", help="skip the host garbler (profiling)")
    ap.add_argument("--rescale", default="mrs", help="rescale construction (mrs | legacy)")
    ap.add_argument("--relu", default="joint", help="relu construction (joint | approx | mrs)")
    ap.add_argument("--sink", type=int, default=0,
                    help="N > 0: garble N GCs straight into the slots of a 2-slot HipEvaluator (zero-copy load), "
                         "timing garble + load per GC like the serving engine")
    args = ap.parse_args()
    c = build_circuit(args.model, Q.ScaleQuant, args.l, seed=0)
    seed = bytes(range(16))
    if args.sink:
        from dash_amd.runtime import HipEvaluator

        kw = dict(rescale=args.rescale, relu=args.relu)
        t0 = GarbledCircuit(c, args.k, 100.0, seed=seed, device=args.device, **kw)
        ev = HipEvaluator(template=t0.model, batch=2, device=args.device)
        del t0
        ts = []
        for r in range(args.sink):
            t = time.perf_counter()
            gc = GarbledCircuit(c, args.k, 100.0, seed=bytes([r % 256]) * 16, device=args.device,
                                sink=ev.sink(r % 2), **kw)
            tg = time.perf_counter() - t
            ev.load(r % 2, gc.model)
            ts.append((tg, time.perf_counter() - t))
        steady = ts[1:] or ts
        print(json.dumps({"mode": "gpu_sink", "model": args.model, "gcs": args.sink,
                          "garble_ms_per_gc": round(1000 * sum(a for a, _ in steady) / len(steady), 2),
                          "garble_load_ms_per_gc": round(1000 * sum(b for _, b in steady) / len(steady), 2),
                          "layer_ms": [round(x, 1) for x in gc.garbling_layer_ms()]}), flush=True)
        return
    blobs = {}
    modes = (("gpu", args.device),) if args.gpu_only else (("gpu", args.device), ("cpu", None))
    for mode, dev in modes:
        times = []
        gc = None
        for _ in range(args.reps):
            t = time.perf_counter()
            gc = GarbledCircuit(c, args.k, 100.0, seed=seed, device=dev, rescale=args.rescale, relu=args.relu)
            times.append(time.perf_counter() - t)
        blobs[mode] = gc.model.serialize()
        print(json.dumps({"mode": mode, "model": args.model, "s_per_gc": round(min(times), 3),
                          "ms_per_gc_min": round(1000 * min(times), 2),
                          "ms_per_gc_median": round(1000 * sorted(times)[len(times) // 2], 2),
                          "layer_ms": [round(x, 1) for x in gc.garbling_layer_ms()]}), flush=True)
    if not args.gpu_only:
        print(json.dumps({"identical": blobs["gpu"] == blobs["cpu"]}), flush=True)
        assert blobs["gpu"] == blobs["cpu"]


if __name__ == "__main__":
    main()
