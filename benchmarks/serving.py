#!/usr/bin/env python
"""End-to-end serving throughput: offline garbling pipelined against online
evaluation (dash_amd.serving.InferenceService), i.e. what a production
deployment sustains when every inference needs a fresh GC — the number the
reference never reports (its benchmarks exclude garbling).

Prints one JSON line: steady-state inferences/s (wall clock, garbling
included), batch latency percentiles, retries/integrity failures, and the
online-only rate for comparison. ``--faults R`` corrupts a fraction R of the
output messages to exercise discard-and-re-garble recovery under load.
"""
from __future__ import annotations

import argparse
import json
import random
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="MODEL_F_MINIONN_POOL_REPL")
    ap.add_argument("--config", default="DASH")
    ap.add_argument("--backend", default="hip", choices=["hip", "cpu"])
    ap.add_argument("--slots", type=int, default=4, help="GC slots per group (online batch)")
    ap.add_argument("--groups", type=int, default=3, help="evaluator groups in the pool")
    ap.add_argument("--requests", type=int, default=8, help="online batches to serve")
    ap.add_argument("--faults", type=float, default=0.0)
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--rescale", default="mrs", choices=["mrs", "legacy"])
    ap.add_argument("--relu", default="joint", choices=["mrs", "approx", "joint"])
    ap.add_argument("--encoding", default="auto", choices=["auto", "hardened", "reference"],
                    help="offline-message encoding (reference: wire-compatible, R_p recoverable; docs/SECURITY.md)")
    ap.add_argument("--garble-workers", type=int, default=None,
                    help="refill workers (GPU garbler: concurrent garblings, one garbling context each, "
                         "DASH_GG_CONTEXTS caps the contexts per device)")
    args = ap.parse_args()

    from dash_amd.ir.quant import QuantizationMethod
    from dash_amd.models import BENCH_CONFIGS, build_circuit, canonical, quantized_inputs
    from dash_amd.serving import InferenceService

    model = canonical(args.model)
    cfg = BENCH_CONFIGS.get(f"{model}/{args.config}") or dict(q_method=QuantizationMethod.ScaleQuant, q_parameter=3,
                                                              crt=8, mrs=100.0)
    qm, qp = QuantizationMethod(cfg["q_method"]), cfg["q_parameter"]
    circuit = build_circuit(model, qm, qp, seed=0)
    from dash_amd.ir.bases import crt_modulus as _cm, first_primes as _fp

    # range calibration arms the mixed-radix rescale's wrap-band guard (GarbledCircuit refuses a tracked violation)
    circuit.calibrate(quantized_inputs(model, 32, qm, qp, seed=0),
                      _cm(cfg["crt"] if isinstance(cfg["crt"], list) else _fp(cfg["crt"])))
    xs = quantized_inputs(model, args.slots * args.requests, qm, qp, seed=11)
    rng = random.Random(5)
    hook = (lambda i, a: a == 0 and rng.random() < args.faults) if args.faults > 0 else None
    t0 = time.perf_counter()
    svc = InferenceService(circuit, cfg["crt"], cfg["mrs"], backend=args.backend, slots_per_group=args.slots,
                           groups=args.groups, fault_hook=hook, step_timeout_s=args.timeout, rescale=args.rescale,
                           relu=args.relu, garble_workers=args.garble_workers,
                           hardened={"auto": None, "hardened": True, "reference": False}[args.encoding])
    fill_s = time.perf_counter() - t0
    svc.stats.t_start = time.perf_counter()
    from dash_amd.ir.bases import crt_modulus, first_primes

    crt = cfg["crt"] if isinstance(cfg["crt"], list) else first_primes(cfg["crt"])
    M = crt_modulus(crt)
    ok = True
    for r in range(args.requests):
        batch = xs[r * args.slots:(r + 1) * args.slots]
        y = svc.infer(batch)
        if r == 0:  # decoded logits == plaintext quantized evaluation
            ok = all((y[i] == circuit.plain_q_eval(x, track=False, crt_modulus=M)).all() for i, x in enumerate(batch))
    st = svc.stats.as_dict()
    online_ms = sum(svc.stats.latencies_ms)
    workers = svc.garble_workers
    svc.close()
    print(json.dumps({
        "metric": f"served garbled inferences/s incl. garbling ({model})", "backend": args.backend,
        "rescale": args.rescale, "relu": args.relu,
        "slots": args.slots, "groups": args.groups, "garble_workers": workers, "pool_fill_s": round(fill_s, 2),
        "online_only_inf_per_s": round(st["inferences"] / (online_ms / 1000.0), 2) if online_ms else None,
        **st, "ok": ok}), flush=True)


if __name__ == "__main__":
    main()
