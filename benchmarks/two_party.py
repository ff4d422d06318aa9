#!/usr/bin/env python
"""Two-party and trusted-garbler deployments at speed: offline shipping, online round, served inferences/s.

The reference's only cross-party path is its SGX split: the garbler runs in an enclave and the untrusted host
evaluates on the GPU behind ocalls (sgx/App/App.cpp:140-365); its SGX model benchmark times the online round
over MODEL_A..F (benchmarks/model_benchmarks/sgx/Enclave/Enclave.cpp:171-183, App/App.cpp:415-482). Here both
splits run as separate processes:

* ``tcp``: an EvaluatorServer process (HIP or host evaluator) and this process as the GarblerClient, over a
  localhost TCP channel (dash_amd.net);
* ``enclave``: GarblerEnclave, the attested trusted-garbler process, with the evaluator server in this process.

The garbler garbles on its own device (``--garble-device``, default 0; -1 = host CPU as in the reference's
enclave) and pipelines the offline phase: GC b + 1 is garbled while GC b is serialized onto the wire and loaded
by the evaluator. Per (model config, split) one JSON line:

  offline_gb_per_gc, offline_s_per_gc, offline_gbps (offline bytes / offline wall time), garble_s_per_gc,
  online_round_ms (p50 over rounds: encode -> send -> evaluate -> receive -> decode for `batch` inferences),
  online_bytes_per_inference, served_inf_per_s (fresh GC per inference, offline + online wall time),
  verified (decoded == plaintext).

The offline message travels over the TCP channel (``--transport tcp``, any host), through a ring of shared-memory
segments of this host (``shm``, the same-host split of the reference's enclave: the channel then carries only the
segment names and the evaluator's acknowledgements), or never leaves device memory (``ipc``: the garbler's GPU
writes each GC's tables straight into the HIP evaluator's slots through their IPC handles, same device or a peer
over xGMI; the channel carries the skeleton of each model). The circuit is range-calibrated first, so the default
("auto") constructions are the headline's (mixed-radix rescale, joint ReLU) where the ranges allow; the record
names the resolved ones.

On a one-GPU lease both parties share device 0: the numbers are a performance rehearsal of the split, not a
trust-valid deployment (the record says so). The ``--splits`` list may name either or both.

    python benchmarks/two_party.py [--models MODEL_A/SIMPLE,...] [--splits tcp,enclave] [--backend hip|cpu]
                                   [--garble-device 0|-1] [--batch B] [--rounds R]
"""
from __future__ import annotations

import argparse
import itertools
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from models import CONFIGS, config_name, load_circuit, quantize_images  # noqa: E402

from dash_amd.models.zoo import synthetic_inputs  # noqa: E402

DEFAULT_MODELS = ["MODEL_A/SIMPLE", "MODEL_B_POOL_REPL/SIMPLE", "MODEL_C/SIMPLE", "MODEL_D_POOL_REPL/SIMPLE",
                  "MODEL_F_GNNP_POOL_REPL/DASH", "MODEL_F_MINIONN_POOL_REPL/DASH",
                  "MODEL_F_MINIONN_POOL_REPL/OPT"]


def _serve(port_q, backend, device):
    from dash_amd.net import listen
    from dash_amd.net.protocol import serve_once

    s = listen("127.0.0.1", 0)
    port_q.put(s.getsockname()[1])
    serve_once(s, backend=backend, device=device)
    s.close()


def _gc_args(cfg):
    if cfg.crt_base:
        return cfg.crt_base, cfg.mrs_base, max(cfg.crt_base)
    return cfg.target_crt_base_size, cfg.relu_accs[0], 0


def _plain(circuit, crt, mrs, x):
    from dash_amd.garbling import GarbledCircuit

    return GarbledCircuit(circuit, crt, mrs, seed=bytes(16), garble_me=False).plain_q_eval(x)


def run_tcp(circuit, cfg, xs, args) -> dict:
    from dash_amd.net import GarblerClient

    crt, mrs, mm = _gc_args(cfg)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_serve, args=(q, args.backend, args.device), daemon=True)
    p.start()
    port = q.get(timeout=300)
    dev = None if args.garble_device < 0 else args.garble_device
    rounds, online = [], []
    ok = True
    try:
        with GarblerClient("127.0.0.1", port, circuit, crt, mrs, batch=args.batch, max_modulus=mm,
                           seed=os.urandom(16), device=dev, pipeline=not args.no_pipeline,
                           transport=args._transport) as cl:
            for r in range(args.rounds + 1):  # round 0 warms up (evaluator build, graph capture)
                batch = xs[(r % 4) * args.batch:(r % 4 + 1) * args.batch]
                t0 = time.perf_counter()
                cl.offline()
                t1 = time.perf_counter()
                outs = cl.infer(batch)
                t2 = time.perf_counter()
                print(f"[two_party] round {r}: offline {t1 - t0:.3f} s, online {1000 * (t2 - t1):.1f} ms",
                      file=sys.stderr, flush=True)
                if r == 0:
                    st0 = dict(cl.stats, online_s=list(cl.stats["online_s"]))
                    ok = all(np.array_equal(y, _plain(circuit, crt, mrs, x)) for x, y in zip(batch, outs))
                    continue
                rounds.append((t1 - t0, t2 - t1))
                online.append(1000.0 * (t2 - t1))
            st = cl.stats
    finally:
        p.join(timeout=120)
    n_gc = args.rounds * args.batch
    off_b = st["offline_bytes"] - st0["offline_bytes"]
    off_s = sum(a for a, _ in rounds)
    tot_s = sum(a + b for a, b in rounds)
    on_b = st["online_bytes"] - st0["online_bytes"]
    return dict(offline_gb_per_gc=off_b / n_gc / 1e9, offline_s_per_gc=off_s / n_gc,
                offline_gbps=off_b / max(off_s, 1e-9) / 1e9,
                garble_s_per_gc=(st["garble_s"] - st0["garble_s"]) / n_gc,
                serialize_s_per_gc=(st["serialize_s"] - st0["serialize_s"]) / n_gc,
                online_round_ms=float(np.median(online)), online_bytes_per_inference=on_b / n_gc,
                served_inf_per_s=n_gc / tot_s, verified=bool(ok), encoding=st.get("encoding"))


def run_enclave(circuit, cfg, xs, args) -> dict:
    import tempfile

    from dash_amd.sgx import GarblerEnclave
    from dash_amd.sgx import attest as at

    crt, mrs, mm = _gc_args(cfg)
    dev = None if args.garble_device < 0 else args.garble_device
    with tempfile.TemporaryDirectory() as td:
        key = os.path.join(td, "platform.key")
        at.platform_key(key)
        with GarblerEnclave(circuit, crt, mrs, max_modulus=mm, batch=args.batch, backend=args.backend,
                            device=args.device, platform_key_file=key, garble_device=dev,
                            client_kw={"pipeline": not args.no_pipeline, "transport": args._transport}) as enc:
            warm = xs[:args.batch]
            y0 = enc.ann_infer(warm)
            ok = all(np.array_equal(y, _plain(circuit, crt, mrs, x)) for x, y in zip(warm, y0))
            st0 = enc.last_stats
            n_gc = args.rounds * args.batch
            batch = [xs[i % len(xs)] for i in range(n_gc)]
            t0 = time.perf_counter()
            enc.ann_infer(batch)
            tot_s = time.perf_counter() - t0
            st = enc.last_stats  # cumulative over the enclave's lifetime
    off_b = st["offline_bytes"] - st0["offline_bytes"]
    off_s = st["offline_s"] - st0["offline_s"]
    on = [1000.0 * v for v in st["online_s"][len(st0["online_s"]):]]
    on_b = st["online_bytes"] - st0["online_bytes"]
    return dict(offline_gb_per_gc=off_b / n_gc / 1e9, offline_s_per_gc=off_s / n_gc,
                offline_gbps=off_b / max(off_s, 1e-9) / 1e9, garble_s_per_gc=(st["garble_s"] - st0["garble_s"]) / n_gc,
                serialize_s_per_gc=(st["serialize_s"] - st0["serialize_s"]) / n_gc,
                online_round_ms=float(np.median(on)), online_bytes_per_inference=on_b / n_gc,
                served_inf_per_s=n_gc / tot_s, verified=bool(ok), attested=True, encoding=st.get("encoding"))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--models", default=",".join(DEFAULT_MODELS))
    ap.add_argument("--splits", default="tcp,enclave")
    ap.add_argument("--backend", default="hip", choices=["hip", "cpu"])
    ap.add_argument("--device", type=int, default=0, help="the evaluator's GPU")
    ap.add_argument("--garble-device", type=int, default=0, help="the garbler's GPU (-1: host CPU garbler)")
    ap.add_argument("--batch", type=int, default=4, help="GCs per offline/online round")
    ap.add_argument("--rounds", type=int, default=4, help="timed rounds (after one warm-up round)")
    ap.add_argument("--no-pipeline", action="store_true")
    ap.add_argument("--transport", default="tcp,shm",
                    help="offline-message transports to measure per split: tcp (any host), shm (same host) and/or "
                         "ipc (same node, device memory; needs --backend hip and a garble device)")
    ap.add_argument("--out", default=None, help="also append the JSON lines to this file")
    args = ap.parse_args(argv)
    if args.backend == "cpu":
        args.garble_device = -1
    want = [m for m in args.models.split(",") if m]
    by_name = {config_name(c): c for c in CONFIGS}
    records = []
    for name in want:
        cfg = by_name[name]
        circuit = load_circuit(cfg, None)
        imgs = synthetic_inputs(cfg.model_name, 4 * args.batch, seed=3)
        xs = quantize_images(cfg, circuit, imgs)
        # range calibration (as the headline bench): lets the "auto" constructions pick the mixed-radix
        # rescale + joint ReLU where the tracked ranges allow (GarbledCircuit defaults)
        print(f"[two_party] {name}: calibrating ranges", file=sys.stderr, flush=True)
        cal = quantize_images(cfg, circuit, synthetic_inputs(cfg.model_name, 32, seed=0))
        crt0, _, _ = _gc_args(cfg)
        from dash_amd.garbling.gc import GarbledCircuit as _GC

        M = _GC(circuit, crt0, _gc_args(cfg)[1], garble_me=False).crt_modulus
        for i, x in enumerate(cal):  # one image at a time with a heartbeat (a large model takes minutes)
            circuit.calibrate([x], M, reset=i == 0)
            if i % 4 == 3:
                print(f"[two_party] {name}: calibrated {i + 1}/{len(cal)}", file=sys.stderr, flush=True)
        cons = _GC(circuit, crt0, _gc_args(cfg)[1], garble_me=False).effective_constructions()
        for split, tr in itertools.product(args.splits.split(","), args.transport.split(",")):
            if tr == "ipc" and (args.backend != "hip" or args.garble_device < 0):
                print(json.dumps({"bench": "two_party", "model": name, "split": split, "transport": tr,
                                  "skipped": "ipc needs --backend hip and a GPU garbler"}), flush=True)
                continue
            args._transport = tr
            t = time.perf_counter()
            r = (run_tcp if split == "tcp" else run_enclave)(circuit, cfg, xs, args)
            rec = dict(bench="two_party", model=name, split=split, transport=tr, constructions=cons,
                       backend=args.backend,
                       garbler=("gpu%d" % args.garble_device) if args.garble_device >= 0 else "cpu",
                       evaluator=f"{args.backend}{args.device if args.backend == 'hip' else ''}", batch=args.batch,
                       rounds=args.rounds, pipeline=not args.no_pipeline,
                       **{k: (round(v, 6) if isinstance(v, float) else v) for k, v in r.items()},
                       wall_s=round(time.perf_counter() - t, 2))
            if args.backend == "hip" and args.garble_device == args.device:
                rec["note"] = ("performance rehearsal: garbler and evaluator share one GPU (separate processes); "
                               "a trust-valid deployment puts the garbler on its own device or host")
            print(json.dumps(rec), flush=True)
            records.append(rec)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(json.dumps(rec) + "\n")
    return records


if __name__ == "__main__":
    main()
