"""Command line driver (reference: dash/example/main.cpp, C42).

  python -m dash_amd info
  python -m dash_amd infer   [--model M | --model-file f.onnx] [--scheme DASH] [--backend hip|cpu] [--batch B]
                             [--dataset cifar10 --data-dir D] [--inputs N]
  python -m dash_amd garble  --out model.dgc [--decoder-out dec.bin] [...model flags]
  python -m dash_amd serve   --port P [--backend hip|cpu]          (evaluator party)
  python -m dash_amd client  --host H --port P [...model flags]    (garbler party)
  python -m dash_amd run-service [...model flags] [--batch B --groups G --max-retries R --step-timeout-s T]
                             (serving engine: GC pool re-garbled in the background, recovery, watchdog)
  python -m dash_amd export-onnx --model M --out m.onnx
"""
from __future__ import annotations

import argparse
import sys
import time

import numpy as np


def _circuit_and_inputs(cfg):
    from .ir.quant import QuantizationMethod, quantize_input
    from .models import build_circuit
    from .models.zoo import synthetic_inputs

    qm, qp, crt, mrs, mm = cfg.resolved()
    if cfg.model_file:
        from .ir.onnx import load_onnx_model

        circuit = load_onnx_model(cfg.model_file, qm, qp, cfg.q_const)
    else:
        circuit = build_circuit(cfg.model, qm, qp, cfg.q_const, seed=0)
    labels = None
    if cfg.dataset and cfg.data_dir:
        from . import data

        ds = data.load(cfg.dataset, cfg.data_dir)
        imgs = [x.reshape(-1) for x in ds.test_images[:cfg.inputs]]
        labels = list(ds.test_labels[:cfg.inputs])
    else:
        imgs = synthetic_inputs(cfg.model, cfg.inputs) if not cfg.model_file else \
            [np.random.default_rng(i).standard_normal(circuit.input_size).astype(np.float32)
             for i in range(cfg.inputs)]
    if qm == QuantizationMethod.SimpleQuant:
        k = crt if isinstance(crt, int) else len(crt)
        circuit.optimize_quantization(k, imgs, 0.25, 0.01, 0.0001)
        xq = [quantize_input(x, qm, -1, circuit.get_q_const()) for x in imgs]
    else:
        xq = [quantize_input(x, qm, qp, cfg.q_const) for x in imgs]
    return circuit, imgs, xq, labels, (crt, mrs, mm)


def cmd_info(_args):
    import dash_amd
    from .native import native
    from .runtime import hip_available

    n = native()
    print(f"dash_amd {dash_amd.__version__}")
    print(f"native extension: {n.__file__}")
    print(f"host threads: {n.get_num_threads()}")
    print(f"HIP devices: {n.hip_device_count() if hip_available() else 0}")


def cmd_infer(args):
    from .config import DashConfig
    from .garbling import GarbledCircuit

    cfg = DashConfig.from_args(args)
    circuit, imgs, xq, labels, (crt, mrs, mm) = _circuit_and_inputs(cfg)
    print(circuit)
    ev = None
    preds, times = [], []
    B = max(1, cfg.batch if cfg.backend == "hip" else 1)
    for s in range(0, len(xq), B):
        chunk = xq[s:s + B]
        gcs = [GarbledCircuit(circuit, crt, mrs, max_modulus=mm, nthreads=cfg.nthreads,
                              device=cfg.device if (cfg.garble_device if cfg.garble_device is not None
                                                     else cfg.backend == "hip") else None,
                              **cfg.gc_kwargs()) for _ in chunk]
        t = time.perf_counter()
        if cfg.backend == "hip":
            from .runtime import HipEvaluator

            if ev is None or ev.batch != len(chunk):
                ev = HipEvaluator(template=gcs[0].model, batch=len(chunk), device=cfg.device, mfma=cfg.mfma)
            t_load = time.perf_counter()
            for b, gc in enumerate(gcs):
                ev.load(b, gc.model)
            t = time.perf_counter()
            for b, (gc, x) in enumerate(zip(gcs, chunk)):
                ev.encode_compressed_into(b, gc, x)
            ev.upload_inputs_compressed()
            ev.run()
            ev.fetch_outputs()
            outs = [ev.decode(b, gc) for b, gc in enumerate(gcs)]
            _ = t_load
        else:
            outs = [gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x), cfg.nthreads)) for gc, x in zip(gcs, chunk)]
        dt = time.perf_counter() - t
        times.append(dt / len(chunk))
        for gc, x, y in zip(gcs, chunk, outs):
            ref = gc.plain_q_eval(x)
            ok = np.array_equal(ref, y)
            preds.append(int(np.argmax(y)))
            print(f"input {len(preds) - 1}: pred {preds[-1]}  garbled==plaintext: {ok}")
    print(f"online time per inference: {1000 * np.mean(times):.2f} ms ({cfg.backend})")
    if labels is not None:
        print(f"accuracy: {np.mean(np.array(preds) == np.array(labels)):.4f}")


def cmd_run_service(args):
    import json

    from .config import DashConfig
    from .serving import InferenceService

    cfg = DashConfig.from_args(args)
    if cfg.seed_bytes() is not None and not cfg.insecure_fixed_seed:
        # a fixed seed replays the same GC sequence (labels, offsets) on every restart, with new inputs
        raise SystemExit("run-service: --seed makes every restart reuse the same garbled circuits; "
                         "pass --insecure-fixed-seed to allow it (tests only)")
    circuit, _, xq, labels, (crt, mrs, mm) = _circuit_and_inputs(cfg)
    with InferenceService(circuit, crt, mrs, max_modulus=mm, slots_per_group=max(1, cfg.batch), groups=cfg.groups,
                          backend=cfg.backend, device=cfg.device, garble_device=cfg.garble_device,
                          max_retries=cfg.max_retries, step_timeout_s=cfg.step_timeout_s, seed=cfg.seed_bytes(),
                          nthreads=cfg.nthreads, insecure_fixed_seed=cfg.insecure_fixed_seed, **cfg.gc_kwargs()) as svc:
        ys = svc.infer(xq)
        stats = svc.stats.as_dict()
    preds = [int(np.argmax(y)) for y in ys]
    for i, p in enumerate(preds):
        print(f"input {i}: pred {p}")
    if labels is not None:
        print(f"accuracy: {np.mean(np.array(preds) == np.array(labels)):.4f}")
    print(json.dumps(stats))


def cmd_garble(args):
    from .config import DashConfig
    from .garbling import GarbledCircuit

    cfg = DashConfig.from_args(args)
    circuit, _, _, _, (crt, mrs, mm) = _circuit_and_inputs(cfg)
    gc = GarbledCircuit(circuit, crt, mrs, max_modulus=mm, seed=cfg.seed_bytes(), nthreads=cfg.nthreads,
                        **cfg.gc_kwargs())
    with open(args.out, "wb") as f:
        f.write(gc.model.serialize())
    if args.decoder_out:
        with open(args.decoder_out, "wb") as f:
            f.write(gc.decoder.serialize())
    print(f"garbled in {gc.garbling_time_s:.2f} s; {gc.table_bytes / 1e9:.3f} GB tables -> {args.out}")


def cmd_serve(args):
    from .net import listen
    from .net.protocol import EvaluatorServer
    from .net.channel import Channel

    s = listen(args.host or "127.0.0.1", int(args.port or 0))
    print(f"evaluator listening on {s.getsockname()[0]}:{s.getsockname()[1]} ({args.backend or 'hip'})", flush=True)
    while True:
        conn, addr = s.accept()
        print(f"garbler connected from {addr}", flush=True)
        EvaluatorServer(args.backend or "hip", int(args.device or 0)).serve(Channel(conn))
        if args.once:
            break


def cmd_client(args):
    from .config import DashConfig
    from .net import GarblerClient

    cfg = DashConfig.from_args(args)
    circuit, _, xq, _, (crt, mrs, mm) = _circuit_and_inputs(cfg)
    B = max(1, cfg.batch)
    with GarblerClient(cfg.host, int(cfg.port), circuit, crt, mrs, batch=B, max_modulus=mm) as cl:
        print("server:", cl.server_info)
        for s in range(0, len(xq) - B + 1, B):
            cl.offline()
            outs = cl.infer(xq[s:s + B])
            for x, y in zip(xq[s:s + B], outs):
                print("pred", int(np.argmax(y)), y.tolist())
        st = cl.stats
        n = max(1, len(st["online_s"]) * B)
        print(f"offline: {st['offline_bytes'] / 1e9:.3f} GB, {st['offline_s']:.2f} s; online: "
              f"{st['online_bytes'] / n / 1e6:.3f} MB/inference, {1000 * sum(st['online_s']) / n:.2f} ms/inference")


def cmd_export(args):
    from .ir.onnx import save_onnx_model
    from .ir.quant import QuantizationMethod
    from .models import build_circuit

    c = build_circuit(args.model, QuantizationMethod.SimpleQuant, -1, seed=0)
    save_onnx_model(args.out, c)
    print("wrote", args.out)


def main(argv=None):
    from .config import DashConfig

    ap = argparse.ArgumentParser(prog="python -m dash_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("info")
    for name in ("infer", "garble", "client", "run-service"):
        p = sub.add_parser(name)
        DashConfig.add_arguments(p)
        if name == "garble":
            p.add_argument("--out", required=True)
            p.add_argument("--decoder-out", default=None)
    p = sub.add_parser("serve")
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--port", default=0, type=int)
    p.add_argument("--backend", default="hip")
    p.add_argument("--device", default=0, type=int)
    p.add_argument("--once", action="store_true")
    p = sub.add_parser("export-onnx")
    p.add_argument("--model", required=True)
    p.add_argument("--out", required=True)
    args = ap.parse_args(argv)
    {"info": cmd_info, "infer": cmd_infer, "garble": cmd_garble, "serve": cmd_serve, "client": cmd_client,
     "export-onnx": cmd_export, "run-service": cmd_run_service}[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())
