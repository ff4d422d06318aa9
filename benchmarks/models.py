#!/usr/bin/env python
"""Model benchmarks: garbled inference of the model zoo on CPU and GPU.

Mirrors benchmarks/model_benchmarks/{non_sgx,runtime_distribution}/main.cpp
of the reference: configs MODEL_A..F (non_sgx/main.cpp:227-335), a fresh
garbled circuit per input (:27-92), timed `cpu_evaluate + decode` (:96-99)
or, on the GPU, the online round `encode -> H2D -> evaluate -> D2H -> decode`
(sgx/Enclave/Enclave.cpp:177-183), SimpleQuant models quantized with
optimize_quantization(target_k, images, 0.25, 0.01, 0.0001) (:353-358).

CSV outputs (same columns as the reference):
  <date>_garbled_models.csv   type, model, target_crt_base_size, optimize_bases, runtime, relu_acc, label, infered_label
  <date>_plain_models.csv     model_name, plain_acc, plain_q_acc, target_crt_base_size
  with --distribution:
  <date>_runtime_distribution_{garbling,evaluation}.csv
                              type, model, layer, target_crt_base_size, optimize_bases, runtime, relu_acc

Weights: `--model-dir` with <MODEL>.onnx files if given, else the zoo's
random-init architecture. Data: `--mnist` / `--cifar10` directories if
given, else synthetic normalized images (labels then come from the plaintext
model, so 'accuracy' is garbled-vs-plaintext agreement).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dash_amd.garbling import GarbledCircuit  # noqa: E402
from dash_amd.ir.quant import QuantizationMethod, quantize_input  # noqa: E402
from dash_amd.models import build_circuit  # noqa: E402
from dash_amd.models.zoo import input_dims, synthetic_inputs  # noqa: E402
from dash_amd.utils.bench_util import InferConfig, csv_path, date_string  # noqa: E402

SQ, SC, SP = QuantizationMethod.SimpleQuant, QuantizationMethod.ScaleQuant, QuantizationMethod.ScaleQuantPlus

CONFIGS = [
    InferConfig("MODEL_A", "mnist", 8, [100.0], quantization_method="SimpleQuant", q_parameter=-1),
    InferConfig("MODEL_B_POOL_REPL", "mnist", 9, [100.0], quantization_method="SimpleQuant", q_parameter=-1),
    InferConfig("MODEL_C", "mnist", 9, [100.0], quantization_method="SimpleQuant", q_parameter=-1),
    InferConfig("MODEL_D_POOL_REPL", "mnist", 8, [100.0], quantization_method="SimpleQuant", q_parameter=-1),
    InferConfig("MODEL_F_GNNP_POOL_REPL", "cifar10", 7, [100.0], quantization_method="ScaleQuantPlus", q_parameter=32,
                optimize_bases=True, crt_base=[32, 167, 173], mrs_base=[26, 25, 21, 13]),
    InferConfig("MODEL_F_GNNP_POOL_REPL", "cifar10", 7, [100.0], quantization_method="ScaleQuantPlus", q_parameter=32,
                crt_base=[32, 3, 5, 7, 11, 13, 17], mrs_base=[10, 9, 9, 8, 7, 7, 6]),
    InferConfig("MODEL_F_GNNP_POOL_REPL", "cifar10", 7, [100.0], quantization_method="ScaleQuant", q_parameter=5),
    InferConfig("MODEL_F_MINIONN_POOL_REPL", "cifar10", 7, [100.0], quantization_method="ScaleQuantPlus",
                q_parameter=32, optimize_bases=True, crt_base=[32, 97, 107], mrs_base=[22, 19, 15, 13]),
    InferConfig("MODEL_F_MINIONN_POOL_REPL", "cifar10", 7, [100.0], quantization_method="ScaleQuantPlus",
                q_parameter=32, crt_base=[32, 3, 5, 7, 11, 13, 17], mrs_base=[10, 9, 9, 8, 7, 7, 6]),
    InferConfig("MODEL_F_MINIONN_POOL_REPL", "cifar10", 7, [100.0], quantization_method="ScaleQuant", q_parameter=5),
]


def config_name(c: InferConfig) -> str:
    tag = "OPT" if c.optimize_bases else ("CPM" if c.quantization_method == "ScaleQuantPlus" else
                                          ("DASH" if c.quantization_method == "ScaleQuant" else "SIMPLE"))
    return f"{c.model_name}/{tag}"


def load_circuit(cfg: InferConfig, model_dir, seed=0):
    qm = QuantizationMethod[cfg.quantization_method]
    path = os.path.join(model_dir, cfg.model_name + ".onnx") if model_dir else None
    if path and os.path.exists(path):
        from dash_amd.ir.onnx import load_onnx_model

        return load_onnx_model(path, qm, cfg.q_parameter)
    return build_circuit(cfg.model_name, qm, cfg.q_parameter, seed=seed)


def load_images(cfg: InferConfig, n: int, args):
    d = args.mnist if cfg.dataset == "mnist" else args.cifar10
    if d:
        from dash_amd import data

        ds = data.load(cfg.dataset, d)
        return [x.reshape(-1) for x in ds.test_images[:n]], list(ds.test_labels[:n])
    return synthetic_inputs(cfg.model_name, n, seed=args.seed), None


def quantize_images(cfg, circuit, imgs):
    qm = QuantizationMethod[cfg.quantization_method]
    if qm == SQ:
        circuit.optimize_quantization(cfg.target_crt_base_size, imgs, 0.25, 0.01, 0.0001)
        qc = circuit.get_q_const()
        return [quantize_input(x, qm, -1, qc) for x in imgs]
    if qm == SC:
        return [quantize_input(x, qm, cfg.q_parameter, 0.0) for x in imgs]
    return [quantize_input(x, qm, cfg.q_parameter, 0.0) for x in imgs]


def make_gc(cfg, circuit, relu_acc, device=None):
    """Reference constructions (the published numbers' gadgets): legacy rescale, approximate-sign ReLU, explicit
    casts. device: garble on this GPU (byte-identical to the host garbler)."""
    kw = dict(device=device, rescale="legacy", relu="approx", fused_sign=False)
    if cfg.crt_base:
        return GarbledCircuit(circuit, cfg.crt_base, cfg.mrs_base, max_modulus=max(cfg.crt_base), **kw)
    return GarbledCircuit(circuit, cfg.target_crt_base_size, relu_acc, **kw)


def scheme_of(cfg: InferConfig) -> str:
    return config_name(cfg).split("/")[1]


def layer_names(circuit):
    return [f"{i}_{l.name}" for i, l in enumerate(circuit.layers)]


def run_cpu(cfg, circuit, xq, labels, relu_acc, rows, dist_g, dist_e):
    preds = []
    for i, x in enumerate(xq):
        gc = make_gc(cfg, circuit, relu_acc)
        g = gc.garble_inputs(x)
        t = time.perf_counter()
        out, ms_layers = gc.cpu_evaluate_timed(g)
        y = gc.decode_outputs(out)
        ms = 1000 * (time.perf_counter() - t)
        pred = int(np.argmax(y))
        preds.append(pred)
        rows.append(["CPU", cfg.model_name, cfg.target_crt_base_size, int(cfg.optimize_bases), ms, relu_acc,
                     labels[i], pred, scheme_of(cfg)])
        for name, gms, ems in zip(layer_names(circuit), gc.garbling_layer_ms(), ms_layers):
            dist_g.append(["CPU", cfg.model_name, name, cfg.target_crt_base_size, int(cfg.optimize_bases), gms,
                           relu_acc, scheme_of(cfg)])
            dist_e.append(["CPU", cfg.model_name, name, cfg.target_crt_base_size, int(cfg.optimize_bases), ems,
                           relu_acc, scheme_of(cfg)])
        print(f"  CPU {config_name(cfg)} input {i}: {ms:.1f} ms  pred={pred} label={labels[i]}", flush=True)
    return preds


def run_gpu(cfg, circuit, xq, labels, relu_acc, rows, dist_e):
    import torch

    from dash_amd.runtime import HipEvaluator

    preds = []
    ev = None
    for i, x in enumerate(xq):
        gc = make_gc(cfg, circuit, relu_acc, device=0)  # fresh GC per input, garbled on the GPU
        if ev is None:
            ev = HipEvaluator(template=gc.model, batch=1, profile=bool(dist_e is not None))
        ev.load(0, gc.model)
        torch.cuda.synchronize()
        t = time.perf_counter()
        ev.encode_compressed_into(0, gc, x)
        ev.upload_inputs_compressed()
        ev.run()
        ev.fetch_outputs()
        y = ev.decode(0, gc)
        ms = 1000 * (time.perf_counter() - t)
        pred = int(np.argmax(y))
        preds.append(pred)
        rows.append(["GPU", cfg.model_name, cfg.target_crt_base_size, int(cfg.optimize_bases), ms, relu_acc,
                     labels[i], pred, scheme_of(cfg)])
        if dist_e is not None:
            for name, ems in ev.layer_times().items():
                dist_e.append(["GPU", cfg.model_name, name, cfg.target_crt_base_size, int(cfg.optimize_bases), ems,
                               relu_acc, scheme_of(cfg)])
        print(f"  GPU {config_name(cfg)} input {i}: {ms:.2f} ms  pred={pred} label={labels[i]}", flush=True)
    return preds


def write_csv(path, header, rows):
    with open(path, "w") as f:
        f.write(header + "\n")
        for r in rows:
            f.write(", ".join(f"{v:f}" if isinstance(v, float) else str(v) for v in r) + "\n")
    print("wrote", path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="", help="comma list of config names (MODEL/TAG), default: all")
    ap.add_argument("--targets", default="cpu,gpu")
    ap.add_argument("--inputs", type=int, default=2)
    ap.add_argument("--model-dir", default=None)
    ap.add_argument("--mnist", default=None)
    ap.add_argument("--cifar10", default=None)
    ap.add_argument("--distribution", action="store_true", help="also write per-layer runtime distribution CSVs")
    ap.add_argument("--out", default="data")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--list", action="store_true")
    args = ap.parse_args()
    if args.list:
        for c in CONFIGS:
            print(config_name(c))
        return
    want = set(filter(None, args.models.split(",")))
    targets = args.targets.split(",")
    if "gpu" in targets:
        from dash_amd.runtime import hip_available

        if not hip_available():
            print("no GPU visible: running cpu only", file=sys.stderr)
            targets = [t for t in targets if t != "gpu"]
    date = date_string()
    rows, plain_rows, dist_g, dist_e = [], [], [], []
    for cfg in CONFIGS:
        if want and config_name(cfg) not in want:
            continue
        print(f"== {config_name(cfg)}", flush=True)
        circuit = load_circuit(cfg, args.model_dir)
        imgs, labels = load_images(cfg, args.inputs, args)
        xq = quantize_images(cfg, circuit, imgs)
        if labels is None:  # synthetic data: reference labels from the plaintext float model
            labels = [int(np.argmax(circuit.plain_eval(x))) for x in imgs]
        plain_acc = circuit.plain_test(imgs, labels)
        plain_q_acc = circuit.plain_q_test(xq, labels)
        plain_rows.append([cfg.model_name, plain_acc, plain_q_acc, cfg.target_crt_base_size])
        for relu_acc in cfg.relu_accs:
            if "cpu" in targets:
                p = run_cpu(cfg, circuit, xq, labels, relu_acc, rows, dist_g, dist_e)
                print(f"  CPU accuracy {np.mean(np.array(p) == np.array(labels)):.3f}")
            if "gpu" in targets:
                p = run_gpu(cfg, circuit, xq, labels, relu_acc, rows, dist_e if args.distribution else None)
                print(f"  GPU accuracy {np.mean(np.array(p) == np.array(labels)):.3f}")
    write_csv(csv_path(args.out, date, "garbled_models"),
              "type, model, target_crt_base_size, optimize_bases, runtime, relu_acc, label, infered_label", rows)
    write_csv(csv_path(args.out, date, "plain_models"), "model_name, plain_acc, plain_q_acc, target_crt_base_size",
              plain_rows)
    if args.distribution:
        h = "type, model, layer, target_crt_base_size, optimize_bases, runtime, relu_acc"
        write_csv(csv_path(args.out, date, "runtime_distribution_garbling"), h, dist_g)
        write_csv(csv_path(args.out, date, "runtime_distribution_evaluation"), h, dist_e)


if __name__ == "__main__":
    main()
