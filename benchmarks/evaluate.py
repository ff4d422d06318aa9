#!/usr/bin/env python
"""Aggregate benchmark CSVs and the analytic communication model.

Reference: benchmarks/evaluation.ipynb (C49): CSV aggregation, CPU/GPU
speed-ups, and the communication model of cells at :895-950 — per inference
  plain input     16 bit per input element
  garbled inputs  input_size * k * 128 bit (compressed labels)
  garbled outputs 10 * k * 128 bit
  plain outputs   64 bit each
with transfer time at 1 Gbit/s plus 100 % overhead.

  python benchmarks/evaluate.py --dir data            # summarize every CSV in data/
  python benchmarks/evaluate.py --comm                # communication table
"""
from __future__ import annotations

import argparse
import glob
import os

import numpy as np


def comm_model(input_size: int, k: int, n_out: int = 10, gbit: float = 1.0, overhead: float = 1.0) -> dict:
    bits = 16 * input_size + input_size * k * 128 + n_out * k * 128 + 64 * n_out
    mb = bits / 8 / 2**20  # the notebook reports MiB (0.335 for CIFAR-10, k = 7)
    return {"MB": mb, "ms_at_link": 1000 * bits * (1 + overhead) / (gbit * 1e9)}


def summarize(path: str) -> str:
    import pandas as pd

    df = pd.read_csv(path, skipinitialspace=True)
    keys = [c for c in ("type", "model", "dimensions", "crt_base_size", "target_crt_base_size", "relu_acc",
                        "sign_acc", "use_legacy_scaling", "nr_threads", "optimize_bases", "layer") if c in df.columns]
    g = df.groupby(keys)["runtime"].agg(["count", "mean", "std", "min"]).reset_index()
    out = [f"== {os.path.basename(path)}", g.to_string(index=False)]
    if "type" in df.columns and set(df["type"]) >= {"CPU", "GPU"}:
        k2 = [k for k in keys if k != "type"]
        cpu = df[df["type"] == "CPU"].groupby(k2)["runtime"].mean()
        gpu = df[df["type"] == "GPU"].groupby(k2)["runtime"].mean()
        sp = (cpu / gpu).dropna()
        if len(sp):
            out.append("GPU speed-up over CPU:\n" + sp.to_string())
    if "infered_label" in df.columns:
        acc = df.assign(ok=df["label"] == df["infered_label"]).groupby(["type", "model"])["ok"].mean()
        out.append("prediction accuracy:\n" + acc.to_string())
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="data")
    ap.add_argument("--comm", action="store_true")
    args = ap.parse_args()
    if args.comm:
        rows = [("CIFAR-10 (3x32x32)", 3072, 7), ("MNIST (1x28x28)", 784, 8)]
        print(f"{'dataset':22s} {'k':>3s} {'MB/inference':>13s} {'ms @1Gbit/s+100%':>17s}")
        for name, n, k in rows:
            c = comm_model(n, k)
            print(f"{name:22s} {k:3d} {c['MB']:13.3f} {c['ms_at_link']:17.2f}")
    files = sorted(glob.glob(os.path.join(args.dir, "*.csv")))
    for f in files:
        try:
            print(summarize(f))
        except Exception as e:  # a malformed file must not stop the report
            print(f"== {f}: {e}")
    if not files and not args.comm:
        print(f"no CSV files in {args.dir}")
    _ = np


if __name__ == "__main__":
    main()
