#!/usr/bin/env python
"""Evaluation: the outputs of the reference's analysis notebooks, from this
framework's benchmark CSVs.

Reference: benchmarks/evaluation.ipynb and benchmarks/evaluation_redash.ipynb (C49):

* CSV aggregation and GPU-over-CPU speed-ups (evaluation.ipynb);
* per-layer runtime distribution, ReDash (optimized / CPM bases) vs DASH, as a
  table and stacked bars (evaluation_redash.ipynb:415-416, :700-740);
* model runtime against competitor frameworks, log scale
  (evaluation.ipynb:848-856);
* micro-benchmark runtime and GPU memory against layer size;
* the analytic communication model (evaluation.ipynb:895-950): per inference
    plain input     16 bit per input element
    garbled inputs  input_size * k * 128 bit (compressed labels)
    garbled outputs 10 * k * 128 bit
    plain outputs   64 bit each
  with transfer time at 1 Gbit/s plus 100 % overhead.

  python benchmarks/evaluate.py --dir data                      # summarize every CSV
  python benchmarks/evaluate.py --comm                          # communication table
  python benchmarks/evaluate.py --dir data --layers             # per-layer ReDash / DASH table
  python benchmarks/evaluate.py --dir data --plots plots [--bench BENCH.json ...]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
from typing import Dict, List, Optional

import numpy as np

# Published per-layer CPU runtimes, ms per inference (evaluation_redash.ipynb:719-740; 16 threads, Xeon Gold 5415+)
PAPER_CPU_LAYERS = {
    ("MODEL_F_MINIONN_POOL_REPL", "DASH"): {"approx_relu": 981, "conv2d": 17760, "dense": 0.6, "rescale": 5274},
    ("MODEL_F_MINIONN_POOL_REPL", "CPM"): {"approx_relu": 982, "conv2d": 13393, "dense": 0.6, "rescale": 763},
    ("MODEL_F_MINIONN_POOL_REPL", "OPT"): {"approx_relu": 433, "conv2d": 2742, "dense": 0.2, "rescale": 455},
    ("MODEL_F_GNNP_POOL_REPL", "DASH"): {"approx_relu": 538, "conv2d": 6771, "dense": 0.6, "rescale": 2841},
    ("MODEL_F_GNNP_POOL_REPL", "CPM"): {"approx_relu": 529, "conv2d": 5135, "dense": 0.5, "rescale": 437},
}
# Whole-model latencies, ms per inference (evaluation.ipynb:848-856; evaluation_redash.ipynb:415-416)
COMPETITORS = {
    "MODEL_F_MINIONN_POOL_REPL": {"MiniONN": 72000, "GAZELLE": 3560, "MUSE/SIMC": 7860, "DASH CPU": 23959,
                                  "DASH GPU (RTX 4090)": 1443},
    "MODEL_F_GNNP_POOL_REPL": {"GNNP": 97000, "DASH CPU": 10263, "DASH GPU (RTX 4090)": 1332},
}
LAYER_KINDS = ("approx_relu", "conv2d", "dense", "rescale", "sign", "max_pool", "sum_pool", "add")


def comm_model(input_size: int, k: int, n_out: int = 10, gbit: float = 1.0, overhead: float = 1.0) -> dict:
    bits = 16 * input_size + input_size * k * 128 + n_out * k * 128 + 64 * n_out
    mb = bits / 8 / 2**20  # the notebook reports MiB (0.335 for CIFAR-10, k = 7)
    return {"MB": mb, "ms_at_link": 1000 * bits * (1 + overhead) / (gbit * 1e9)}


def _read(path: str):
    import pandas as pd

    return pd.read_csv(path, skipinitialspace=True)


def summarize(path: str) -> str:
    df = _read(path)
    keys = [c for c in ("type", "model", "scheme", "dimensions", "crt_base_size", "target_crt_base_size", "relu_acc",
                        "sign_acc", "use_legacy_scaling", "nr_threads", "optimize_bases", "layer") if c in df.columns]
    g = df.groupby(keys)["runtime"].agg(["count", "mean", "std", "min"]).reset_index()
    out = [f"== {os.path.basename(path)}", g.to_string(index=False)]
    if "type" in df.columns and {"CPU", "GPU"} <= set(df["type"]):
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


def _kind(layer: str) -> str:
    """'conv2d#3' (GPU op names) / '3_conv2d' (CPU per-layer timers) -> 'conv2d'."""
    name = str(layer).split("#")[0]
    return re.sub(r"^\d+_", "", name)


def _scheme(row) -> str:
    if "scheme" in row and isinstance(row["scheme"], str):
        return row["scheme"]
    return "OPT" if int(row.get("optimize_bases", 0)) else "DASH"


def layer_table(dist_paths: List[str]):
    """Per-layer-kind runtime per inference (ms) for every (type, model, scheme) of the
    runtime-distribution CSVs, beside the paper's CPU numbers where published."""
    import pandas as pd

    frames = [_read(p) for p in dist_paths]
    df = pd.concat(frames, ignore_index=True)
    df["kind"] = df["layer"].map(_kind)
    df["scheme"] = df.apply(_scheme, axis=1)
    rows = []
    for (typ, model, scheme), g in df.groupby(["type", "model", "scheme"]):
        first = g["layer"].iloc[0]
        n_inputs = max(1, int((g["layer"] == first).sum()))
        per = g.groupby("kind")["runtime"].sum() / n_inputs
        rec = {"type": typ, "model": model, "scheme": scheme, **{k: float(per.get(k, 0.0)) for k in per.index}}
        rec["total"] = float(per.sum())
        paper = PAPER_CPU_LAYERS.get((model, scheme))
        if paper:
            rec["paper_cpu_total"] = float(sum(paper.values()))
            rec["speedup_vs_paper_cpu"] = rec["paper_cpu_total"] / rec["total"] if rec["total"] else float("nan")
        rows.append(rec)
    for (model, scheme), paper in PAPER_CPU_LAYERS.items():
        rows.append({"type": "paper CPU", "model": model, "scheme": scheme, **paper, "total": float(sum(paper.values()))})
    return pd.DataFrame(rows).fillna(0.0)


def _plt():
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    return plt


def plot_distribution(table, out_dir: str) -> List[str]:
    """Stacked per-layer bars (log y) per model: this framework's runs and the paper's CPU numbers."""
    plt = _plt()
    paths = []
    kinds = [k for k in LAYER_KINDS if k in table.columns and table[k].sum() > 0]
    for model, g in table.groupby("model"):
        g = g.sort_values(["type", "scheme"])
        labels = [f"{t}\n{s}" for t, s in zip(g["type"], g["scheme"])]
        fig, ax = plt.subplots(figsize=(max(6, 1.2 * len(g)), 4.5))
        bottom = np.zeros(len(g))
        for k in kinds:
            v = g[k].to_numpy(dtype=float)
            ax.bar(labels, v, bottom=bottom, label=k)
            bottom += v
        ax.set_yscale("log")
        ax.set_ylabel("ms per inference")
        ax.set_title(f"{model}: runtime distribution by layer kind")
        ax.legend(fontsize=8)
        fig.tight_layout()
        p = os.path.join(out_dir, f"distribution_{model}.png")
        fig.savefig(p, dpi=120)
        plt.close(fig)
        paths.append(p)
    return paths


def plot_competitors(ours: Dict[str, Dict[str, float]], out_dir: str) -> List[str]:
    """Model latency against other frameworks (log y); `ours`: model -> {label: ms}."""
    plt = _plt()
    paths = []
    for model, comp in COMPETITORS.items():
        vals = dict(comp)
        vals.update(ours.get(model, {}))
        fig, ax = plt.subplots(figsize=(8, 4.5))
        names = list(vals)
        colors = ["tab:orange" if n in ours.get(model, {}) else "tab:gray" for n in names]
        ax.bar(names, [vals[n] for n in names], color=colors)
        ax.set_yscale("log")
        ax.set_ylabel("ms per inference")
        ax.set_title(f"{model}: garbled inference vs other frameworks")
        ax.tick_params(axis="x", labelrotation=30, labelsize=8)
        for i, n in enumerate(names):
            ax.text(i, vals[n], f"{vals[n]:.3g}", ha="center", va="bottom", fontsize=7)
        fig.tight_layout()
        p = os.path.join(out_dir, f"competitors_{model}.png")
        fig.savefig(p, dpi=120)
        plt.close(fig)
        paths.append(p)
    return paths


def plot_micro(paths_csv: List[str], out_dir: str) -> List[str]:
    """Runtime (and GPU memory) against layer size for every micro-benchmark CSV, one line per target."""
    plt = _plt()
    out = []
    for path in paths_csv:
        df = _read(path)
        if "dimensions" not in df.columns or "type" not in df.columns:
            continue
        layer = os.path.basename(path).rsplit("_", 1)[-1].replace(".csv", "")
        fig, axes = plt.subplots(1, 2, figsize=(10, 4))
        for typ, g in df.groupby("type"):
            m = g.groupby("dimensions", sort=False)[["runtime", "gpu_mem_usage"]].mean()
            x = list(m.index.astype(str))
            axes[0].plot(x, m["runtime"], marker="o", label=typ)
            if (m["gpu_mem_usage"] > 0).any():
                axes[1].plot(x, m["gpu_mem_usage"] / 2**20, marker="o", label=typ)
        axes[0].set_yscale("log")
        axes[0].set_ylabel("ms per garbled circuit")
        axes[1].set_ylabel("GPU MiB per garbled circuit")
        for ax in axes:
            ax.set_xlabel("dimensions")
            ax.tick_params(axis="x", labelrotation=30, labelsize=7)
            ax.legend(fontsize=8)
        fig.suptitle(f"micro-benchmark: {layer}")
        fig.tight_layout()
        p = os.path.join(out_dir, f"micro_{layer}.png")
        fig.savefig(p, dpi=120)
        plt.close(fig)
        out.append(p)
    return out


def ours_from(bench_jsons: List[str], models_csvs: List[str]) -> Dict[str, Dict[str, float]]:
    """This framework's MiniONN / GNNP latencies: batch-1 GPU latency from the model-benchmark CSVs and the
    throughput-equivalent ms per inference (1000 / inf/s) of bench.py JSON lines."""
    ours: Dict[str, Dict[str, float]] = {}
    for p in models_csvs:
        df = _read(p)
        if "runtime" not in df.columns:
            continue
        for (typ, model), g in df.groupby(["type", "model"]):
            ours.setdefault(model, {})[f"dash_amd {typ} batch 1"] = float(g["runtime"].mean())
    for p in bench_jsons:
        try:
            d = json.loads(open(p).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        model = d.get("config", {}).get("model")
        if model and d.get("value"):
            n = d.get("n_gpus", 1)
            ours.setdefault(model, {})[f"dash_amd {n}x MI355X (throughput)"] = 1000.0 / float(d["value"])
            if d.get("reference_constructions_value"):
                ours[model][f"dash_amd {n}x MI355X, ref. gadgets"] = 1000.0 / float(d["reference_constructions_value"])
            if d.get("served_inf_per_s"):
                ours[model][f"dash_amd {n}x MI355X, fresh GC (served)"] = 1000.0 / float(d["served_inf_per_s"])
    return ours


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="data")
    ap.add_argument("--comm", action="store_true")
    ap.add_argument("--layers", action="store_true", help="per-layer ReDash / DASH table from runtime-distribution CSVs")
    ap.add_argument("--plots", default=None, help="write PNG plots to this directory")
    ap.add_argument("--bench", nargs="*", default=[], help="bench.py JSON outputs (competitor plot)")
    args = ap.parse_args()
    if args.comm:
        rows = [("CIFAR-10 (3x32x32)", 3072, 7), ("MNIST (1x28x28)", 784, 8)]
        print(f"{'dataset':22s} {'k':>3s} {'MB/inference':>13s} {'ms @1Gbit/s+100%':>17s}")
        for name, n, k in rows:
            c = comm_model(n, k)
            print(f"{name:22s} {k:3d} {c['MB']:13.3f} {c['ms_at_link']:17.2f}")
    files = sorted(glob.glob(os.path.join(args.dir, "*.csv")))
    dist = [f for f in files if "runtime_distribution_evaluation" in f]
    models = [f for f in files if f.endswith("garbled_models.csv")]
    micro = [f for f in files if re.search(r"_(dense|conv2d|approx_relu|sign|rescaling)\.csv$", f)]
    table = None
    if args.layers or args.plots:
        if dist:
            table = layer_table(dist)
            if args.layers:
                import pandas as pd

                with pd.option_context("display.width", 200, "display.max_columns", 20):
                    print("== per-layer runtime, ms per inference (ReDash OPT / CPM vs DASH)")
                    print(table.round(3).to_string(index=False))
        elif args.layers:
            print(f"no runtime_distribution_evaluation CSV in {args.dir}")
    if args.plots:
        os.makedirs(args.plots, exist_ok=True)
        made = []
        if table is not None:
            made += plot_distribution(table, args.plots)
        made += plot_competitors(ours_from(args.bench, models), args.plots)
        made += plot_micro(micro, args.plots)
        for p in made:
            print("wrote", p)
    if not (args.layers or args.plots):
        for f in files:
            try:
                print(summarize(f))
            except Exception as e:  # a malformed file must not stop the report
                print(f"== {f}: {e}")
        if not files and not args.comm:
            print(f"no CSV files in {args.dir}")
    return table


if __name__ == "__main__":
    main()
