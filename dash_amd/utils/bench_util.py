"""Benchmark utilities (reference: benchmarks/benchmark_utilities.h:19-35):
date-stamped CSV naming, run configuration records, JSON-lines metrics."""
from __future__ import annotations

import json
import os
import time
from dataclasses import asdict, dataclass, field
from typing import Optional


def date_string() -> str:
    return time.strftime("%Y-%m-%d_%H-%M-%S")


def create_dir(path: str) -> str:
    os.makedirs(path, exist_ok=True)
    return path


def csv_path(out_dir: str, date: str, name: str) -> str:
    return os.path.join(create_dir(out_dir), f"{date}_{name}.csv")


@dataclass
class InferConfig:
    """infer_config_t of the reference (benchmark_utilities.h:19-28)."""
    model_name: str
    dataset: str = "cifar10"
    target_crt_base_size: int = 7
    relu_accs: list = field(default_factory=lambda: [100.0])
    model_file: Optional[str] = None
    quantization_method: str = "ScaleQuant"
    q_parameter: int = 5
    optimize_bases: bool = False
    crt_base: Optional[list] = None
    mrs_base: Optional[list] = None
    max_modulus: int = 0


class MetricsWriter:
    """JSON-lines metrics sink: one record per call."""

    def __init__(self, path: Optional[str]):
        self.path = path
        if path:
            create_dir(os.path.dirname(path) or ".")

    def write(self, **rec) -> None:
        rec.setdefault("time", time.time())
        line = json.dumps(rec, default=lambda o: asdict(o) if hasattr(o, "__dataclass_fields__") else str(o))
        if self.path:
            with open(self.path, "a") as f:
                f.write(line + "\n")
        else:
            print(line, flush=True)
