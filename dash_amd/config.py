"""Typed run configuration.

The reference has no CLI flags: configuration is spread over compile-time
macros (SGX, BENCHMARK, GRR3, ...), constants (DEFAULT_NUM_THREADS, QL, ...),
API parameters and the benchmark `infer_config_t` structs. `DashConfig` mirrors
those parameters 1:1 and adds the run-time switches of this framework
(backend, garbler location, GCs per GPU, world size). Load from JSON/YAML or
argparse; every field has a CLI flag `--<field-with-dashes>`.

Environment variables (read by the native layer / build):
  DASH_NUM_THREADS   host worker threads (default min(#cpu, 16); reference DEFAULT_NUM_THREADS 16)
  DASH_AUTOBUILD     build the extension on import when missing (default 1)
  DASH_GPU_ARCH      offload arch for the HIP build (default gfx950)
  DASH_BENCH_BATCH   default GCs per GPU in bench.py
"""
from __future__ import annotations

import argparse
import json
from dataclasses import asdict, dataclass, field, fields
from typing import Optional, Union

from .ir.quant import QuantizationMethod

SCHEMES = {
    # scheme -> (q_method, q_parameter, crt, mrs)
    "DASH": (QuantizationMethod.ScaleQuant, 5, 7, 100.0),
    "REDASH_CPM": (QuantizationMethod.ScaleQuantPlus, 32, [32, 3, 5, 7, 11, 13, 17], [10, 9, 9, 8, 7, 7, 6]),
    "SIMPLE": (QuantizationMethod.SimpleQuant, -1, 8, 100.0),
}
OPT_BASES = {  # benchmarks/model_benchmarks/non_sgx/main.cpp:39-50
    "MODEL_F_GNNP_POOL_REPL": ([32, 167, 173], [26, 25, 21, 13]),
    "MODEL_F_MINIONN_POOL_REPL": ([32, 97, 107], [22, 19, 15, 13]),
}


@dataclass
class DashConfig:
    # model
    model: str = "MODEL_F_MINIONN_POOL_REPL"
    model_file: Optional[str] = None          # ONNX file; default: zoo architecture, random init
    scheme: str = "DASH"                      # DASH | REDASH_OPT | REDASH_CPM | SIMPLE
    q_method: Optional[str] = None            # override: SimpleQuant | ScaleQuant | ScaleQuantPlus
    q_parameter: Optional[int] = None
    q_const: float = 0.02                     # SimpleQuant constant (onnx_modelloader.h:377)
    # garbling
    crt: Union[int, list, None] = None        # k (first k primes) or explicit base
    mrs: Union[float, list, None] = None      # ReLU accuracy (table lookup) or explicit MRS base
    max_modulus: int = 0
    rescale: str = "auto"                     # DASH rescale construction: auto (mrs where the base and ranges allow) | mrs (one mixed-radix gadget) | legacy
    relu: str = "auto"                        # ReLU sign: auto (joint with the mrs rescale, else approx) | approx (reference gadget) | mrs (exact mixed radix) | joint (from the preceding mixed-radix rescale)
    sign: str = "fused"                       # approximate sign gadget: fused casts | reference
    encoding: str = "auto"                    # offline-message encoding: auto (hardened where the constructions allow; the serving engine then refuses the reference one) | hardened | reference (wire-compatible, R_p recoverable: docs/SECURITY.md §1.1)
    seed: Optional[str] = None                # hex seed for reproducible garbling (tests only)
    insecure_fixed_seed: bool = False         # allow `seed` in the serving engine (reuses labels across restarts)
    # execution
    backend: str = "hip"                      # hip | cpu
    garbler: str = "host"                     # host (in-process) | remote (dash_amd.net)
    device: int = 0
    batch: int = 8                            # garbled circuits per GPU evaluated together
    world_size: int = 1
    nthreads: int = 0
    mfma: bool = True
    profile: bool = False
    # serving (dash_amd.serving.InferenceService)
    groups: int = 2                           # evaluator groups in the GC slot pool (each `batch` slots)
    garble_device: Optional[bool] = None      # GPU garbler (default: on with the hip backend)
    max_retries: int = 2                      # re-garble + resubmit attempts after an IntegrityError
    step_timeout_s: float = 120.0             # watchdog deadline of one GPU evaluation
    # data
    dataset: Optional[str] = None             # mnist | cifar10 (None: synthetic)
    data_dir: Optional[str] = None
    inputs: int = 2
    # network (two-party)
    host: str = "127.0.0.1"
    port: int = 0
    extra: dict = field(default_factory=dict)

    # ------------------------------------------------------------ derived
    def gc_kwargs(self) -> dict:
        """GarbledCircuit keyword arguments selecting the gadget constructions."""
        if self.rescale not in ("auto", "mrs", "legacy") or self.relu not in ("auto", "approx", "mrs", "joint") or \
                self.sign not in ("fused", "reference"):
            raise ValueError(f"bad gadget construction: rescale={self.rescale} relu={self.relu} sign={self.sign}")
        if self.encoding not in ("auto", "hardened", "reference"):
            raise ValueError(f"bad encoding {self.encoding!r}: auto | hardened | reference")
        hardened = {"auto": None, "hardened": True, "reference": False}[self.encoding]
        return dict(rescale=self.rescale, relu=self.relu, fused_sign=self.sign == "fused", hardened=hardened)

    def resolved(self):
        """(q_method, q_parameter, crt, mrs, max_modulus) after applying the scheme."""
        if self.scheme == "REDASH_OPT":
            crt, mrs = OPT_BASES[self.model]
            qm, qp, mm = QuantizationMethod.ScaleQuantPlus, 32, max(crt)
        else:
            qm, qp, crt, mrs = SCHEMES[self.scheme]
            mm = max(crt) if isinstance(crt, list) else 0
        if self.q_method is not None:
            qm = QuantizationMethod[self.q_method]
        if self.q_parameter is not None:
            qp = self.q_parameter
        crt = self.crt if self.crt is not None else crt
        mrs = self.mrs if self.mrs is not None else mrs
        return qm, qp, crt, mrs, (self.max_modulus or mm)

    def seed_bytes(self) -> Optional[bytes]:
        """The 16-byte garbling seed, or None (fresh randomness).

        CLI values are JSON-decoded, so an all-digit hex seed arrives as an
        int: coerce to text and left-pad to 32 hex digits."""
        if self.seed is None or self.seed == "":
            return None
        text = str(self.seed).strip().lower()
        if text.startswith("0x"):
            text = text[2:]
        if len(text) > 32:
            raise ValueError("seed must be at most 16 bytes (32 hex digits)")
        return bytes.fromhex(text.zfill(32))

    # --------------------------------------------------------------- I/O
    def to_dict(self) -> dict:
        return asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "DashConfig":
        known = {f.name for f in fields(cls)}
        extra = {k: v for k, v in d.items() if k not in known}
        c = cls(**{k: v for k, v in d.items() if k in known})
        c.extra.update(extra)
        return c

    @classmethod
    def load(cls, path: str) -> "DashConfig":
        with open(path) as f:
            text = f.read()
        if path.endswith((".yaml", ".yml")):
            import yaml

            return cls.from_dict(yaml.safe_load(text) or {})
        return cls.from_dict(json.loads(text))

    def save(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=2)

    @classmethod
    def add_arguments(cls, ap: argparse.ArgumentParser) -> None:
        ap.add_argument("--config", default=None, help="JSON/YAML DashConfig file")
        for f in fields(cls):
            if f.name == "extra":
                continue
            flag = "--" + f.name.replace("_", "-")
            if f.type in ("bool",) or isinstance(f.default, bool):
                ap.add_argument(flag, default=None, action=argparse.BooleanOptionalAction)
            else:
                ap.add_argument(flag, default=None, type=_parse_value)

    @classmethod
    def from_args(cls, args: argparse.Namespace) -> "DashConfig":
        base = cls.load(args.config) if getattr(args, "config", None) else cls()
        d = base.to_dict()
        for f in fields(cls):
            v = getattr(args, f.name, None)
            if v is not None:
                d[f.name] = v
        return cls.from_dict(d)


def _parse_value(s: str):
    """CLI values: JSON when it parses (numbers, lists), else the raw string."""
    try:
        return json.loads(s)
    except (ValueError, TypeError):
        return s
