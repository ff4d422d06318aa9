"""Model zoo: the paper's architectures (models/train_pytorch.ipynb, SURVEY
Appendix B) plus LeNet-5, VGG-16 and ResNet-18 for CIFAR-10, built directly in
the IR with random (PyTorch-default) initialisation and quantized with one of
Dash's three schemes. Rescale layers are auto-inserted after every linear
layer exactly like the ONNX loader does (onnx_modelloader.h:263-270, :334-341).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from ..ir.circuit import Circuit
from ..ir.layers import Add, Conv2d, Dense, Flatten, MaxPool2d, Relu, Rescale, Sign, SumPool2d
from ..ir.quant import QuantizationMethod, quantize_input

# architecture ops: ("conv", out_ch, k, stride, pad) | ("relu",) | ("sign",) | ("flatten",) | ("fc", out)
#                   | ("maxpool", k, s) | ("res", [ops...]) residual block | ("sumpool", k)
ARCHS: dict[str, dict] = {
    "MODEL_A": {"input": (1, 28, 28), "ops": [("flatten",), ("fc", 128), ("relu",), ("fc", 128), ("relu",), ("fc", 10)]},
    "MODEL_B_POOL_REPL": {"input": (1, 28, 28), "ops": [
        ("conv", 5, 5, 1, 0), ("relu",), ("conv", 5, 3, 3, 0), ("relu",), ("conv", 10, 3, 1, 0), ("relu",),
        ("conv", 10, 3, 3, 0), ("flatten",), ("fc", 100), ("relu",), ("fc", 10)]},
    "MODEL_C": {"input": (1, 28, 28), "ops": [
        ("conv", 5, 4, 2, 0), ("relu",), ("flatten",), ("fc", 100), ("relu",), ("fc", 10)]},
    "MODEL_D_POOL_REPL": {"input": (1, 28, 28), "ops": [
        ("conv", 16, 6, 2, 0), ("relu",), ("conv", 16, 6, 2, 0), ("relu",), ("flatten",), ("fc", 100), ("relu",),
        ("fc", 10)]},
    "MODEL_E_30": {"input": (1, 28, 28), "ops": [("flatten",), ("fc", 30), ("sign",), ("fc", 10)]},
    "MODEL_E_100": {"input": (1, 28, 28), "ops": [("flatten",), ("fc", 100), ("sign",), ("fc", 10)]},
    "MODEL_F_MINIONN_POOL_REPL": {"input": (3, 32, 32), "ops": [
        ("conv", 64, 3, 1, 0), ("relu",), ("conv", 64, 3, 1, 0), ("relu",), ("conv", 64, 2, 2, 0),
        ("conv", 64, 3, 1, 0), ("relu",), ("conv", 64, 3, 1, 0), ("relu",), ("conv", 64, 2, 2, 0),
        ("conv", 64, 3, 1, 0), ("relu",), ("conv", 64, 1, 1, 0), ("relu",), ("conv", 16, 1, 1, 0), ("relu",),
        ("flatten",), ("fc", 10)]},
    "MODEL_F_GNNP_POOL_REPL": {"input": (3, 32, 32), "ops": [
        ("conv", 32, 3, 1, 0), ("relu",), ("conv", 32, 3, 1, 0), ("relu",), ("conv", 32, 2, 2, 0),
        ("conv", 64, 3, 1, 0), ("relu",), ("conv", 64, 3, 1, 0), ("relu",), ("conv", 64, 2, 2, 0),
        ("conv", 128, 3, 1, 0), ("relu",), ("conv", 128, 3, 1, 0), ("relu",), ("flatten",), ("fc", 10)]},
    # beyond the reference (BASELINE configs 2, 4, 5)
    "LENET5": {"input": (1, 28, 28), "ops": [
        ("conv", 6, 5, 1, 2), ("relu",), ("maxpool", 2, 2), ("conv", 16, 5, 1, 0), ("relu",), ("maxpool", 2, 2),
        ("flatten",), ("fc", 120), ("relu",), ("fc", 84), ("relu",), ("fc", 10)]},
    "VGG16": {"input": (3, 32, 32), "ops": [
        ("conv", 64, 3, 1, 1), ("relu",), ("conv", 64, 3, 1, 1), ("relu",), ("maxpool", 2, 2),
        ("conv", 128, 3, 1, 1), ("relu",), ("conv", 128, 3, 1, 1), ("relu",), ("maxpool", 2, 2),
        ("conv", 256, 3, 1, 1), ("relu",), ("conv", 256, 3, 1, 1), ("relu",), ("conv", 256, 3, 1, 1), ("relu",),
        ("maxpool", 2, 2),
        ("conv", 512, 3, 1, 1), ("relu",), ("conv", 512, 3, 1, 1), ("relu",), ("conv", 512, 3, 1, 1), ("relu",),
        ("maxpool", 2, 2),
        ("conv", 512, 3, 1, 1), ("relu",), ("conv", 512, 3, 1, 1), ("relu",), ("conv", 512, 3, 1, 1), ("relu",),
        ("maxpool", 2, 2), ("flatten",), ("fc", 512), ("relu",), ("fc", 10)]},
    "RESNET18": {"input": (3, 32, 32), "ops": [
        ("conv", 64, 3, 1, 1), ("relu",),
        ("res", 64, 1), ("res", 64, 1), ("res", 128, 2), ("res", 128, 1),
        ("res", 256, 2), ("res", 256, 1), ("res", 512, 2), ("res", 512, 1),
        ("sumpool", 4), ("flatten",), ("fc", 10)]},
}

ALIASES = {"MINIONN": "MODEL_F_MINIONN_POOL_REPL", "GNNP": "MODEL_F_GNNP_POOL_REPL", "MLP": "MODEL_A",
           "MNIST_MLP": "MODEL_A", "LENET": "LENET5", "VGG": "VGG16", "RESNET": "RESNET18"}


@dataclass
class ModelConfig:
    name: str
    q_method: QuantizationMethod = QuantizationMethod.ScaleQuant
    q_parameter: int = 5
    q_const: float = 0.02
    seed: int = 0
    width_mult: float = 1.0


def canonical(name: str) -> str:
    n = name.upper()
    return ALIASES.get(n, n)


def _init(rng, shape, fan_in):
    bound = 1.0 / np.sqrt(fan_in)
    return rng.uniform(-bound, bound, size=shape).astype(np.float32)


def build_circuit(name: str, q_method: QuantizationMethod = QuantizationMethod.ScaleQuant, q_parameter: int = 5,
                  q_const: float = 0.02, seed: int = 0, weights: Optional[dict] = None) -> Circuit:
    """Random-init (or given float weights) circuit with Dash quantization."""
    arch = ARCHS[canonical(name)]
    rng = np.random.default_rng(seed)
    C, H, W = arch["input"]
    dims = (C, H, W)
    layers = []
    qm = QuantizationMethod(q_method)

    def rescale_after(d):
        if qm == QuantizationMethod.ScaleQuant:
            layers.append(Rescale(q_parameter, d))
        elif qm == QuantizationMethod.ScaleQuantPlus:
            layers.append(Rescale([q_parameter], d))

    def conv(cout, k, s, p, cin, h, w):
        wt = _init(rng, (cout, cin, k, k), cin * k * k)
        bs = _init(rng, (cout,), cin * k * k)
        c = Conv2d(wt, bs, w, h, cin, cout, k, k, s, s, q_parameter, qm, q_const, pad_width=p, pad_height=p)
        layers.append(c)
        rescale_after(c.out_dims)
        return c.out_dims

    for op in arch["ops"]:
        kind = op[0]
        if kind == "flatten":
            layers.append(Flatten(dims))
            dims = (int(np.prod(dims)),)
        elif kind == "fc":
            fin = int(np.prod(dims))
            wt = _init(rng, (op[1], fin), fin)
            bs = _init(rng, (op[1],), fin)
            d = Dense(wt, bs, q_parameter, qm, q_const)
            layers.append(d)
            dims = d.out_dims
            rescale_after(dims)
        elif kind == "conv":
            _, cout, k, s, p = op
            dims = conv(cout, k, s, p, dims[0], dims[1], dims[2])
        elif kind == "relu":
            layers.append(Relu(dims))
        elif kind == "sign":
            layers.append(Sign(dims))
        elif kind == "maxpool":
            _, k, s = op
            mp = MaxPool2d(dims[2], dims[1], dims[0], k, k, s, s)
            layers.append(mp)
            dims = mp.out_dims
        elif kind == "sumpool":
            sp = SumPool2d(dims[2], dims[1], dims[0], op[1], op[1])
            layers.append(sp)
            dims = sp.out_dims
        elif kind == "res":
            _, cout, stride = op
            cin = dims[0]
            src = len(layers) - 1  # index of the layer whose output feeds the block
            d1 = conv(cout, 3, stride, 1, cin, dims[1], dims[2])
            layers.append(Relu(d1))
            d2 = conv(cout, 3, 1, 1, cout, d1[1], d1[2])
            if stride != 1 or cin != cout:
                # projection shortcut: 1x1 conv reading the block input (in_src), then add the main path
                main_last = len(layers) - 1
                sc = len(layers)
                conv(cout, 1, stride, 0, cin, dims[1], dims[2])
                layers[sc].in_src = src
                layers.append(Add(d2, main_last))
            else:
                layers.append(Add(d2, src))
            layers.append(Relu(d2))
            dims = d2
        else:
            raise ValueError(f"unknown op {kind}")
    return Circuit(layers, q_parameter)


def input_dims(name: str):
    return ARCHS[canonical(name)]["input"]


def synthetic_inputs(name: str, n: int, seed: int = 1) -> list[np.ndarray]:
    """CIFAR/MNIST-shaped normalized synthetic images (no dataset download)."""
    rng = np.random.default_rng(seed)
    C, H, W = input_dims(name)
    return [np.clip(rng.standard_normal(C * H * W), -2.5, 2.5).astype(np.float32) for _ in range(n)]


def quantized_inputs(name: str, n: int, q_method=QuantizationMethod.ScaleQuant, q_parameter: int = 5,
                     q_const: float = 0.02, seed: int = 1) -> list[np.ndarray]:
    return [quantize_input(x, QuantizationMethod(q_method), q_parameter, q_const) for x in synthetic_inputs(name, n, seed)]


# Benchmark configurations (benchmarks/model_benchmarks/non_sgx/main.cpp:227-335)
BENCH_CONFIGS = {
    "MODEL_F_MINIONN_POOL_REPL/DASH": dict(model="MODEL_F_MINIONN_POOL_REPL", q_method=QuantizationMethod.ScaleQuant,
                                          q_parameter=5, crt=7, mrs=100.0),
    "MODEL_F_GNNP_POOL_REPL/DASH": dict(model="MODEL_F_GNNP_POOL_REPL", q_method=QuantizationMethod.ScaleQuant,
                                       q_parameter=5, crt=7, mrs=100.0),
    "MODEL_F_MINIONN_POOL_REPL/REDASH_OPT": dict(model="MODEL_F_MINIONN_POOL_REPL",
                                                q_method=QuantizationMethod.ScaleQuantPlus, q_parameter=32,
                                                crt=[32, 97, 107], mrs=[22, 19, 15, 13]),
    "MODEL_F_GNNP_POOL_REPL/REDASH_OPT": dict(model="MODEL_F_GNNP_POOL_REPL",
                                             q_method=QuantizationMethod.ScaleQuantPlus, q_parameter=32,
                                             crt=[32, 167, 173], mrs=[26, 25, 21, 13]),
    "MODEL_F_MINIONN_POOL_REPL/REDASH_CPM": dict(model="MODEL_F_MINIONN_POOL_REPL",
                                                q_method=QuantizationMethod.ScaleQuantPlus, q_parameter=32,
                                                crt=[32, 3, 5, 7, 11, 13, 17], mrs=[10, 9, 9, 8, 7, 7, 6]),
    "MODEL_A/SIMPLE": dict(model="MODEL_A", q_method=QuantizationMethod.SimpleQuant, q_parameter=-1, crt=8, mrs=100.0),
}
