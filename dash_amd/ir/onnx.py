"""ONNX model import/export.

`load_onnx_model(path, q_method, q_parameter)` mirrors the reference loader
(circuit/onnx_modelloader.h:156-406): Flatten / Reshape(flatten), Gemm, Conv,
MaxPool, Relu, Tanh|SignTanh -> Sign, with a Rescale inserted after every
Gemm/Conv for ScaleQuant (legacy `l` halvings) and ScaleQuantPlus (one ReDash
factor), q_const = 0.02 for SimpleQuant. Differences (deliberate):

* the protobuf is decoded by the native wire-format reader (csrc/onnx.cpp), no
  libprotobuf;
* attributes are looked up by name and initializers by the node's input
  names, not by position (the reference's positional access, :280-295, is
  exporter-specific);
* Conv `pads` (symmetric) are honoured, Gemm `transB`/`alpha`/`beta`,
  MatMul+Add, BatchNormalization folding into the preceding Conv/Gemm,
  residual Add of two activations, Identity/Dropout are accepted.

`save_onnx_model(path, circuit)` writes a pytorch-style ONNX graph of a float
circuit with a small protobuf encoder (the python `onnx` package is not
available on the target image), so that models built or trained here can be
exchanged with other tools and re-imported.
"""
from __future__ import annotations

import struct
from pathlib import Path
from typing import Optional

import numpy as np

from ..native import native
from .circuit import Circuit
from .layers import Add, Conv2d, Dense, Flatten, MaxPool2d, Relu, Rescale, Sign
from .quant import QuantizationMethod

DEFAULT_Q_CONST = 0.02  # onnx_modelloader.h:377


def parse_onnx(path_or_bytes) -> dict:
    """Decoded ModelProto as plain python (nodes, initializers, inputs, outputs)."""
    if isinstance(path_or_bytes, (bytes, bytearray)):
        blob = bytes(path_or_bytes)
    else:
        blob = Path(path_or_bytes).read_bytes()
    return native().onnx_parse(blob)


def _input_dims(model: dict, init_names: set) -> tuple:
    inputs = [i for i in model["inputs"] if i["name"] not in init_names]
    assert inputs, "onnx: graph has no data input"
    d = [int(v) for v in inputs[0]["dims"]]
    tf = model["producer_name"] == "tf2onnx"
    if tf and len(d) == 4:  # NHWC
        return (d[3], d[1], d[2])
    if tf and len(d) == 3:
        return (d[0], d[1], d[2])
    if len(d) == 4:  # NCHW
        return (d[1], d[2], d[3])
    if len(d) == 3:
        return (d[0], d[1], d[2])
    if len(d) == 2:
        return (d[1],)
    return (d[0],)


class _Spec:
    """A float layer awaiting quantization (BatchNorm may still fold into it)."""

    def __init__(self, kind: str, **kw):
        self.kind = kind
        self.kw = kw


def create_circuit_from_onnx(model: dict, q_method: QuantizationMethod = QuantizationMethod.SimpleQuant,
                             q_const: float = DEFAULT_Q_CONST, q_parameter: int = -1) -> Circuit:
    q_method = QuantizationMethod(q_method)
    inits = {t["name"]: t for t in model["initializers"]}
    tf = model["producer_name"] == "tf2onnx"

    def arr(name: str) -> np.ndarray:
        t = inits[name]
        return np.asarray(t["values"], dtype=np.float32).reshape([int(v) for v in t["dims"]] or [-1])

    dims = _input_dims(model, set(inits))
    specs: list[_Spec] = []
    producer: dict[str, int] = {}  # tensor name -> index of the spec producing it (-1 = graph input)
    data_inputs = [i["name"] for i in model["inputs"] if i["name"] not in inits]
    producer[data_inputs[0]] = -1
    alias: dict[str, str] = {}
    first_dense = True
    last_conv_filters = 0
    nodes = model["nodes"]
    skip = set()

    def src_of(name: str) -> Optional[int]:
        name = alias.get(name, name)
        return producer.get(name)

    def emit(spec: _Spec, out_name: str):
        specs.append(spec)
        producer[out_name] = len(specs) - 1

    for ni, node in enumerate(nodes):
        if ni in skip:
            continue
        op, a = node["op_type"], node["attrs"]
        ins, outs = node["inputs"], node["outputs"]
        if op in ("Identity", "Dropout"):
            alias[outs[0]] = alias.get(ins[0], ins[0])
            continue
        if op == "Flatten" or op == "Reshape":
            if op == "Reshape" and len(dims) == 1:
                alias[outs[0]] = alias.get(ins[0], ins[0])
                continue
            emit(_Spec("flatten", dims=dims), outs[0])
            dims = (int(np.prod(dims)),)
        elif op in ("Gemm", "MatMul"):
            w = arr(ins[1])
            trans_b = int(a.get("transB", 0)) if op == "Gemm" else 0
            if not trans_b:
                w = w.T  # [in][out] -> [out][in]
            w = w * float(a.get("alpha", 1.0))
            bias = np.zeros(w.shape[0], np.float32)
            if op == "Gemm" and len(ins) > 2 and ins[2]:
                bias = arr(ins[2]).reshape(-1) * float(a.get("beta", 1.0))
            out_name = outs[0]
            if op == "MatMul" and ni + 1 < len(nodes):
                nxt = nodes[ni + 1]
                other = [x for x in nxt["inputs"] if x != out_name]
                if nxt["op_type"] == "Add" and out_name in nxt["inputs"] and other and other[0] in inits:
                    bias = arr(other[0]).reshape(-1)
                    out_name = nxt["outputs"][0]
                    skip.add(ni + 1)
            channel_tf = 0
            if tf and first_dense and last_conv_filters > 0:
                channel_tf = last_conv_filters
            first_dense = False
            emit(_Spec("dense", w=w, b=bias, channel_tf=channel_tf), out_name)
            dims = (w.shape[0],)
        elif op == "Conv":
            w = arr(ins[1])
            F, C, kh, kw = (int(v) for v in w.shape)
            assert int(a.get("group", 1)) == 1, "onnx: grouped convolutions are not supported"
            assert all(int(v) == 1 for v in a.get("dilations", [1, 1])), "onnx: dilated convolutions are not supported"
            st = [int(v) for v in a.get("strides", [1, 1])]
            pads = [int(v) for v in a.get("pads", [0, 0, 0, 0])]
            assert pads[0] == pads[2] and pads[1] == pads[3], "onnx: only symmetric padding is supported"
            bias = arr(ins[2]).reshape(-1) if len(ins) > 2 and ins[2] else np.zeros(F, np.float32)
            assert len(dims) == 3 and dims[0] == C, f"onnx: conv expects {C} input channels, got dims {dims}"
            emit(_Spec("conv", w=w, b=bias, dims=dims, stride=st, pads=(pads[0], pads[1])), outs[0])
            H = (dims[1] + 2 * pads[0] - kh) // st[0] + 1
            W = (dims[2] + 2 * pads[1] - kw) // st[1] + 1
            dims = (F, H, W)
            last_conv_filters = F
        elif op == "BatchNormalization":
            j = src_of(ins[0])
            assert j is not None and j >= 0 and specs[j].kind in ("conv", "dense"), \
                "onnx: BatchNormalization must follow a Conv or Gemm"
            scale, shift, mean, var = (arr(n).reshape(-1) for n in ins[1:5])
            eps = float(a.get("epsilon", 1e-5))
            g = scale / np.sqrt(var + eps)
            s = specs[j]
            s.kw["w"] = s.kw["w"] * g.reshape((-1,) + (1,) * (s.kw["w"].ndim - 1))
            s.kw["b"] = (s.kw["b"] - mean) * g + shift
            producer[outs[0]] = j
        elif op == "MaxPool":
            k = [int(v) for v in a["kernel_shape"]]
            st = [int(v) for v in a.get("strides", [1, 1])]
            emit(_Spec("maxpool", dims=dims, k=k, stride=st), outs[0])
            dims = (dims[0], (dims[1] - k[0]) // st[0] + 1, (dims[2] - k[1]) // st[1] + 1)
        elif op == "Relu":
            emit(_Spec("relu", dims=dims), outs[0])
        elif op in ("Tanh", "SignTanh", "Sign"):
            emit(_Spec("sign", dims=dims), outs[0])
        elif op == "Add":
            srcs = [src_of(x) for x in ins]
            if any(x in inits for x in ins):
                raise NotImplementedError("onnx: Add of a constant is only supported directly after MatMul")
            assert None not in srcs, "onnx: Add operand produced by an unsupported node"
            prev = len(specs) - 1
            other = srcs[0] if srcs[1] == prev else srcs[1]
            emit(_Spec("add", dims=dims, src=other), outs[0])
        else:
            raise NotImplementedError(f"onnx: unsupported operator {op}")

    # materialize: quantize weights, insert rescales, remap spec indices -> layer indices
    layers = []
    spec_to_layer: dict[int, int] = {-1: -1}
    for i, s in enumerate(specs):
        kw = s.kw
        if s.kind == "flatten":
            layers.append(Flatten(kw["dims"]))
        elif s.kind == "dense":
            layers.append(Dense(kw["w"], kw["b"], q_parameter, q_method, q_const, channel_tf=kw["channel_tf"]))
        elif s.kind == "conv":
            C, H, W = kw["dims"]
            F, _, kh, kw_ = kw["w"].shape
            layers.append(Conv2d(kw["w"], kw["b"], W, H, C, F, kw_, kh, kw["stride"][1], kw["stride"][0],
                                 q_parameter, q_method, q_const, pad_width=kw["pads"][1], pad_height=kw["pads"][0]))
        elif s.kind == "maxpool":
            C, H, W = kw["dims"]
            layers.append(MaxPool2d(W, H, C, kw["k"][1], kw["k"][0], kw["stride"][1], kw["stride"][0]))
        elif s.kind == "relu":
            layers.append(Relu(kw["dims"]))
        elif s.kind == "sign":
            layers.append(Sign(kw["dims"]))
        elif s.kind == "add":
            layers.append(Add(kw["dims"], spec_to_layer[kw["src"]]))
        spec_to_layer[i] = len(layers) - 1
        if s.kind in ("dense", "conv"):
            out = layers[-1].out_dims
            if q_method == QuantizationMethod.ScaleQuant:
                layers.append(Rescale(q_parameter, out))
                spec_to_layer[i] = len(layers) - 1
            elif q_method == QuantizationMethod.ScaleQuantPlus:
                layers.append(Rescale([q_parameter], out))
                spec_to_layer[i] = len(layers) - 1
    return Circuit(layers, q_parameter)


def load_onnx_model(path, q_method: QuantizationMethod = QuantizationMethod.SimpleQuant, q_parameter: int = -1,
                    q_const: float = DEFAULT_Q_CONST) -> Circuit:
    """Reference: load_onnx_model (onnx_modelloader.h:371-406)."""
    return create_circuit_from_onnx(parse_onnx(path), q_method, q_const, q_parameter)


# ------------------------------------------------------------------ export
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _ld(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _s(field: int, s: str) -> bytes:
    return _ld(field, s.encode())


def _i(field: int, v: int) -> bytes:
    return _key(field, 0) + _varint(v)


def _tensor(name: str, a: np.ndarray) -> bytes:
    a = np.ascontiguousarray(a, dtype=np.float32)
    body = b"".join(_i(1, d) for d in a.shape) + _i(2, 1) + _s(8, name) + _ld(9, a.tobytes())
    return body


def _attr_ints(name: str, vals) -> bytes:
    return _ld(5, _s(1, name) + b"".join(_i(8, int(v)) for v in vals) + _i(20, 7))


def _attr_int(name: str, v: int) -> bytes:
    return _ld(5, _s(1, name) + _i(3, int(v)) + _i(20, 2))


def _attr_float(name: str, v: float) -> bytes:
    return _ld(5, _s(1, name) + _key(2, 5) + struct.pack("<f", v) + _i(20, 1))


def _node(op: str, ins, outs, name: str, attrs: bytes = b"") -> bytes:
    return _ld(1, b"".join(_s(1, x) for x in ins) + b"".join(_s(2, x) for x in outs) + _s(3, name) + _s(4, op) + attrs)


def _value_info(name: str, dims) -> bytes:
    shape = b"".join(_ld(1, _i(1, int(d))) for d in dims)
    # ValueInfoProto{name, type: TypeProto{tensor_type: {elem_type FLOAT, shape}}}
    return _s(1, name) + _ld(2, _ld(1, _i(1, 1) + _ld(2, shape)))


def save_onnx_model(path, circuit: Circuit, producer: str = "dash_amd") -> None:
    """Write the float weights of `circuit` as an ONNX (opset 13) graph in the
    layout pytorch's exporter uses (NCHW input, Gemm with transB=1). Rescale
    layers are quantization artefacts and are dropped; loading the file back
    with the same q_method re-inserts them."""
    nodes, inits = [], []
    cur = "input"
    in_dims = circuit.input_dims
    for i, l in enumerate(circuit.layers):
        out = f"t{i}"
        name = f"{l.name}_{i}"
        if isinstance(l, Rescale):
            continue
        if isinstance(l, Flatten):
            nodes.append(_node("Flatten", [cur], [out], name, _attr_int("axis", 1)))
        elif isinstance(l, Dense):
            assert l.channel_tf == 0, "onnx export: TF channel order is not representable"
            inits += [_tensor(f"{name}.weight", l.weights), _tensor(f"{name}.bias", l.biases)]
            nodes.append(_node("Gemm", [cur, f"{name}.weight", f"{name}.bias"], [out], name,
                               _attr_float("alpha", 1.0) + _attr_float("beta", 1.0) + _attr_int("transB", 1)))
        elif isinstance(l, Conv2d):
            inits += [_tensor(f"{name}.weight", l.weights), _tensor(f"{name}.bias", l.biases)]
            attrs = (_attr_ints("dilations", [1, 1]) + _attr_int("group", 1) + _attr_ints("kernel_shape", [l.kh, l.kw])
                     + _attr_ints("pads", [l.ph, l.pw, l.ph, l.pw]) + _attr_ints("strides", [l.sh, l.sw]))
            nodes.append(_node("Conv", [cur, f"{name}.weight", f"{name}.bias"], [out], name, attrs))
        elif isinstance(l, MaxPool2d):
            attrs = _attr_ints("kernel_shape", [l.kh, l.kw]) + _attr_ints("pads", [0, 0, 0, 0]) + \
                _attr_ints("strides", [l.sh, l.sw])
            nodes.append(_node("MaxPool", [cur], [out], name, attrs))
        elif isinstance(l, Relu):
            nodes.append(_node("Relu", [cur], [out], name))
        elif isinstance(l, Sign):
            nodes.append(_node("Sign", [cur], [out], name))
        else:
            raise NotImplementedError(f"onnx export: layer {l.name} has no ONNX equivalent")
        cur = out
    dims = (1,) + tuple(in_dims)
    graph = b"".join(nodes) + _s(2, "dash_amd") + b"".join(_ld(5, t) for t in inits)
    graph += _ld(11, _value_info("input", dims))
    graph += _ld(12, _value_info(cur, (1,) + tuple(circuit.output_dims)))
    model = _i(1, 7) + _s(2, producer) + _s(3, "1") + _ld(7, graph) + _ld(8, _s(1, "") + _i(2, 13))
    Path(path).write_bytes(model)
