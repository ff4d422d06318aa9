"""Training pipeline for the model zoo (reference: models/train_pytorch.ipynb, C48).

Builds a PyTorch `nn.Sequential` from a zoo architecture, trains it (optionally
with the reference's fake quantization: x -> round(x / c) * c with a
straight-through gradient, notebook cell 7), converts the trained network to
a float `Circuit` with the requested Dash quantization and exports ONNX
through the built-in writer (the notebook used torch.onnx.export; the onnx
package is not available on the target image).

Data: `--data-dir` with the MNIST / CIFAR-10 files, otherwise a synthetic
stand-in with the same shapes (useful to exercise the pipeline offline).

    python -m dash_amd.models.train --model MODEL_A --epochs 2 --out MODEL_A.onnx
"""
from __future__ import annotations

import argparse
from typing import Optional

import numpy as np

from ..ir.circuit import Circuit
from ..ir.layers import Conv2d, Dense, Flatten, MaxPool2d, Relu, Rescale, Sign, SumPool2d
from ..ir.quant import QuantizationMethod
from .zoo import ARCHS, canonical


def _torch():
    import torch
    import torch.nn as nn

    return torch, nn


class _FakeQuant:
    """round(x / c) * c with an identity gradient (straight-through)."""

    def __init__(self, c: float):
        self.c = c

    def __call__(self, x):
        if not self.c:
            return x
        return x + (x / self.c).round().mul(self.c).sub(x).detach()


def build_torch_model(name: str, fake_quant: float = 0.0):
    torch, nn = _torch()
    arch = ARCHS[canonical(name)]
    C, H, W = arch["input"]
    dims = [C, H, W]
    mods = []
    fq = _FakeQuant(fake_quant)

    class FQLinear(nn.Linear):
        def forward(self, x):
            return nn.functional.linear(fq(x), fq(self.weight), fq(self.bias))

    class FQConv(nn.Conv2d):
        def forward(self, x):
            return self._conv_forward(fq(x), fq(self.weight), fq(self.bias))

    for op in arch["ops"]:
        k = op[0]
        if k == "flatten":
            mods.append(nn.Flatten())
            dims = [int(np.prod(dims))]
        elif k == "fc":
            mods.append(FQLinear(int(np.prod(dims)), op[1]))
            dims = [op[1]]
        elif k == "conv":
            _, cout, ks, s, p = op
            mods.append(FQConv(dims[0], cout, ks, stride=s, padding=p))
            dims = [cout, (dims[1] + 2 * p - ks) // s + 1, (dims[2] + 2 * p - ks) // s + 1]
        elif k == "relu":
            mods.append(nn.ReLU())
        elif k == "sign":
            mods.append(nn.Tanh())  # trained as tanh, garbled as sign (onnx_modelloader.h Tanh -> Sign)
        elif k == "maxpool":
            mods.append(nn.MaxPool2d(op[1], op[2]))
            dims = [dims[0], (dims[1] - op[1]) // op[2] + 1, (dims[2] - op[1]) // op[2] + 1]
        elif k == "sumpool":
            mods.append(nn.AvgPool2d(op[1]))
            dims = [dims[0], dims[1] // op[1], dims[2] // op[1]]
        else:
            raise NotImplementedError(f"training: op {k} (residual blocks) not supported by the sequential trainer")
    seq = nn.Sequential(*mods)
    seq.fq = fq  # set seq.fq.c = 0 to evaluate the float network
    return seq


def to_circuit(model, name: str, q_method=QuantizationMethod.ScaleQuant, q_parameter: int = 5,
               q_const: float = 0.02) -> Circuit:
    """Convert a trained sequential model to a Dash circuit (float weights, quantized per q_method)."""
    torch, nn = _torch()
    arch = ARCHS[canonical(name)]
    C, H, W = arch["input"]
    dims = (C, H, W)
    qm = QuantizationMethod(q_method)
    layers = []

    def rescale(d):
        if qm == QuantizationMethod.ScaleQuant:
            layers.append(Rescale(q_parameter, d))
        elif qm == QuantizationMethod.ScaleQuantPlus:
            layers.append(Rescale([q_parameter], d))

    for m in model:
        if isinstance(m, nn.Flatten):
            layers.append(Flatten(dims))
            dims = (int(np.prod(dims)),)
        elif isinstance(m, nn.Linear):
            d = Dense(m.weight.detach().cpu().numpy(), m.bias.detach().cpu().numpy(), q_parameter, qm, q_const)
            layers.append(d)
            dims = d.out_dims
            rescale(dims)
        elif isinstance(m, nn.Conv2d):
            w = m.weight.detach().cpu().numpy()
            F, Cin, kh, kw = w.shape
            c = Conv2d(w, m.bias.detach().cpu().numpy(), dims[2], dims[1], Cin, F, kw, kh, m.stride[1], m.stride[0],
                       q_parameter, qm, q_const, pad_width=m.padding[1], pad_height=m.padding[0])
            layers.append(c)
            dims = c.out_dims
            rescale(dims)
        elif isinstance(m, nn.ReLU):
            layers.append(Relu(dims))
        elif isinstance(m, nn.Tanh):
            layers.append(Sign(dims))
        elif isinstance(m, nn.MaxPool2d):
            k, s = int(m.kernel_size), int(m.stride)
            mp = MaxPool2d(dims[2], dims[1], dims[0], k, k, s, s)
            layers.append(mp)
            dims = mp.out_dims
        elif isinstance(m, nn.AvgPool2d):
            k = int(m.kernel_size)
            sp = SumPool2d(dims[2], dims[1], dims[0], k, k)
            layers.append(sp)
            dims = sp.out_dims
        elif isinstance(m, nn.Dropout):
            continue
    return Circuit(layers, q_parameter)


def train(name: str, epochs: int = 1, data_dir: Optional[str] = None, fake_quant: float = 0.0, lr: float = 1e-3,
          batch_size: int = 128, n_synthetic: int = 2048, seed: int = 0, device: Optional[str] = None,
          log=print):
    torch, nn = _torch()
    torch.manual_seed(seed)
    arch = ARCHS[canonical(name)]
    shape = arch["input"]
    if data_dir:
        from .. import data

        ds = data.load("mnist" if shape[0] == 1 else "cifar10", data_dir)
        xtr, ytr = ds.train_images, ds.train_labels
        xte, yte = ds.test_images, ds.test_labels
    else:
        rng = np.random.default_rng(seed)
        # synthetic, learnable: the label is the argmax of a fixed random projection
        proj = rng.standard_normal((int(np.prod(shape)), 10)).astype(np.float32)
        xtr = rng.standard_normal((n_synthetic, *shape)).astype(np.float32)
        ytr = np.argmax(xtr.reshape(len(xtr), -1) @ proj, axis=1)
        xte = rng.standard_normal((n_synthetic // 4, *shape)).astype(np.float32)
        yte = np.argmax(xte.reshape(len(xte), -1) @ proj, axis=1)
    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    model = build_torch_model(name, fake_quant).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    lossf = nn.CrossEntropyLoss()
    Xtr, Ytr = torch.from_numpy(np.asarray(xtr)), torch.from_numpy(np.asarray(ytr, np.int64))
    for ep in range(epochs):
        model.train()
        perm = torch.randperm(len(Xtr))
        tot = 0.0
        for s in range(0, len(Xtr), batch_size):
            idx = perm[s:s + batch_size]
            xb, yb = Xtr[idx].to(dev), Ytr[idx].to(dev)
            opt.zero_grad()
            loss = lossf(model(xb), yb)
            loss.backward()
            opt.step()
            tot += float(loss.detach()) * len(idx)
        acc = evaluate(model, xte, yte, dev)
        log(f"epoch {ep + 1}/{epochs}: loss {tot / len(Xtr):.4f}  test acc {acc:.4f}")
    return model.cpu(), (xte, yte)


def evaluate(model, x, y, dev=None) -> float:
    torch, _ = _torch()
    model.eval()
    with torch.no_grad():
        xt = torch.from_numpy(np.asarray(x))
        if dev is not None:
            xt = xt.to(dev)
        pred = model(xt).argmax(1).cpu().numpy()
    return float(np.mean(pred == np.asarray(y)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="MODEL_A")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--fake-quant", type=float, default=0.0)
    ap.add_argument("--out", default=None, help="ONNX output path")
    args = ap.parse_args()
    model, _ = train(args.model, args.epochs, args.data_dir, args.fake_quant)
    if args.out:
        from ..ir.onnx import save_onnx_model

        save_onnx_model(args.out, to_circuit(model, args.model, QuantizationMethod.SimpleQuant, -1),
                        producer="pytorch")
        print("wrote", args.out)


if __name__ == "__main__":
    main()
