"""Garbled-table layouts of the reference <-> this framework's.

The framework stores a sign gadget's approximate-residue table fan-out-major:
the t digit entries of one (residue, color) are adjacent (``t*prefix_j + color*t + d``,
one contiguous read per residue on the GPU). The reference stores it digit-major,
``#mrs*prefix_i + d*p_i + c`` (sign_gadget.h:295-316 allocation, :61-75 kernel
indexing). Every other table of the reference sign / ReLU / legacy-rescale
gadgets already has the reference order:

* cast-1  ``(k+1)*sum(mrs[1:])`` per element, digits t-1..1, k residue casts then the carry
  (sign_gadget.h:443, :486-515);
* cast-2  per digit ``(k+1)*m_d`` entries (sign_gadget.h:444, :527-529);
* sign    ``o*m_0 + c`` (sign_gadget.h:445, :555-568);
* ReLU half gates ``G[in*sum(p) + prefix_j + c]``, ``E[in*k*3 + j*3 + c]`` (garbled_relu.h:155-160);
* legacy rescale trans ``in*(k-1)*2 + (j-1)*2 + c`` (the CUDA reader's order, cuda_util.h:426-428).

Only the reference's own construction has a reference layout: models garbled
with the fused sign gadget (no cast-1 table) or the mixed-radix constructions
raise. ``export_reference`` returns copies; ``import_reference`` writes
reference-layout tables back into a model's arrays (host copies).
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

from ..ir.layers import Kind

SIGN_FAMILY = ("s.approx", "s.cast1", "s.cast2", "s.sign", "mm.g", "mm.e", "trans")


def _approx_blocks(crt, t):
    pre = 0
    for p in crt:
        yield pre, int(p)
        pre += int(p)


def approx_to_reference(a: np.ndarray, crt, t: int) -> np.ndarray:
    """[N, t*sum(p), 2] fan-out-major (color*t + d) -> digit-major (d*p + color) per residue block."""
    out = np.empty_like(a)
    N = a.shape[0]
    for pre, p in _approx_blocks(crt, t):
        blk = a[:, t * pre:t * (pre + p)].reshape(N, p, t, 2)
        out[:, t * pre:t * (pre + p)] = blk.transpose(0, 2, 1, 3).reshape(N, t * p, 2)
    return out


def approx_from_reference(a: np.ndarray, crt, t: int) -> np.ndarray:
    out = np.empty_like(a)
    N = a.shape[0]
    for pre, p in _approx_blocks(crt, t):
        blk = a[:, t * pre:t * (pre + p)].reshape(N, t, p, 2)
        out[:, t * pre:t * (pre + p)] = blk.transpose(0, 2, 1, 3).reshape(N, t * p, 2)
    return out


def _tables(model):
    if model.sign_fused:
        raise ValueError("the fused sign construction has no reference layout (the reference casts explicitly); "
                         "garble with fused_sign=False")
    for li in range(model.num_layers):
        kind = model.layer_kind(li)
        if kind not in (Kind.RELU, Kind.SIGN, Kind.RESCALE):
            continue
        params = model.layer_params(li)
        if kind == Kind.RESCALE and params.get("mode", [0])[0] == 2 or kind == Kind.RELU and "smode" in params:
            raise ValueError(f"layer {li} uses a mixed-radix construction, which has no reference layout")
        for name, arr in model.layer_arrays(li).items():
            if name.split(".", 1)[-1] in SIGN_FAMILY or name in SIGN_FAMILY:
                yield li, name, arr


def export_reference(model) -> Dict[Tuple[int, str], np.ndarray]:
    """{(layer, table): uint64 [N, entries, 2]} in the reference's layouts (copies)."""
    crt, t = list(model.crt), len(model.mrs)
    out = {}
    for li, name, arr in _tables(model):
        out[(li, name)] = approx_to_reference(arr, crt, t) if name.endswith("s.approx") else np.array(arr, copy=True)
    return out


def import_reference(model, tables: Dict[Tuple[int, str], np.ndarray]) -> None:
    """Write reference-layout tables (export_reference's form) into the model's arrays."""
    crt, t = list(model.crt), len(model.mrs)
    for li, name, arr in _tables(model):
        src = tables[(li, name)]
        if src.shape != arr.shape:
            raise ValueError(f"table ({li}, {name}) has shape {src.shape}, the model expects {arr.shape}")
        arr[...] = approx_from_reference(src, crt, t) if name.endswith("s.approx") else src
