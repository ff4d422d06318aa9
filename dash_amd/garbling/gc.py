"""High-level garbled-circuit API.

`GarbledCircuit` mirrors the reference's public entry points
(garbling/garbled_circuit.h:43-109 constructors; garbled_circuit_interface.h:
garble_inputs :325-343, cpu_evaluate :345-380, decode_outputs :422-467,
cuda_move/cuda_evaluate/cuda_move_outputs :477-736) on top of the split
garbler / evaluator roles:

    garbler  = native.Garbler   (secrets: R_p, input base labels, decoder)
    model    = native.GarbledModel  (offline message, serializable)
    evaluator = cpu_evaluate / dash_amd.runtime.HipEvaluator
"""
from __future__ import annotations

import os
import time
import warnings
from typing import Optional, Sequence, Union

import numpy as np

from ..ir.bases import crt_modulus as _crt_mod
from ..ir.bases import first_primes, get_mrs_base
from ..ir.circuit import Circuit
from ..native import native

Labels = list  # list[(modulus, np.ndarray int16 [N, n_p])]


class ReferenceEncodingWarning(UserWarning):
    """hardened=None resolved to the reference (wire-compatible, R_p-leaking) encoding."""


def mrs_capable(crt_base: Sequence[int]) -> bool:
    """The mixed-radix rescale / sign constructions need residue 0 = 2 and odd other residues."""
    return len(crt_base) >= 2 and int(crt_base[0]) == 2 and all(int(p) % 2 == 1 for p in crt_base[1:])


def resolve_constructions(circuit: Circuit, crt_base: Sequence[int], rescale: str, relu: str,
                          fused_sign: bool = True, hardened: Optional[bool] = None):
    """Resolve "auto" gadget constructions and guard the mixed-radix rescale's range.

    The mixed-radix constructions exist only in the hardened encoding, which needs the fused sign: with
    fused_sign=False or hardened=False, "auto" resolves to the reference constructions ("legacy" /
    "approx") instead of picking a construction the requested encoding cannot carry.

    rescale="auto" -> "mrs" when the base allows it and the circuit was calibrated
    (Circuit.calibrate: every DASH rescale has a tracked input range) with every
    tracked input at least one further 2^l band below the wrap band
    (Circuit.mrs_rescale_violations(headroom=True)); otherwise "legacy", the
    reference's construction, exact on the whole signed range. "auto" therefore
    depends on how well the calibration samples cover the inputs served later:
    an input beyond the calibrated range by more than 2^l that lands in the
    band (< 2^l values just below M/2, i.e. next to a CRT overflow) would wrap.
    An explicit "mrs" on a circuit whose tracked range enters the band raises.
    relu="auto" -> "joint" with the mixed-radix rescale, else "approx"."""
    if rescale not in ("auto", "legacy", "mrs"):
        raise ValueError(f"rescale construction must be 'auto', 'legacy' or 'mrs', got {rescale!r}")
    if relu not in ("auto", "approx", "mrs", "joint"):
        raise ValueError(f"relu construction must be 'auto', 'approx', 'mrs' or 'joint', got {relu!r}")
    M = _crt_mod(crt_base)
    dash_rescales = circuit._dash_rescales()
    bad = circuit.mrs_rescale_violations(M) if dash_rescales else []
    mrs_ok = mrs_capable(crt_base) and bool(fused_sign) and hardened is not False
    if rescale == "auto":
        calibrated = bool(dash_rescales) and all(l.input_tracked for l in dash_rescales)
        tight = circuit.mrs_rescale_violations(M, headroom=True) if dash_rescales else []
        rescale = "mrs" if (mrs_ok and calibrated and not bad and not tight) else "legacy"
    elif rescale == "mrs" and bad:
        i, hi, lim = bad[0]
        raise ValueError(f"rescale='mrs': layer {i}'s tracked input reaches {hi} >= {lim}, inside the mixed-radix "
                         f"wrap band below M/2 = {M // 2}; use rescale='legacy' or a larger CRT base "
                         f"(Circuit.infer_crt_base_size reserves the band)")
    if relu == "auto":
        relu = "joint" if rescale == "mrs" and mrs_ok else "approx"
    return rescale, relu


def hardened_supported(circuit: Circuit, fused_sign: bool, rescale: str) -> bool:
    """The hardened encoding keys no projection with a public label: the reference sign construction's zero
    carry and the legacy rescale's zero residue 0 (fed to a sign gadget) do, so it needs the fused sign and,
    when the circuit has DASH Rescale(l) layers, the mixed-radix rescale."""
    return bool(fused_sign) and (rescale == "mrs" or not circuit._dash_rescales())


class GarbledCircuit:
    def __init__(self, circuit: Circuit, crt: Union[int, Sequence[int]], mrs: Union[None, float, Sequence[int]] = None,
                 max_modulus: int = 0, seed: Optional[bytes] = None, garble_me: bool = True, nthreads: int = 0,
                 device: Optional[int] = None, fused_sign: bool = True, rescale: str = "auto",
                 relu: str = "auto", sink=None, hardened: Optional[bool] = None, range_guard: str = "auto"):
        """fused_sign: sign-gadget construction. True (default): the MRS casts are folded into the approx and
        carry projections (same function, 3.7x fewer gates per sign; gadgets.h SignPlan::fused). False: the
        reference construction with explicit identity casts (sign_gadget.h:456-546).

        rescale: construction of the DASH legacy rescale (divide by 2^l, Rescale(l)). "legacy": l iterations of
        the reference's sign-base-extension gadget (rescale_gadget.h:115-242). "mrs": one exact mixed-radix
        conversion computing the same ceil(x / 2^l) (gadgets.h RescaleMrsPlan; k + 1 hashes per element instead
        of l sign gadgets); it differs only on the top U - M/2 < 2^l values of the signed range, which wrap, so a
        circuit whose tracked range enters that band is refused (resolve_constructions) and
        Circuit.infer_crt_base_size sizes M with the band reserved. "auto" (default, = the benchmark's choice):
        "mrs" where the CRT base and the tracked ranges allow it, else "legacy".

        relu: sign of the ReLU gadget. "approx": the reference's approximate sign gadget (construction per
        fused_sign). "mrs": exact mixed-radix sign with the mod-2 residue converted last (gadgets.h SignMrsPlan;
        k - 1 hashes, 147 instead of 568 table entries per element at k = 7, exact for every x). "joint": a ReLU
        that directly follows a mixed-radix rescale takes its sign from that rescale's conversion (residue 2
        converted last: its digit is the sign; gadgets.h RescaleMrsPlan::sign_last), so it costs only the
        mixed-modulus half gates; other ReLUs use the approximate gadget. Needs rescale="mrs" to have effect.
        "auto" (default): "joint" with the mixed-radix rescale, else "approx".

        sink: with `device`, a HipEvaluator slot destination (HipEvaluator.sink(b)): the GPU garbler writes the
        garbled tables straight into that slot's HBM arena (zero-copy offline phase; HipEvaluator.load(b, model)
        then skips them). The model's tables alias the slot and are valid only while it holds this GC.

        hardened: the offline-message encoding (docs/SECURITY.md). True: no evaluator-visible constant labels
        (public-constant wires have label 0 and their constants are folded into the garbler's base labels) and
        every table entry masked by its own tweaked pad, closing the reference encoding's R_p recovery from
        Z_p / bias labels and its shared-hash leaks (mixed half gate mini tables, repeated MRS digit moduli).
        Needs the fused sign and no legacy rescale. False: the reference's wire-compatible encoding. None
        (default): hardened whenever the resolved constructions allow it.

        range_guard: the garbler's exact per-input range check (garbling/guard.py): "auto" (default) = on when
        the GC has the mixed-radix rescale (an input in its wrap band would decode to a valid but wrong label),
        "on" = always (also catches CRT overflow of the reference constructions), "off". A refused input raises
        RangeGuardError before it is encoded (host paths) or before its result is released (batched paths:
        ``guard.submit`` / ``raise_if_bad``)."""
        self.circuit = circuit
        self.crt_base = first_primes(crt) if isinstance(crt, int) else [int(p) for p in crt]
        if mrs is None:
            self.mrs_base: list[int] = []
        elif isinstance(mrs, (int, float)) and not isinstance(mrs, bool):
            self.mrs_base = get_mrs_base(len(self.crt_base), float(mrs))
        else:
            self.mrs_base = [int(m) for m in mrs]
        self.crt_modulus = _crt_mod(self.crt_base)
        self.seed = seed if seed is not None else os.urandom(16)
        self.nthreads = nthreads
        # device: garble the ReLU / Sign / legacy-rescale layers on this GPU (bit-identical to the CPU garbler)
        self.device = -1 if device is None else int(device)
        self.fused_sign = bool(fused_sign)
        self.rescale, self.relu = resolve_constructions(circuit, self.crt_base, rescale, relu, self.fused_sign,
                                                        hardened)
        supported = hardened_supported(circuit, self.fused_sign, self.rescale)
        # the mixed-radix constructions are this framework's own (not wire-compatible with anything): they only
        # exist in the hardened encoding, whose kernels they use
        needs = self.rescale == "mrs" or self.relu in ("mrs", "joint")
        if hardened is None:
            hardened = supported
            if not supported:
                # the reference encoding ships public-constant labels that reveal R_p (docs/SECURITY.md §1.1):
                # never a silent choice
                warnings.warn("GarbledCircuit: the resolved constructions (sign=%s, rescale=%s) cannot use the "
                              "hardened encoding; falling back to the reference encoding, whose constant labels "
                              "reveal the offsets R_p (docs/SECURITY.md §1.1). Pass hardened=False to choose it "
                              "explicitly." % ("fused" if self.fused_sign else "reference", self.rescale),
                              ReferenceEncodingWarning, stacklevel=2)
        if hardened and not supported:
            raise ValueError("hardened=True needs the fused sign construction and no legacy DASH rescale "
                             "(rescale='mrs'); the reference constructions use the wire-compatible encoding")
        if needs and not hardened:
            raise ValueError("the mixed-radix constructions (rescale='mrs', relu='mrs' / 'joint') use the hardened "
                             "encoding only (fused sign; hardened=None or True)")
        self.hardened = bool(hardened)
        if range_guard == "auto" and os.environ.get("DASH_RANGE_GUARD") in ("on", "off"):
            range_guard = os.environ["DASH_RANGE_GUARD"]  # A/B knob (bench records say which was used)
        if range_guard not in ("auto", "on", "off"):
            raise ValueError("range_guard must be 'auto', 'on' or 'off'")
        self.guard_enabled = range_guard == "on" or (range_guard == "auto" and self.rescale == "mrs"
                                                      and bool(circuit._dash_rescales()))
        self.sink = sink
        self._n = native()
        self.garbler = self._n.Garbler(self.crt_base, self.mrs_base, self.seed, int(max_modulus))
        self.model = None
        self.decoder = None
        self.garbling_time_s = 0.0
        if garble_me:
            self.garble()

    # -------------------------------------------------------------- offline
    def garble(self):
        specs = self.circuit.garble_specs_native()
        t = time.perf_counter()
        self.model = self.garbler.garble(specs, list(self.circuit.input_dims), self.nthreads, self.device,
                                         self.fused_sign, self.rescale == "mrs", self.relu == "mrs",
                                         self.relu == "joint", self.sink if self.device >= 0 else None,
                                         self.hardened)
        self.sink = None  # single use: the slot now holds this GC
        self.garbling_time_s = time.perf_counter() - t
        self.decoder = self.garbler.decoder()
        return self.model

    # --------------------------------------------------------------- online
    @property
    def guard(self):
        """The circuit's exact range guard for this GC's constructions (shared by every GC of the circuit)."""
        from .guard import guard_for

        return guard_for(self.circuit, self.crt_modulus, self.rescale == "mrs",
                         self.device if self.device >= 0 else None)

    def check_inputs(self, xs) -> None:
        """Raise RangeGuardError if a garbled evaluation of any of xs would leave an exact gadget range."""
        if self.guard_enabled:
            self.guard.check(xs)

    def garble_inputs(self, x: np.ndarray) -> Labels:
        x = np.asarray(x, dtype=np.int64).reshape(-1)
        assert x.size == self.circuit.input_size, "input dimension does not match circuit input dimension"
        self.check_inputs([x])
        return self.garbler.encode(x)

    def garble_inputs_cm(self, x: np.ndarray) -> list:
        """Online message #1 in the GPU wire layout: per residue an int16 (n_p, N) array."""
        x = np.asarray(x, dtype=np.int64).reshape(-1)
        assert x.size == self.circuit.input_size, "input dimension does not match circuit input dimension"
        self.check_inputs([x])
        return self.garbler.encode_cm(x)

    def device_input_encoder(self, device: int, slots: int = 1, slot: int = 0):
        """The garbler's input-encoding state (base labels W0, offsets R) of this GC on GPU `device`, placed once
        (offline): ``HipEvaluator.encode_device_into(b, enc, x)`` then writes online message #1 for x straight
        into an evaluator slot on that device (no host label work, only x crosses PCIe). With slots > 1 the
        encoder holds one GC per slot (this one in slot `slot`, the others empty until ``enc.load(gc.garbler,
        s)`` arms slot s with its own GC) and encodes a (slots, N) batch of inputs into consecutive evaluator
        slots with one launch."""
        return self._n.DeviceInputEncoder(self.garbler, int(device), int(slots), int(slot))

    def garble_inputs_compressed(self, x: np.ndarray) -> np.ndarray:
        """Online message #1 in wire form: (k, N, 2) uint64, one 16-B compressed label per residue."""
        x = np.asarray(x, dtype=np.int64).reshape(-1)
        assert x.size == self.circuit.input_size, "input dimension does not match circuit input dimension"
        self.check_inputs([x])
        return self.garbler.encode_compressed(x)

    def decode_compressed(self, labels: np.ndarray) -> np.ndarray:
        """Decode online message #2 in wire form ((k, n_out, 2) uint64)."""
        return np.asarray(self.decoder.decode_compressed(labels), dtype=np.int64)

    def garbling_layer_ms(self) -> list:
        """Per-layer garbling wall time (ms) of the last garble()."""
        return list(self.garbler.layer_ms())

    def cpu_evaluate_timed(self, labels: Labels, nr_threads: int = 0):
        """(output labels, per-layer evaluation ms) — the reference's BENCHMARK timers."""
        out, ms = self._n.cpu_evaluate_timed(self.model, labels, nr_threads)
        return out, list(ms)

    def cpu_evaluate(self, labels: Labels, nr_threads: int = 0) -> Labels:
        return self._n.cpu_evaluate(self.model, labels, nr_threads)

    def decode_outputs(self, labels: Labels) -> np.ndarray:
        return self.decoder.decode(labels)

    # ------------------------------------------------------------------ HIP
    def hip_evaluator(self, **kw):
        from ..runtime import HipEvaluator

        return HipEvaluator([self.model], **kw)

    # -------------------------------------------------------------- helpers
    def effective_constructions(self) -> dict:
        """The gadget constructions this GC actually contains (not the requested ones): the mixed-radix
        rescale applies only to DASH Rescale(l) layers (ReDash Rescale({s}) layers use the base-extension
        gadget), and a joint ReLU only to a ReLU directly after such a rescale (garbler.cpp joint_out)."""
        from ..ir.layers import Kind

        specs = self.circuit.garble_specs()
        dash = [i for i, (k, p) in enumerate(specs) if k == Kind.RESCALE and p.get("mode") == 0]
        redash = [i for i, (k, p) in enumerate(specs) if k == Kind.RESCALE and p.get("mode") == 1]
        relus = [i for i, (k, p) in enumerate(specs) if k == Kind.RELU]
        mrs = self.rescale == "mrs" and bool(dash)
        parts = []
        if dash:
            parts.append("mrs" if mrs else "legacy")
        if redash:
            parts.append("redash-base-extension")
        rescale = "+".join(parts) if parts else "none"
        joint = [i for i in relus if mrs and self.relu == "joint" and i - 1 in dash and "in_src" not in specs[i][1]]
        other = "mrs" if self.relu == "mrs" else "approx"
        if not relus:
            relu = "none"
        elif len(joint) == len(relus):
            relu = "joint"
        elif joint:
            relu = f"joint({len(joint)})+{other}({len(relus) - len(joint)})"
        else:
            relu = other
        return dict(sign="fused" if self.fused_sign else "reference", rescale=rescale, relu=relu,
                    encoding="hardened" if self.hardened else "reference")

    @property
    def table_bytes(self) -> int:
        return self.model.table_bytes()

    def plain_q_eval(self, x: np.ndarray) -> np.ndarray:
        return self.circuit.plain_q_eval(x, track=False, crt_modulus=self.crt_modulus)


def garble(circuit: Circuit, crt, mrs=None, **kw) -> GarbledCircuit:
    return GarbledCircuit(circuit, crt, mrs, **kw)
