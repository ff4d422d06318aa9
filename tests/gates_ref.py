"""Pure-Python oracle of the reference's garbled gates, written from the
reference formulas (not from this repository's C++):

* ProjectionGate::garble (/root/reference/dash/include/garbling/gates/projection_gate.h:62-87):
  for i < p_in: key = i*R_in + in0 (component-wise mod p_in); payload = f(i)*out_offset + out_base (mod p_out);
  T[color(key)] = compress(payload) + H(compress(key))  (mod 2^128)
* ProjectionGateMini::garble (projection_gate_mini.h:25-43):
  ((int16*)T)[color(key)] = f(i) + (int16)H(compress(key))
* MixedModHalfGate::garble (mixed_mod_half_gate.h:56-89): r = color(x0);
  garbler gate  G: x -> x*r,        payload base sk03, offset R_p
  evaluator gate E: y -> -(y+r) mod p, payload base sk04, offset x0 (!)
  mini gate E[q]: y -> (y+r) mod p; output base label sk04 - sk03.

compress: C = sum_c L_c p^c (label_tensor.h:715-724); H: fixed-key AES-128 (tests/aes_ref.py).
"""
from __future__ import annotations

from tests.aes_ref import dash_hash

MASK = (1 << 128) - 1


def compress(label, p: int) -> int:
    return sum(int(c) * p ** i for i, c in enumerate(label)) & MASK


def affine(base, offset, x: int, p: int) -> list:
    return [(int(b) + x * int(o)) % p for b, o in zip(base, offset)]


def projection_table(in0, Rin, pin, out0, out_off, pout, f) -> list:
    T = [None] * pin
    for i in range(pin):
        key = affine(in0, Rin, i, pin)
        pay = affine(out0, out_off, f(i) % pout, pout)
        T[key[0]] = (compress(pay, pout) + dash_hash(compress(key, pin))) & MASK
    return T


def mini_entry(in0, Rin, pin, f) -> int:
    slots = [0] * 8
    for i in range(pin):
        key = affine(in0, Rin, i, pin)
        h16 = dash_hash(compress(key, pin)) & 0xFFFF
        slots[key[0]] = (f(i) + h16) & 0xFFFF
    return sum(v << (16 * s) for s, v in enumerate(slots))


def mixed_mod_half_gate(x0, p, y0, q, Rp, Rq, sk03, sk04):
    r = int(x0[0])
    G = projection_table(x0, Rp, p, sk03, Rp, p, lambda v: v * r)
    E = projection_table(y0, Rq, q, sk04, x0, p, lambda v: (-(v + r)) % p)
    E.append(mini_entry(y0, Rq, q, lambda v: (v + r) % p))
    out0 = [(int(a) - int(b)) % p for a, b in zip(sk04, sk03)]
    return G, E, out0


def from_u64(arr) -> list:
    """(entries, 2) uint64 (lo, hi) -> python ints."""
    return [int(lo) | (int(hi) << 64) for lo, hi in arr]
