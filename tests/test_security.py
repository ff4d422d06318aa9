"""Attacks on the offline message, run from the evaluator's view (docs/SECURITY.md).

Each attack uses only what the evaluator holds: the GarbledModel (offline message), the public circuit, its own
input labels and the labels it computes while evaluating (native.cpu_evaluate_trace). The garbler's secrets are
read only to CHECK a recovered value.

* test_bias_labels_reveal_offset: the reference encoding ships Z_p and bias labels b R_p + Z_p; two bias labels
  give R_p (R_p[0] = 1), and R_p forges an output that decodes without an integrity error.
* test_mini_table_reveals_relu_sign: a ReLU's k mixed-modulus half gates and their 16-bit mini entries are all
  masked by the same H(sign label): the unopened row's mini entries differ by a known amount, which reveals the
  sign of every ReLU input.
* test_repeated_digit_modulus_reveals_offset: the approximate sign gadget projects one residue label into every
  MRS digit under one hash; the headline MRS base (k = 7, 100 %: 86, 7, 6, 6, 5) has two digits of the same
  modulus, and the difference of their unopened entries is a digit-wise function of R_m: R_m is recovered.

All three succeed against the reference encoding (the reference's own wire format shares these properties,
SURVEY §0.1) and fail against the hardened encoding (the default of the flagship constructions).
"""
from __future__ import annotations

import numpy as np
import pytest

import dash_amd as d
from dash_amd.garbling import GarbledCircuit
from dash_amd.native import native

SEED = bytes(range(16))
M128 = 1 << 128


def _u128(a) -> int:
    a = np.asarray(a, dtype=np.uint64).reshape(-1)
    return int(a[0]) | (int(a[1]) << 64)


def _compress(L, m: int) -> int:
    c = 0
    for v in reversed([int(x) for x in L]):
        c = c * m + v
    return c


def _decompress(C: int, m: int, n: int) -> list:
    out = []
    for _ in range(n):
        out.append(C % m)
        C //= m
    out[-1] %= m
    return out


def _dense_relu(rng, nin=24, nout=32, relu=True):
    w = rng.integers(-6, 7, size=(nout, nin))
    b = rng.integers(-40, 41, size=nout)
    layers = [d.Dense.from_quantized(w, b)]
    if relu:
        layers.append(d.Relu((nout,)))
    return d.Circuit(layers), w, b


# ------------------------------------------------------------------------------------------------ primitives
def test_chacha_rfc7539_block():
    # RFC 7539 section 2.3.2 test vector (ChaCha20 block function)
    key = bytes(range(32))
    nonce = bytes.fromhex("000000090000004a00000000")
    st = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    st += list(np.frombuffer(key, dtype="<u4"))
    st += [1] + list(np.frombuffer(nonce, dtype="<u4"))
    out = native().chacha_block([int(x) for x in st], 20)
    assert out == [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204, 0x4E6CD4C3,
                   0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE, 0xE883D0CB, 0x4E3C50A2]


def test_hard_pads_are_tweaked_chacha12():
    n = native()
    K = 0x0123456789ABCDEF_FEDCBA9876543210
    gate, sub = n.stream_id(3, 30, 17), (7 << 16) | 2
    st = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574,
          K & 0xFFFFFFFF, (K >> 32) & 0xFFFFFFFF, (K >> 64) & 0xFFFFFFFF, K >> 96,
          gate & 0xFFFFFFFF, gate >> 32, sub, 0x44524148, 1, 0, 0, 0]
    w = n.chacha_block(st, 12)
    pads = n.hard_pads(K, gate, sub, 1)
    for q in range(4):
        assert pads[q] == sum(w[4 * q + i] << (32 * i) for i in range(4))
    # every tweak component changes every pad
    others = [n.hard_pads(K, gate ^ 1, sub, 1), n.hard_pads(K, gate, sub ^ 1, 1), n.hard_pads(K, gate, sub, 2),
              n.hard_pads(K ^ 1, gate, sub, 1)]
    for o in others:
        assert all(a != b for a, b in zip(o, pads))


# ------------------------------------------------------------------------------ attack 1: constant labels
def _recover_R_from_bias(model, crt):
    """The evaluator's R_p from two bias labels of one residue (b_o R + Z) - (b_o' R + Z) = (b_o - b_o') R."""
    bias = {k: v for k, v in model.layer_arrays(0).items() if k.startswith("bias.")}
    out = {}
    for j, p in enumerate(crt):
        B = bias[f"bias.{j}"].astype(np.int64)
        for o in range(1, B.shape[0]):
            delta = (B[o] - B[0]) % p
            if delta[0] % p:
                out[p] = (delta * native().mul_inv(int(delta[0]), p)) % p
                break
    return out


def test_bias_labels_reveal_offset():
    rng = np.random.default_rng(1)
    c, w, b = _dense_relu(rng, relu=False)
    crt = [2, 3, 5, 7, 11, 13]
    gc = GarbledCircuit(c, crt, None, seed=SEED, hardened=False)
    assert not gc.model.hardened and gc.model.const_names()
    R = _recover_R_from_bias(gc.model, crt)
    assert set(R) == set(crt)
    for p, r in R.items():
        np.testing.assert_array_equal(r, gc.garbler.offset_label(p))
    # forgery: shift output 0 by one in every residue; the decoder accepts it
    x = rng.integers(-20, 21, size=24)
    out = gc.cpu_evaluate(gc.garble_inputs(x))
    forged = [(p, np.array(L, copy=True)) for p, L in out]
    for p, L in forged:
        L[0] = (L[0] + R[p]) % p
    y = gc.decode_outputs(forged)
    ref = gc.plain_q_eval(x)
    assert y[0] == ref[0] + 1 and np.array_equal(y[1:], ref[1:])


def test_hardened_ships_no_constant_labels():
    rng = np.random.default_rng(1)
    c, w, b = _dense_relu(rng, relu=False)
    crt = [2, 3, 5, 7, 11, 13]
    gc = GarbledCircuit(c, crt, None, seed=SEED)  # default: hardened
    assert gc.hardened and gc.model.hardened
    assert gc.model.const_names() == []
    assert not [k for k in gc.model.layer_arrays(0) if k.startswith("bias.")]
    x = rng.integers(-20, 21, size=24)
    out = gc.cpu_evaluate(gc.garble_inputs(x))
    assert np.array_equal(gc.decode_outputs(out), gc.plain_q_eval(x))
    # a shift by anything but the (unknown) offset is caught by the decoder
    forged = [(p, np.array(L, copy=True)) for p, L in out]
    forged[1][1][0] = (forged[1][1][0] + 1) % forged[1][0]
    with pytest.raises(native().IntegrityError):
        gc.decode_outputs(forged)
    # round trip keeps the flag
    m2 = native().GarbledModel.deserialize(gc.model.serialize())
    assert m2.hardened and m2.const_names() == []


# -------------------------------------------------------------- attack 2: the ReLU half gates' mini tables
def _relu_sign_attack(gc, x, layer=1):
    """Per element: the sign value y the attack infers (or -1 when it cannot decide)."""
    n = native()
    k = len(gc.crt_base)
    _, trace = n.cpu_evaluate_trace(gc.model, gc.garble_inputs(x), 0)
    _, Y = trace[layer]
    E = gc.model.layer_arrays(layer)["mm.e"]  # (N, k, 3, 2) uint64: rows 0, 1 and the mini entry
    guesses = []
    for e in range(Y.shape[0]):
        c = int(Y[e][0]) & 1
        h16 = n.aes_hash(_compress(Y[e], 2)) & 0xFFFF
        mini = [_u128(E[e, j, 2]) for j in range(k)]
        t16 = [[(mv >> (16 * col)) & 0xFFFF for col in (0, 1)] for mv in mini]
        ypr = [((t16[j][c] - h16) & 0xFFFF) for j in range(k)]
        ypr = [(v - 0x10000 if v >= 0x8000 else v) % gc.crt_base[j] for j, v in enumerate(ypr)]
        obs = [(t16[j][1 - c] - t16[0][1 - c]) & 0xFFFF for j in range(k)]
        ok = []
        for y in (0, 1):
            f = [(ypr[j] + 1 - 2 * y) % gc.crt_base[j] for j in range(k)]
            if all(((f[j] - f[0]) & 0xFFFF) == obs[j] for j in range(1, k)):
                ok.append(y)
        guesses.append(ok[0] if len(ok) == 1 else -1)
    return np.array(guesses)


def _dense_signs(x, w, b):
    return ((np.asarray(w) @ np.asarray(x) + np.asarray(b)) >= 0).astype(int)


def test_mini_table_reveals_relu_sign():
    rng = np.random.default_rng(2)
    c, w, b = _dense_relu(rng)
    gc = GarbledCircuit(c, 6, 100.0, seed=SEED, hardened=False, relu="approx")
    x = rng.integers(-20, 21, size=24)
    got = _relu_sign_attack(gc, x)
    np.testing.assert_array_equal(got, _dense_signs(x, w, b))  # every ReLU input's sign


def test_hardened_mini_table_hides_relu_sign():
    rng = np.random.default_rng(2)
    c, w, b = _dense_relu(rng)
    gc = GarbledCircuit(c, 6, 100.0, seed=SEED)
    assert gc.hardened
    x = rng.integers(-20, 21, size=24)
    assert np.array_equal(gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x))), gc.plain_q_eval(x))
    got = _relu_sign_attack(gc, x)
    truth = _dense_signs(x, w, b)
    assert np.mean(got == truth) < 0.25  # undecided (-1) for almost every element


# ----------------------------------------------------- attack 3: repeated MRS digit modulus (approx sign gadget)
def _recover_R_repeated_digit(gc, x, d1=2, d2=3, layer=1, tries=24):
    """R_m from the entries of digits d1, d2 (same modulus m) of approx rows, or None."""
    n = native()
    sp_crt, mrs = gc.crt_base, gc.mrs_base
    t = len(mrs)
    k = len(sp_crt)
    fused = gc.fused_sign
    mod = (lambda dd: (k + 1) * mrs[dd] if (fused and dd >= 1) else mrs[dd])
    m = mod(d1)
    assert mod(d2) == m
    nm = n.nr_comps(m)
    lut = n.gen_approx_lookup(sp_crt, mrs)
    prefix = np.concatenate([[0], np.cumsum(sp_crt)[:-1]]).astype(int)
    relu_in, _ = n.cpu_evaluate_trace(gc.model, gc.garble_inputs(x), 0)[1][layer]
    A = gc.model.layer_arrays(layer)["s.approx"]  # (N, t * sum(crt), 2)
    found = 0
    for e in range(min(tries, A.shape[0])):
        for j, p in enumerate(sp_crt):
            X = relu_in[j][1][e]
            cx = int(X[0]) % p
            h = n.aes_hash(_compress(X, p))  # the reference mask of this key (every digit shares it)
            base = t * prefix[j]
            ent = lambda col, dd: _u128(A[e, base + col * t + dd])
            A1 = _decompress((ent(cx, d1) - h) % M128, m, nm)
            A2 = _decompress((ent(cx, d2) - h) % M128, m, nm)
            rows = []
            for col in range(p):
                if col == cx:
                    continue
                D = (ent(col, d1) - ent(col, d2)) % M128
                rows.append((D - M128 if D >= 1 << 127 else D, col))
            for vx in range(p):  # the evaluator guesses x mod p
                cons = []
                for D, col in rows:
                    vc = (vx + col - cx) % p
                    cons.append([D, lut[j][vc * t + d1] - lut[j][vx * t + d1], lut[j][vc * t + d2] - lut[j][vx * t + d2]])
                R = _dfs_offset(cons, A1, A2, m, nm)
                if R is not None:
                    if np.array_equal(R, gc.garbler.offset_label(m)):
                        return R
    return None


def _dfs_offset(cons, A1, A2, m, nm, c=0, R=None):
    R = [] if R is None else R
    if c == nm:
        return np.array(R) if all(cc[0] == 0 for cc in cons) else None
    cands = [1] if c == 0 else range(m)
    for r in cands:
        nxt = []
        for D, da, db in cons:
            diff = (A1[c] + da * r) % m - (A2[c] + db * r) % m
            if (D - diff) % m:
                break
            nxt.append([(D - diff) // m, da, db])
        else:
            got = _dfs_offset(nxt, A1, A2, m, nm, c + 1, R + [r])
            if got is not None:
                return got
    return None


@pytest.mark.parametrize("fused", [False, True])
def test_repeated_digit_modulus_reveals_offset(fused):
    rng = np.random.default_rng(3)
    c, w, b = _dense_relu(rng, nout=16)
    gc = GarbledCircuit(c, 7, 100.0, seed=SEED, hardened=False, fused_sign=fused, relu="approx")
    assert gc.mrs_base == [86, 7, 6, 6, 5]
    x = rng.integers(-20, 21, size=24)
    assert _recover_R_repeated_digit(gc, x) is not None


def test_hardened_repeated_digit_modulus_hides_offset():
    rng = np.random.default_rng(3)
    c, w, b = _dense_relu(rng, nout=16)
    gc = GarbledCircuit(c, 7, 100.0, seed=SEED, relu="approx")
    assert gc.hardened
    x = rng.integers(-20, 21, size=24)
    assert np.array_equal(gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x))), gc.plain_q_eval(x))
    assert _recover_R_repeated_digit(gc, x, tries=8) is None


def test_mrs_constructions_require_hardened():
    rng = np.random.default_rng(4)
    c, _, _ = _dense_relu(rng)
    with pytest.raises(ValueError):
        GarbledCircuit(c, 6, 100.0, seed=SEED, hardened=False, relu="mrs")
    with pytest.raises(ValueError):
        GarbledCircuit(c, 6, 100.0, seed=SEED, hardened=True, fused_sign=False)


def _calibrated_rescale_circuit(rng):
    """Dense -> Rescale(2) -> ReLU, calibrated: rescale='auto' may pick the mixed-radix construction."""
    w = rng.integers(-6, 7, size=(16, 12))
    b = rng.integers(-40, 41, size=16)
    c = d.Circuit([d.Dense.from_quantized(w, b), d.Rescale(2, (16,)), d.Relu((16,))])
    from dash_amd.ir.bases import crt_modulus, first_primes

    c.calibrate([rng.integers(-20, 21, size=12) for _ in range(8)], crt_modulus(first_primes(7)))
    return c


def test_auto_constructions_follow_requested_encoding():
    """'auto' never resolves to a construction the requested sign / encoding cannot carry (the mixed-radix
    ones exist only in the hardened encoding, which needs the fused sign): it falls back to the reference
    constructions instead of raising."""
    rng = np.random.default_rng(11)
    c = _calibrated_rescale_circuit(rng)
    gc = GarbledCircuit(c, 7, 100.0, seed=SEED)
    assert (gc.rescale, gc.relu, gc.hardened) == ("mrs", "joint", True)
    gc = GarbledCircuit(c, 7, 100.0, seed=SEED, fused_sign=False, hardened=False)
    assert (gc.rescale, gc.relu, gc.hardened) == ("legacy", "approx", False)
    gc = GarbledCircuit(c, 7, 100.0, seed=SEED, hardened=False)
    assert (gc.rescale, gc.relu, gc.hardened) == ("legacy", "approx", False)
    x = rng.integers(-20, 21, size=12)
    assert np.array_equal(gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x))), gc.plain_q_eval(x))


def test_reference_encoding_fallback_is_never_silent():
    from dash_amd.garbling import ReferenceEncodingWarning
    from dash_amd.serving import InferenceService

    rng = np.random.default_rng(12)
    c = _calibrated_rescale_circuit(rng)
    with pytest.warns(ReferenceEncodingWarning):
        gc = GarbledCircuit(c, 7, 100.0, seed=SEED, fused_sign=False)  # hardened=None, reference sign
    assert not gc.hardened
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("error", ReferenceEncodingWarning)
        GarbledCircuit(c, 7, 100.0, seed=SEED, fused_sign=False, hardened=False)  # explicit: no warning
    # the serving engine refuses the reference encoding unless it is asked for
    with pytest.raises(ValueError, match="hardened=False"):
        InferenceService(c, 7, 100.0, backend="cpu", fused_sign=False, prefetch=False)
    with InferenceService(c, 7, 100.0, backend="cpu", fused_sign=False, hardened=False, prefetch=False,
                          slots_per_group=1, groups=1) as svc:
        x = rng.integers(-20, 21, size=12)
        y = svc.infer([x])
        assert svc.stats.as_dict()["encoding"] == "reference"
    with InferenceService(c, 7, 100.0, backend="cpu", prefetch=False, slots_per_group=1, groups=1) as svc:
        svc.infer([x])
        assert svc.stats.as_dict()["encoding"] == "hardened"
