"""Wire-compatibility vectors: the native garbler's gate tables equal, byte for
byte, tables built from the reference's formulas by a pure-Python oracle
(tests/gates_ref.py), for fixed labels. Covers the projection gate (any
function, modulus change both ways), the mini projection's int16 packing and
the mixed-modulus half gate of the ReLU."""
import numpy as np
import pytest

from tests import gates_ref as ref


def _lab(rng, p, first=None):
    from dash_amd.native import native

    n = native().nr_comps(p)
    v = rng.integers(0, p, n).astype(np.int16)
    if first is not None:
        v[0] = first
    return v


@pytest.mark.parametrize("pin,pout,fn", [(19, 19, "ident"), (19, 91, "sq"), (91, 19, "div"), (2, 17, "sign"),
                                         (17, 2, "par"), (7, 86, "lut"), (64, 13, "fin")])
def test_projection_gate_matches_reference_formula(native, pin, pout, fn):
    rng = np.random.default_rng(pin * 1000 + pout)
    in0, Rin = _lab(rng, pin), _lab(rng, pin, first=1)  # R_p[0] = 1: colors permute
    out0, outR = _lab(rng, pout), _lab(rng, pout, first=1)
    lut = rng.integers(-500, 500, pin)
    f = {"ident": lambda v: v, "sq": lambda v: v * v, "div": lambda v: v // 5, "sign": lambda v: 1 - 2 * v,
         "par": lambda v: v % 2, "lut": lambda v: int(lut[v]), "fin": lambda v: -v}[fn]
    fv = [f(v) for v in range(pin)]
    got = ref.from_u64(native.garble_projection_gate(in0, Rin, pin, out0, outR, pout, fv))
    exp = ref.projection_table(in0, Rin, pin, out0, outR, pout, lambda v: fv[v])
    assert got == exp


@pytest.mark.parametrize("pin", [2, 3, 5, 7])
def test_mini_projection_int16_packing(native, pin):
    rng = np.random.default_rng(pin)
    in0, Rin = _lab(rng, pin), _lab(rng, pin, first=1)
    fv = [int(v) for v in rng.integers(0, 30000, pin)]
    got = ref.from_u64(native.garble_mini_gate(in0, Rin, pin, fv))[0]
    assert got == ref.mini_entry(in0, Rin, pin, lambda v: fv[v])


@pytest.mark.parametrize("p", [3, 5, 7, 11, 13, 17])
def test_mixed_mod_half_gate_matches_reference_formula(native, p):
    """The ReLU's x (mod p) * sign (mod 2) gate: G [p], E [q + 1] (mini entry last), out0 = sk04 - sk03, with
    sk03 / sk04 the two PRG labels the native garbler draws (Prg::label, oracle-tested in test_crypto_labels)."""
    q = 2
    rng = np.random.default_rng(p)
    x0, y0 = _lab(rng, p), _lab(rng, q)
    Rp, Rq = _lab(rng, p, first=1), _lab(rng, q, first=1)
    seed, stream = bytes(range(40, 56)), 77
    g, e, out0 = native.garble_mixed_mod_gate(x0, p, y0, q, Rp, Rq, seed, stream)
    n = native.nr_comps(p)
    m = 128 // (p.bit_length() - 1) if p & (p - 1) == 0 else max(i for i in range(1, 64) if p ** i <= 2 ** 64)
    sk03 = native.prg_label(seed, stream, 0, p)
    sk04 = native.prg_label(seed, stream, -(-n // m), p)
    G, E, o = ref.mixed_mod_half_gate(x0, p, y0, q, Rp, Rq, sk03, sk04)
    assert ref.from_u64(g) == G
    assert ref.from_u64(e) == E
    assert [int(v) for v in out0] == o


def test_reference_layout_export_import_roundtrip():
    """Sign / ReLU / legacy-rescale tables exported to the reference's layouts (Appendix A.3) sit where the
    reference indexes them, and a model whose tables are wiped and re-imported from that export still decodes."""
    import dash_amd as d
    from dash_amd.garbling import GarbledCircuit
    from dash_amd.garbling.reflayout import export_reference, import_reference
    from dash_amd.ir.layers import Relu, Rescale, Sign

    n = 40
    c = d.Circuit([Rescale(1, (n,)), Relu((n,)), Sign((n,))])
    x = np.arange(-n // 2, n // 2, dtype=np.int64) * 3
    gc = GarbledCircuit(c, 7, 100.0, seed=bytes(range(16)), fused_sign=False, rescale="legacy", relu="approx")
    m = gc.model
    exp = export_reference(m)
    crt, t = list(m.crt), len(m.mrs)
    # digit-major approx table: entry (residue j, digit dd, color cc) of element e at t*prefix_j + dd*p_j + cc
    li, name = next(k for k in exp if k[1].endswith("s.approx"))
    ours, refl = m.layer_arrays(li)[name], exp[(li, name)]
    pre = 0
    for p in crt:
        for dd in range(t):
            for cc in range(p):
                np.testing.assert_array_equal(refl[:, t * pre + dd * p + cc], ours[:, t * pre + cc * t + dd])
        pre += p
    y0 = gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x)))
    for (li, name) in exp:
        m.layer_arrays(li)[name][...] = 0
    import_reference(m, exp)
    np.testing.assert_array_equal(gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x))), y0)
    np.testing.assert_array_equal(y0, c.plain_q_eval(x, False, gc.crt_modulus))
    with pytest.raises(ValueError, match="fused"):
        export_reference(GarbledCircuit(c, 7, 100.0, seed=bytes(16), fused_sign=True, rescale="legacy").model)
