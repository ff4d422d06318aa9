"""GarbledModel / Decoder serialization, fault injection (IntegrityError),
determinism across thread counts, config + CLI."""
import json

import numpy as np
import pytest

import dash_amd as d
from dash_amd.garbling import GarbledCircuit
from dash_amd.models import build_circuit, quantized_inputs
from dash_amd.native import native


@pytest.fixture(scope="module")
def small():
    from dash_amd.ir.quant import QuantizationMethod as Q

    c = build_circuit("MODEL_B_POOL_REPL", Q.ScaleQuant, 3, seed=2)
    xs = quantized_inputs("MODEL_B_POOL_REPL", 2, Q.ScaleQuant, 3)
    return c, xs


def test_serialize_roundtrip(small):
    c, xs = small
    gc = GarbledCircuit(c, 8, 100.0, seed=b"s" * 16)
    blob = gc.model.serialize()
    m2 = native().GarbledModel.deserialize(blob)
    assert m2.serialize() == blob
    dec2 = native().Decoder.deserialize(gc.decoder.serialize())
    g = gc.garble_inputs(xs[0])
    out = native().cpu_evaluate(m2, g, 0)
    np.testing.assert_array_equal(np.asarray(dec2.decode(out)), gc.plain_q_eval(xs[0]))
    with pytest.raises(RuntimeError):
        native().GarbledModel.deserialize(blob[:-7])
    with pytest.raises(RuntimeError):
        native().GarbledModel.deserialize(b"XXXXXXXX" + blob[8:])


def test_fault_injection_raises_integrity_error(small):
    c, xs = small
    gc = GarbledCircuit(c, 8, 100.0, seed=b"f" * 16)
    g = gc.garble_inputs(xs[0])
    ref = gc.decode_outputs(gc.cpu_evaluate(g))
    # flip every entry of the last ReLU's sign table: the evaluated labels become invalid
    relu = max(i for i, l in enumerate(c.layers) if l.name == "approx_relu")
    arr = gc.model.layer_arrays(relu)["s.sign"]
    for e in range(arr.shape[0] * arr.shape[1]):
        gc.model.flip_table_bit(relu, "s.sign", e, 77)
    with pytest.raises(d.IntegrityError):
        gc.decode_outputs(gc.cpu_evaluate(g))
    assert ref is not None


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_garbling_is_deterministic_across_threads(small, threads):
    c, xs = small
    ref = GarbledCircuit(c, 8, 100.0, seed=b"d" * 16, nthreads=1).model.serialize()
    got = GarbledCircuit(c, 8, 100.0, seed=b"d" * 16, nthreads=threads).model.serialize()
    assert got == ref
    gc = GarbledCircuit(c, 8, 100.0, seed=b"d" * 16, nthreads=threads)
    g = gc.garble_inputs(xs[1])
    a = gc.cpu_evaluate(g, 1)
    b = gc.cpu_evaluate(g, threads)
    for (p1, x1), (p2, x2) in zip(a, b):
        assert p1 == p2
        np.testing.assert_array_equal(x1, x2)


def test_fresh_seeds_give_fresh_labels(small):
    c, xs = small
    a = GarbledCircuit(c, 8, 100.0).garble_inputs_compressed(xs[0])
    b = GarbledCircuit(c, 8, 100.0).garble_inputs_compressed(xs[0])
    assert not np.array_equal(a, b)


def test_config_roundtrip_and_schemes(tmp_path):
    from dash_amd.config import DashConfig
    from dash_amd.ir.quant import QuantizationMethod as Q

    cfg = DashConfig(model="MODEL_F_MINIONN_POOL_REPL", scheme="REDASH_OPT", batch=4)
    qm, qp, crt, mrs, mm = cfg.resolved()
    assert qm == Q.ScaleQuantPlus and qp == 32 and crt == [32, 97, 107] and mrs == [22, 19, 15, 13] and mm == 107
    p = tmp_path / "c.json"
    cfg.save(str(p))
    assert DashConfig.load(str(p)) == cfg
    assert DashConfig(scheme="DASH").resolved()[:4] == (Q.ScaleQuant, 5, 7, 100.0)
    y = tmp_path / "c.yaml"
    y.write_text("model: MODEL_A\nscheme: SIMPLE\nbackend: cpu\nunknown_key: 3\n")
    c2 = DashConfig.load(str(y))
    assert c2.model == "MODEL_A" and c2.backend == "cpu" and c2.extra == {"unknown_key": 3}


def test_cli_infer_and_garble(tmp_path, capsys):
    from dash_amd.__main__ import main

    main(["infer", "--model", "MODEL_A", "--scheme", "SIMPLE", "--backend", "cpu", "--inputs", "2"])
    out = capsys.readouterr().out
    assert out.count("garbled==plaintext: True") == 2
    main(["garble", "--model", "MODEL_A", "--scheme", "SIMPLE", "--out", str(tmp_path / "a.dgc"),
          "--decoder-out", str(tmp_path / "a.dec"), "--seed", json.dumps("00" * 16)])
    blob = (tmp_path / "a.dgc").read_bytes()
    assert blob[:8] == b"DAMDGC01"
    assert (tmp_path / "a.dec").read_bytes()[:8] == b"DAMDDEC1"


def test_compressed_encoding_matches_label_encoding(small):
    """Online message #1 in wire form == compress(label-form encoding), every residue and element."""
    c, xs = small
    gc = GarbledCircuit(c, 8, 100.0, seed=b"w" * 16)
    for x in xs:
        wire = np.asarray(gc.garble_inputs_compressed(x))
        ref = np.asarray(native().compress_labels(gc.garble_inputs(x))).reshape(wire.shape)
        np.testing.assert_array_equal(wire, ref)
