"""Trusted-garbler process split (reference SGX flow, C40/C41), CPU evaluator: attestation, sealing, hardening."""
import os
import subprocess
import sys

import numpy as np
import pytest

from dash_amd.garbling import GarbledCircuit
from dash_amd.models import build_circuit, quantized_inputs
from dash_amd.sgx import GarblerEnclave, _config
from dash_amd.sgx import attest as at


@pytest.fixture
def keyfile(tmp_path, monkeypatch):
    p = tmp_path / "platform.key"
    monkeypatch.setenv("DASH_PLATFORM_KEY_FILE", str(p))
    at.platform_key(p)  # created 0600
    return str(p)


def test_enclave_ann_infer_attested_cpu(keyfile):
    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 4)
    with GarblerEnclave(c, 7, 100.0, batch=2, backend="cpu", platform_key_file=keyfile) as enc:
        assert enc.quote is not None and enc.quote["measurement"] == at.measure(_config(c, 7, 100.0, 0)).hex()
        assert enc.hardening["dumpable"] == 0
        out = enc.ann_infer(xs)
        assert enc.last_stats["online_bytes"] > 0
        blob = enc.seal_state()
    ref = GarbledCircuit(c, 7, 100.0, garble_me=False)
    np.testing.assert_array_equal(out, np.stack([ref.plain_q_eval(x) for x in xs]))
    # a later enclave of the same build + configuration resumes the sealed master secret and GC counter
    with GarblerEnclave(c, 7, 100.0, batch=2, backend="cpu", platform_key_file=keyfile, sealed_state=blob) as enc2:
        out2 = enc2.ann_infer(xs[:2])
    np.testing.assert_array_equal(out2, out[:2])
    # resuming one blob twice (a replay by the untrusted host) must not repeat any GC seed: the same inputs
    # are encoded under different labels
    with GarblerEnclave(c, 7, 100.0, batch=2, backend="cpu", platform_key_file=keyfile, sealed_state=blob) as enc3:
        out3 = enc3.ann_infer(xs[:2])
    np.testing.assert_array_equal(out3, out[:2])
    assert enc2._server.input_digests and enc3._server.input_digests
    assert enc2._server.input_digests[0] != enc3._server.input_digests[0]
    # a modified blob is refused at start
    bad = bytearray(blob)
    bad[-40] ^= 1
    with pytest.raises(at.SealError):
        GarblerEnclave(c, 7, 100.0, batch=2, backend="cpu", platform_key_file=keyfile, sealed_state=bytes(bad))


def test_enclave_start_failure_does_not_block(keyfile, monkeypatch):
    """An enclave that dies before 'ready' (here: an unsealable blob makes it exit) is reported, not waited on."""
    import time

    c = build_circuit("MODEL_A")
    t = time.perf_counter()
    with pytest.raises(at.SealError):
        GarblerEnclave(c, 7, 100.0, batch=2, backend="cpu", platform_key_file=keyfile, sealed_state=b"x" * 64,
                       start_timeout_s=60)
    assert time.perf_counter() - t < 60


def test_quote_checks(keyfile):
    key = at.platform_key()
    m = at.measure({"crt": 7})
    nonce = os.urandom(16)
    q = at.make_quote(m, b"report", nonce, key)
    assert at.verify_quote(q, m, nonce, key, report_data=b"report") == b"report"
    with pytest.raises(at.AttestationError, match="measurement"):
        at.verify_quote(q, at.measure({"crt": 8}), nonce, key)
    with pytest.raises(at.AttestationError, match="nonce"):
        at.verify_quote(q, m, os.urandom(16), key)
    forged = dict(q, report_data=b"other".hex())
    with pytest.raises(at.AttestationError, match="MAC"):
        at.verify_quote(forged, m, nonce, key)
    with pytest.raises(at.AttestationError, match="MAC"):
        at.verify_quote(q, m, nonce, os.urandom(32))
    with pytest.raises(at.AttestationError, match="malformed"):
        at.verify_quote({"version": 1}, m, nonce, key)


def test_measurement_covers_code_and_config(tmp_path):
    root = tmp_path / "pkg"
    (root / "garbling").mkdir(parents=True)
    f = root / "garbling" / "gc.py"
    f.write_text("x = 1\n")
    m1 = at.measure({"a": 1}, root=root)
    assert at.measure({"a": 1}, root=root) == m1
    assert at.measure({"a": 2}, root=root) != m1
    f.write_text("x = 2\n")
    assert at.measure({"a": 1}, root=root) != m1


def test_seal_roundtrip_and_binding(keyfile):
    key = at.platform_key()
    m = at.measure({"crt": 7})
    blob = at.seal(b"secret" * 20, m, key, aad=b"hdr")
    assert b"secret" not in blob
    assert at.unseal(blob, m, key) == (b"secret" * 20, b"hdr")
    with pytest.raises(at.SealError):
        at.unseal(blob, at.measure({"crt": 8}), key)  # another build / configuration
    for i in (len(at.SEAL_MAGIC) + 12, len(blob) // 2, len(blob) - 1):
        bad = bytearray(blob)
        bad[i] ^= 0x80
        with pytest.raises(at.SealError):
            at.unseal(bytes(bad), m, key)
    with pytest.raises(at.SealError):
        at.unseal(b"junk", m, key)


def test_platform_key_permissions(tmp_path):
    p = tmp_path / "k"
    k = at.platform_key(p)
    assert len(k) == 32 and at.platform_key(p) == k
    assert (p.stat().st_mode & 0o777) == 0o600
    os.chmod(p, 0o644)
    with pytest.raises(at.AttestationError, match="accessible"):
        at.platform_key(p)


def test_harden_subprocess():
    code = ("from dash_amd.sgx.attest import harden; r = harden(lock_memory=False); "
            "print(r['dumpable'])")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "0"
