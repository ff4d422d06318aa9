"""Attestation, sealing and process hardening of the trusted garbler (software TEE model).

The reference keeps the garbler's secrets (offsets R_p, input base labels,
decoder) inside an Intel SGX enclave (sgx/Enclave/Enclave.edl:37-135,
sgx/App/App.cpp:140-365). MI355X nodes run AMD EPYC hosts: no SGX, and the
confidential-computing equivalent (SEV-SNP guest attestation through
/dev/sev-guest) needs a confidential VM this framework cannot assume. This
module provides the same three trust mechanisms behind an interface a
hardware backend can implement:

  measurement  MRENCLAVE analogue: SHA-256 over the garbler's code (the
               garbling / IR / enclave Python modules and the native
               extension) and the circuit configuration.
  quote        the enclave's signed report {measurement, report_data, nonce},
               MACed with the platform attestation key (HMAC-SHA256). The
               relying party checks it against the measurement it expects
               before it trusts the garbler with inputs.
  sealing      authenticated encryption of garbler state under a key derived
               from the platform key and the measurement (MRENCLAVE policy):
               a different garbler build, or a modified blob, cannot unseal.

The platform key stands in for the CPU's attestation / sealing root keys: a
32-byte secret in a 0600 file (`DASH_PLATFORM_KEY_FILE`, default
~/.cache/dash_amd/platform.key), created on first use. Whoever can read that
file can forge quotes: on real hardware the key never leaves the security
processor, which is the one property a software model cannot give.

`harden()` is the enclave process's OS-level isolation: it marks the process
non-dumpable (PR_SET_DUMPABLE 0: no ptrace attach, no /proc/<pid>/mem reads by
other processes of the same user, no core dumps) and locks its pages in
memory where the memory-lock limit allows (no garbler secrets in swap).
"""
from __future__ import annotations

import ctypes
import hashlib
import hmac
import json
import os
import secrets
import struct
from pathlib import Path
from typing import Iterable, Optional

QUOTE_VERSION = 1
SEAL_MAGIC = b"DASHSEAL"
SEAL_VERSION = 1


class AttestationError(RuntimeError):
    pass


class SealError(RuntimeError):
    pass


# ------------------------------------------------------------------ platform key
def _key_path() -> Path:
    p = os.environ.get("DASH_PLATFORM_KEY_FILE")
    return Path(p) if p else Path.home() / ".cache" / "dash_amd" / "platform.key"


def platform_key(path: Optional[Path] = None) -> bytes:
    """The platform's attestation / sealing root key (created 0600 on first use)."""
    path = Path(path) if path else _key_path()
    if not path.exists():
        path.parent.mkdir(parents=True, exist_ok=True)
        fd = os.open(str(path), os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
        try:
            os.write(fd, secrets.token_bytes(32))
        finally:
            os.close(fd)
    st = path.stat()
    if st.st_mode & 0o077:
        raise AttestationError(f"platform key {path} is accessible to other users (mode {oct(st.st_mode & 0o777)})")
    key = path.read_bytes()
    if len(key) != 32:
        raise AttestationError(f"platform key {path} is not 32 bytes")
    return key


def _kdf(key: bytes, label: bytes, context: bytes) -> bytes:
    # HKDF-SHA256 (RFC 5869) with a single output block
    prk = hmac.new(b"dash_amd-kdf", key, hashlib.sha256).digest()
    return hmac.new(prk, label + b"\x00" + context + b"\x01", hashlib.sha256).digest()


# ------------------------------------------------------------------ measurement
_PKG = Path(__file__).resolve().parents[1]
_MEASURED = ("garbling/*.py", "ir/*.py", "sgx/*.py", "net/*.py", "native.py", "_dash_native*.so")


def code_files(root: Path = _PKG, patterns: Iterable[str] = _MEASURED) -> list:
    files = set()
    for pat in patterns:
        files.update(p for p in root.glob(pat) if p.is_file())
    return sorted(files)


def measure(config: Optional[dict] = None, root: Path = _PKG) -> bytes:
    """MRENCLAVE analogue: SHA-256 over (relative path, length, contents) of the garbler's code, then the
    canonical JSON of `config` (CRT base, MRS base, circuit digest: what the garbler will garble)."""
    h = hashlib.sha256(b"dash_amd-measurement-v1")
    for f in code_files(root):
        data = f.read_bytes()
        rel = str(f.relative_to(root)).encode()
        h.update(struct.pack("<I", len(rel)) + rel + struct.pack("<Q", len(data)))
        h.update(data)
    h.update(json.dumps(config or {}, sort_keys=True, separators=(",", ":")).encode())
    return h.digest()


def circuit_digest(circuit) -> str:
    """Digest of a circuit's garbling structure: input shape and every layer spec (kind, scalar parameters,
    weight arrays by dtype, shape and bytes)."""
    import numpy as np

    h = hashlib.sha256(repr(list(circuit.input_dims)).encode())
    for kind, params in circuit.garble_specs():
        h.update(struct.pack("<i", int(kind)))
        for name in sorted(params):
            v = params[name]
            h.update(name.encode() + b"=")
            if isinstance(v, np.ndarray):
                h.update(f"{v.dtype}{v.shape}".encode() + np.ascontiguousarray(v).tobytes())
            else:
                h.update(repr(v).encode())
    return h.hexdigest()


# ------------------------------------------------------------------ quotes
def _quote_body(measurement: bytes, report_data: bytes, nonce: bytes) -> bytes:
    return (b"DASHQUOT" + struct.pack("<I", QUOTE_VERSION) + measurement + struct.pack("<I", len(report_data)) +
            report_data + struct.pack("<I", len(nonce)) + nonce)


def make_quote(measurement: bytes, report_data: bytes, nonce: bytes, key: Optional[bytes] = None) -> dict:
    """The enclave's quote over (measurement, report_data, nonce)."""
    key = key if key is not None else platform_key()
    mac = hmac.new(_kdf(key, b"attest", b""), _quote_body(measurement, report_data, nonce), hashlib.sha256).digest()
    return {"version": QUOTE_VERSION, "measurement": measurement.hex(), "report_data": report_data.hex(),
            "nonce": nonce.hex(), "mac": mac.hex()}


def verify_quote(quote: dict, expected_measurement: bytes, nonce: bytes, key: Optional[bytes] = None,
                 report_data: Optional[bytes] = None) -> bytes:
    """Check a quote: MAC under the platform key, the expected measurement, freshness (our nonce) and, if
    given, the report data. Returns the report data; raises AttestationError otherwise."""
    key = key if key is not None else platform_key()
    try:
        if quote.get("version") != QUOTE_VERSION:
            raise AttestationError(f"quote version {quote.get('version')} != {QUOTE_VERSION}")
        m = bytes.fromhex(quote["measurement"])
        rd = bytes.fromhex(quote["report_data"])
        n = bytes.fromhex(quote["nonce"])
        mac = bytes.fromhex(quote["mac"])
    except (KeyError, ValueError, AttributeError) as e:
        raise AttestationError(f"malformed quote: {e}") from None
    want = hmac.new(_kdf(key, b"attest", b""), _quote_body(m, rd, n), hashlib.sha256).digest()
    if not hmac.compare_digest(want, mac):
        raise AttestationError("quote MAC does not verify under the platform key")
    if not hmac.compare_digest(m, expected_measurement):
        raise AttestationError(f"garbler measurement {m.hex()[:16]}... is not the expected "
                               f"{expected_measurement.hex()[:16]}...")
    if not hmac.compare_digest(n, nonce):
        raise AttestationError("stale quote (nonce mismatch)")
    if report_data is not None and not hmac.compare_digest(rd, report_data):
        raise AttestationError("report data mismatch")
    return rd


# ------------------------------------------------------------------ sealing
def _stream(key: bytes, iv: bytes, n: int) -> bytes:
    # HMAC-SHA256 in counter mode as the keystream (a PRF-based stream cipher)
    out = bytearray()
    ctr = 0
    while len(out) < n:
        out += hmac.new(key, iv + struct.pack("<Q", ctr), hashlib.sha256).digest()
        ctr += 1
    return bytes(out[:n])


def seal(data: bytes, measurement: bytes, key: Optional[bytes] = None, aad: bytes = b"") -> bytes:
    """Encrypt-then-MAC `data` to this measurement (MRENCLAVE policy)."""
    key = key if key is not None else platform_key()
    k_enc = _kdf(key, b"seal-enc", measurement)
    k_mac = _kdf(key, b"seal-mac", measurement)
    iv = secrets.token_bytes(16)
    ct = bytes(a ^ b for a, b in zip(data, _stream(k_enc, iv, len(data))))
    head = SEAL_MAGIC + struct.pack("<II", SEAL_VERSION, len(aad)) + aad + iv
    tag = hmac.new(k_mac, head + ct, hashlib.sha256).digest()
    return head + ct + tag


def unseal(blob: bytes, measurement: bytes, key: Optional[bytes] = None) -> tuple:
    """-> (data, aad); SealError if the blob was modified or sealed to another measurement."""
    key = key if key is not None else platform_key()
    if len(blob) < len(SEAL_MAGIC) + 8 + 16 + 32 or not blob.startswith(SEAL_MAGIC):
        raise SealError("not a sealed blob")
    ver, naad = struct.unpack_from("<II", blob, len(SEAL_MAGIC))
    if ver != SEAL_VERSION:
        raise SealError(f"seal version {ver} != {SEAL_VERSION}")
    o = len(SEAL_MAGIC) + 8
    aad = blob[o:o + naad]
    iv = blob[o + naad:o + naad + 16]
    head_len = o + naad + 16
    ct, tag = blob[head_len:-32], blob[-32:]
    k_mac = _kdf(key, b"seal-mac", measurement)
    if not hmac.compare_digest(hmac.new(k_mac, blob[:head_len] + ct, hashlib.sha256).digest(), tag):
        raise SealError("sealed blob does not authenticate (modified, or sealed by a different garbler build)")
    k_enc = _kdf(key, b"seal-enc", measurement)
    return bytes(a ^ b for a, b in zip(ct, _stream(k_enc, iv, len(ct)))), aad


# ------------------------------------------------------------------ hardening
PR_SET_DUMPABLE = 4
PR_GET_DUMPABLE = 3
MCL_CURRENT, MCL_FUTURE = 1, 2


def harden(lock_memory: bool = True) -> dict:
    """Enclave-process isolation (Linux): non-dumpable (no ptrace / /proc/<pid>/mem by peers, no core dump),
    memory locked where RLIMIT_MEMLOCK allows. Returns what took effect."""
    res = {"dumpable": None, "mlock": False}
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        libc.prctl.argtypes = [ctypes.c_int, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong]
        if libc.prctl(PR_SET_DUMPABLE, 0, 0, 0, 0) == 0:
            res["dumpable"] = int(libc.prctl(PR_GET_DUMPABLE, 0, 0, 0, 0))
        if lock_memory:
            res["mlock"] = libc.mlockall(MCL_CURRENT | MCL_FUTURE) == 0
    except (OSError, AttributeError):
        pass
    return res
