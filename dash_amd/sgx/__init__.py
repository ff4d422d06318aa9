"""Trusted-garbler deployment (the reference's SGX split, C40/C41).

The reference runs the garbler inside an Intel SGX enclave and the GPU
evaluator in the untrusted host process; every device operation is an ocall
(sgx/Enclave/Enclave.edl:37-135, sgx/App/App.cpp). Intel SGX does not exist on
AMD EPYC hosts of MI355X nodes; the equivalent trust boundary there is a
separate process — optionally inside an SEV-SNP confidential VM — that holds
all garbler secrets (offsets R_p, input base labels, decoder).

`GarblerEnclave` reproduces the reference's `ecall_ann_infer` flow with that
boundary:

    host (untrusted, owns the GPU)              enclave process (trusted)
    ------------------------------              -------------------------
    ann_infer(images)  ---- ecall (pipe) ---->  quantize, garble fresh GCs
    EvaluatorServer    <--- MODL (offline) ---  serialized GarbledModel
                       <--- INPT (online #1) -  compressed input labels
                       ---- OUTP (online #2) -> decode (integrity-checked)
    predictions        <--- return (pipe) ----

The host never sees R_p or the decoder; the enclave never touches the GPU.

Trust mechanisms (attest.py): the enclave process hardens itself (non-dumpable,
memory locked), the host verifies its quote (measurement of the garbler build
and circuit configuration, fresh nonce) before handing over inputs, and the
garbler's master secret + GC counter can be sealed to that measurement and
resumed by a later enclave of the same build.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import socket
import threading
from typing import Optional, Sequence

import numpy as np


def _config(circuit, crt, mrs, max_modulus) -> dict:
    from .attest import circuit_digest

    return {"crt": crt if isinstance(crt, int) else [int(p) for p in crt],
            "mrs": mrs if mrs is None or isinstance(mrs, (int, float)) else [int(m) for m in mrs],
            "max_modulus": int(max_modulus), "circuit": circuit_digest(circuit)}


def _enclave_main(conn, sock_fd_port, circuit, crt, mrs, max_modulus, batch, sealed, key_file, garble_device=None,
                  client_kw=None):
    import hashlib
    import json
    import secrets

    from ..net.protocol import GarblerClient
    from . import attest

    try:
        if key_file:
            os.environ["DASH_PLATFORM_KEY_FILE"] = key_file
        hard = attest.harden(lock_memory=False)  # mlockall(MCL_FUTURE) makes later allocations fail at the limit
        cfg = _config(circuit, crt, mrs, max_modulus)
        meas = attest.measure(cfg)
        report = hashlib.sha256(b"dash_amd garbler v1" + json.dumps(cfg, sort_keys=True).encode()).digest()
        if sealed is not None:
            # resume: the sealed master secret is re-keyed with fresh enclave randomness, so a replayed or
            # duplicated blob (the host controls which blob it hands back) can never reproduce a per-GC seed;
            # the counter only continues the numbering
            state, _ = attest.unseal(sealed, meas)
            master = hashlib.sha256(b"dash_amd resume" + state[:32] + secrets.token_bytes(32)).digest()
            ctr = int.from_bytes(state[32:40], "little")
        else:
            master, ctr = secrets.token_bytes(32), 0
    except BaseException as e:  # every failure before 'ready' reaches the host instead of a silent death
        conn.send(("error", repr(e), None))
        conn.close()
        return
    # ready before connecting: the host starts its evaluator server only after this message, and the client's
    # HELO waits for that server
    conn.send(("ready", hard, None))
    host, port = sock_fd_port
    client = None
    try:
        client = GarblerClient(host, port, circuit, crt, mrs, batch=batch, max_modulus=max_modulus, seed=master,
                               device=garble_device, **(client_kw or {}))
        client._ctr = ctr
        while True:
            msg = conn.recv()
            if msg is None:
                break
            op, arg = msg
            if op == "attest":
                conn.send(("ok", attest.make_quote(meas, report, arg), None))
            elif op == "seal":
                state = master + client._ctr.to_bytes(8, "little")
                conn.send(("ok", attest.seal(state, meas, aad=b"dash_amd garbler state"), None))
            elif op == "infer":
                xs = arg
                outs = []
                for s in range(0, len(xs), batch):
                    client.offline()
                    outs += client.infer(xs[s:s + batch])
                conn.send(("ok", np.stack(outs), dict(client.stats, online_s=list(client.stats["online_s"]))))
            else:
                conn.send(("error", f"unknown ecall {op!r}", None))
    except Exception as e:  # report to the host instead of dying silently
        conn.send(("error", repr(e), None))
    finally:
        if client is not None:
            client.close()
        conn.close()


class GarblerEnclave:
    """Host-side handle of a trusted garbler process.

    attest: verify the enclave's quote (fresh nonce, expected measurement of this garbler build and circuit
    configuration) before any input is handed over; AttestationError otherwise.
    sealed_state: a blob from seal_state() of an earlier enclave of the same build and configuration: the
    garbler resumes from it with its master secret re-keyed by fresh enclave randomness, so no per-GC seed is
    reused even when the host replays one blob to several enclaves.

    start_timeout_s: the enclave must report ready (and connect back) within this time, else SealError.
    garble_device: the trusted garbler garbles on this GPU (its own device in a deployment whose accelerator is
    inside the trust boundary, e.g. a confidential-computing GPU); None garbles on the enclave's CPU, as the
    reference's SGX enclave does. client_kw: GarblerClient options (pipeline, rescale / relu constructions)."""

    def __init__(self, circuit, crt, mrs=None, max_modulus: int = 0, batch: int = 1, backend: str = "hip",
                 device: int = 0, attest: bool = True, sealed_state: Optional[bytes] = None,
                 platform_key_file: Optional[str] = None, start_timeout_s: float = 120.0,
                 garble_device: Optional[int] = None, client_kw: Optional[dict] = None):
        from ..net.channel import Channel
        from ..net.protocol import EvaluatorServer
        from . import attest as at

        self.batch = batch
        self._key_file = platform_key_file
        lst = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        lst.bind(("127.0.0.1", 0))
        lst.listen(1)
        port = lst.getsockname()[1]
        ctx = mp.get_context("spawn")
        self._conn, child = ctx.Pipe()
        self._proc = ctx.Process(target=_enclave_main,
                                 args=(child, ("127.0.0.1", port), circuit, crt, mrs, max_modulus, batch,
                                       sealed_state, platform_key_file, garble_device, client_kw),
                                 daemon=True)
        self._proc.start()
        child.close()  # the child's end lives in the child only: a dead child reads as EOF here

        def _fail(why: str):
            lst.close()
            if self._proc.is_alive():
                self._proc.terminate()
            self._proc.join(timeout=30)
            raise at.SealError(f"garbler enclave failed to start: {why}")

        try:
            if not self._conn.poll(start_timeout_s):
                _fail(f"no ready message within {start_timeout_s:.0f} s (alive={self._proc.is_alive()})")
            status, info, _ = self._conn.recv()
        except EOFError:
            _fail(f"enclave process exited (code {self._proc.exitcode})")
        if status != "ready":
            _fail(str(info))
        self.hardening = info
        lst.settimeout(start_timeout_s)
        try:
            conn, _ = lst.accept()
        except OSError:  # timeout: the enclave's client never connected; its reason is on the pipe
            why = self._conn.recv()[1] if self._conn.poll(1.0) else "no connection"
            _fail(f"garbler did not connect: {why}")
        conn.settimeout(None)
        lst.close()
        self._server = EvaluatorServer(backend, device)
        self._thread = threading.Thread(target=self._server.serve, args=(Channel(conn),), daemon=True)
        self._thread.start()
        self.last_stats: Optional[dict] = None
        self.quote: Optional[dict] = None
        self._cfg = _config(circuit, crt, mrs, max_modulus)
        if attest:
            try:
                self.attest()
            except Exception:
                self.close()
                raise

    def _ecall(self, op, arg=None):
        self._conn.send((op, arg))
        status, out, stats = self._conn.recv()
        if status != "ok":
            raise RuntimeError(f"garbler enclave failed: {out}")
        return out, stats

    def attest(self, nonce: Optional[bytes] = None) -> dict:
        """Challenge the enclave with a fresh nonce and verify its quote against the measurement this host
        expects for the garbler build + circuit configuration."""
        import os as _os

        from . import attest as at

        # this enclave's platform key (explicit file, else the process default): an environment variable left by
        # an earlier enclave of this process must not pick another platform's key
        key = at.platform_key(self._key_file) if self._key_file else None
        nonce = nonce or _os.urandom(16)
        quote, _ = self._ecall("attest", nonce)
        at.verify_quote(quote, at.measure(self._cfg), nonce, key=key)
        self.quote = quote
        return quote

    def seal_state(self) -> bytes:
        """The garbler's master secret and GC counter, sealed to this build + configuration."""
        blob, _ = self._ecall("seal")
        return blob

    def ann_infer(self, inputs: Sequence[np.ndarray]) -> np.ndarray:
        """ecall: quantized inputs -> decoded outputs [n, n_out] (n multiple of batch)."""
        assert len(inputs) % self.batch == 0, "number of inputs must be a multiple of the batch"
        out, stats = self._ecall("infer", [np.asarray(x, dtype=np.int64) for x in inputs])
        self.last_stats = stats
        return out

    def close(self) -> None:
        try:
            self._conn.send(None)
        except (OSError, BrokenPipeError):
            pass
        self._proc.join(timeout=60)
        self._thread.join(timeout=60)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
