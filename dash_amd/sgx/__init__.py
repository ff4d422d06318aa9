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
"""
from __future__ import annotations

import multiprocessing as mp
import socket
import threading
from typing import Optional, Sequence

import numpy as np


def _enclave_main(conn, sock_fd_port, circuit, crt, mrs, max_modulus, batch):
    from ..net.protocol import GarblerClient

    host, port = sock_fd_port
    client = GarblerClient(host, port, circuit, crt, mrs, batch=batch, max_modulus=max_modulus)
    try:
        while True:
            msg = conn.recv()
            if msg is None:
                break
            xs = msg
            outs = []
            for s in range(0, len(xs), batch):
                client.offline()
                outs += client.infer(xs[s:s + batch])
            conn.send(("ok", np.stack(outs), dict(client.stats, online_s=list(client.stats["online_s"]))))
    except Exception as e:  # report to the host instead of dying silently
        conn.send(("error", repr(e), None))
    finally:
        client.close()
        conn.close()


class GarblerEnclave:
    """Host-side handle of a trusted garbler process."""

    def __init__(self, circuit, crt, mrs=None, max_modulus: int = 0, batch: int = 1, backend: str = "hip",
                 device: int = 0):
        from ..net.channel import Channel
        from ..net.protocol import EvaluatorServer

        self.batch = batch
        lst = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        lst.bind(("127.0.0.1", 0))
        lst.listen(1)
        port = lst.getsockname()[1]
        ctx = mp.get_context("spawn")
        self._conn, child = ctx.Pipe()
        self._proc = ctx.Process(target=_enclave_main,
                                 args=(child, ("127.0.0.1", port), circuit, crt, mrs, max_modulus, batch),
                                 daemon=True)
        self._proc.start()
        conn, _ = lst.accept()
        lst.close()
        self._server = EvaluatorServer(backend, device)
        self._thread = threading.Thread(target=self._server.serve, args=(Channel(conn),), daemon=True)
        self._thread.start()
        self.last_stats: Optional[dict] = None

    def ann_infer(self, inputs: Sequence[np.ndarray]) -> np.ndarray:
        """ecall: quantized inputs -> decoded outputs [n, n_out] (n multiple of batch)."""
        assert len(inputs) % self.batch == 0, "number of inputs must be a multiple of the batch"
        self._conn.send([np.asarray(x, dtype=np.int64) for x in inputs])
        status, out, stats = self._conn.recv()
        if status != "ok":
            raise RuntimeError(f"garbler enclave failed: {out}")
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
