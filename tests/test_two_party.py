"""Garbler and evaluator in separate processes over localhost TCP
(SURVEY §4.3 item 4). Replaces the reference's SGX enclave/host split."""
import multiprocessing as mp

import numpy as np
import pytest

import dash_amd as d
from dash_amd.models import build_circuit, quantized_inputs
from dash_amd.net import GarblerClient, listen
from dash_amd.net.protocol import serve_once


def _server(port_q, backend, tamper):
    s = listen("127.0.0.1", 0)
    port_q.put(s.getsockname()[1])
    serve_once(s, backend=backend, tamper=tamper)
    s.close()


def _start(backend="cpu", tamper=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_server, args=(q, backend, tamper), daemon=True)
    p.start()
    return p, q.get(timeout=120)


def test_two_party_cpu_rounds():
    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 4)
    p, port = _start()
    try:
        with GarblerClient("127.0.0.1", port, c, 7, 100.0, batch=2, seed=b"t" * 16) as cl:
            for r in range(2):
                cl.offline()
                outs = cl.infer(xs[2 * r:2 * r + 2])
                for x, y in zip(xs[2 * r:2 * r + 2], outs):
                    np.testing.assert_array_equal(y, _plain(c, x))
            # online traffic: k*16 B per input and output label (+ 2 frame headers / round)
            k, n_in, n_out = 7, c.input_size, c.output_size
            per_round = 2 * (k * 16 * n_in + k * 16 * n_out) + 2 * 16
            assert cl.stats["online_bytes"] == 2 * per_round
            # GCs are single use
            with pytest.raises(RuntimeError):
                cl.infer(xs[:2])
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0


def _plain(c, x):
    from dash_amd.garbling import GarbledCircuit

    g = GarbledCircuit(c, 7, 100.0, seed=bytes(16), garble_me=False)
    return g.plain_q_eval(x)


def test_two_party_detects_tampering():
    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 1)
    p, port = _start(tamper=True)
    try:
        with GarblerClient("127.0.0.1", port, c, 7, 100.0, batch=1) as cl:
            cl.offline()
            with pytest.raises(d.IntegrityError):
                cl.infer(xs)
    finally:
        p.join(timeout=60)


def test_two_party_rejects_incomplete_batch():
    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 2)
    p, port = _start()
    try:
        cl = GarblerClient("127.0.0.1", port, c, 7, 100.0, batch=2)
        from dash_amd.garbling import GarbledCircuit

        gc = GarbledCircuit(c, 7, 100.0)
        cl.ch.send(b"MODL", gc.model.serialize(), flags=0)
        cl.ch.recv(b"ACK_")
        cl.gcs = [gc, gc]
        with pytest.raises(RuntimeError, match="slots"):
            cl.infer(xs)
        cl.close()
    finally:
        p.join(timeout=60)


@pytest.mark.gpu
def test_two_party_hip_server_in_thread():
    """HIP evaluator party; both parties in one process (no process spawn on the GPU box)."""
    import threading

    from dash_amd.net.channel import Channel
    from dash_amd.net.protocol import EvaluatorServer

    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 4)
    s = listen("127.0.0.1", 0)
    port = s.getsockname()[1]

    def serve():
        conn, _ = s.accept()
        EvaluatorServer("hip").serve(Channel(conn))

    th = threading.Thread(target=serve, daemon=True)
    th.start()
    with GarblerClient("127.0.0.1", port, c, 7, 100.0, batch=2) as cl:
        for r in range(2):
            cl.offline()
            outs = cl.infer(xs[2 * r:2 * r + 2])
            for x, y in zip(xs[2 * r:2 * r + 2], outs):
                np.testing.assert_array_equal(y, _plain(c, x))
    th.join(timeout=60)
    s.close()


def test_two_party_benchmark_cpu():
    """benchmarks/two_party.py over both splits (TCP client/server processes, attested enclave process) on the
    host evaluator: one JSON record per split, verified against the plaintext model, offline bytes counted."""
    import os
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "benchmarks"))  # importable by name in the spawned server too
    import two_party as tp
    recs = tp.main(["--backend", "cpu", "--models", "MODEL_A/SIMPLE", "--batch", "2", "--rounds", "1",
                    "--transport", "tcp,shm"])
    assert [(r["split"], r["transport"]) for r in recs] == [("tcp", "tcp"), ("tcp", "shm"), ("enclave", "tcp"),
                                                            ("enclave", "shm")]
    for r in recs:
        assert r["verified"] and r["offline_gb_per_gc"] > 0 and r["served_inf_per_s"] > 0
        assert r["online_bytes_per_inference"] > 0 and r["online_round_ms"] > 0


def test_shm_transport_matches_tcp():
    """The same-host shared-memory offline transport ships the same models: same seeds -> identical outputs,
    serial and pipelined (the ring of 3 segments is reused after each ACK across 2 rounds of 4 GCs)."""
    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 4)
    res = []
    for transport, pipe in (("tcp", False), ("shm", False), ("shm", True)):
        p, port = _start()
        try:
            with GarblerClient("127.0.0.1", port, c, 7, 100.0, batch=4, seed=b"s" * 16, pipeline=pipe,
                               transport=transport) as cl:
                outs = []
                for _ in range(2):
                    cl.offline()
                    outs.append(np.stack(cl.infer(xs)))
                res.append(np.stack(outs))
        finally:
            p.join(timeout=60)
    np.testing.assert_array_equal(res[0], res[1])
    np.testing.assert_array_equal(res[0], res[2])


def test_pipelined_offline_matches_serial():
    """The pipelined offline phase (garbling overlapped with shipping, ACKs collected last) ships the same
    models as the serial one: same seeds -> identical outputs and offline byte counts."""
    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 3)
    res = []
    for pipe in (False, True):
        p, port = _start()
        try:
            with GarblerClient("127.0.0.1", port, c, 7, 100.0, batch=3, seed=b"p" * 16, pipeline=pipe) as cl:
                cl.offline()
                res.append((np.stack(cl.infer(xs)), cl.stats["offline_bytes"]))
        finally:
            p.join(timeout=60)
    np.testing.assert_array_equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1]


def test_ipc_transport_needs_a_gpu_garbler():
    """transport='ipc' writes tables from the garbler's GPU into the evaluator's slots: refused without a device."""
    c = build_circuit("MODEL_A")
    with pytest.raises(ValueError, match="device"):
        GarblerClient("127.0.0.1", 1, c, 7, 100.0, transport="ipc")


def test_skeleton_of_host_model_is_the_full_message():
    """A host-garbled model has no slot-resident tables: its skeleton is the whole offline message, and the
    skeleton reader parses ordinary blobs."""
    from dash_amd.garbling import GarbledCircuit
    from dash_amd.native import native

    gc = GarbledCircuit(build_circuit("MODEL_A"), 7, 100.0, seed=b"k" * 16)
    blob = gc.model.serialize()
    assert gc.model.serialize_skeleton() == blob
    assert native().GarbledModel.deserialize_skeleton(blob).serialize() == blob


def _ipc_server(port_q):
    s = listen("127.0.0.1", 0)
    port_q.put(s.getsockname()[1])
    serve_once(s, backend="hip", device=0)
    s.close()


@pytest.mark.gpu
def test_ipc_transport_two_processes():
    """Device transport: the evaluator (a child process, HIP) exports its table arenas' IPC handles; the garbler
    (this process, GPU garbler) writes every GC's tables straight into the evaluator's slots and sends skeletons
    only. Two rounds of 2 fresh GCs decode to the plaintext outputs, and the offline bytes on the channel are a
    fraction of what four full offline messages would take."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_ipc_server, args=(q,), daemon=True)
    p.start()
    port = q.get(timeout=300)
    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 4)
    try:
        with GarblerClient("127.0.0.1", port, c, 7, 100.0, batch=2, seed=b"i" * 16, device=0,
                           transport="ipc") as cl:
            for r in range(2):
                cl.offline()
                outs = cl.infer(xs[2 * r:2 * r + 2])
                for x, y in zip(xs[2 * r:2 * r + 2], outs):
                    np.testing.assert_array_equal(y, _plain(c, x))
            from dash_amd.garbling import GarbledCircuit

            full = len(GarbledCircuit(c, 7, 100.0, seed=b"f" * 16).model.serialize())
            assert cl.stats["offline_bytes"] < 4 * full  # 5 skeletons (one template) vs 4 full offline messages
    finally:
        p.join(timeout=120)
    assert p.exitcode == 0
