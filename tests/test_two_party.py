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
