"""Serving engine: GC slot pool with background re-garbling, integrity-failure
recovery (discard + re-garble + resubmit), watchdogs.

The reference has no equivalent (its only failure detector is the decode
assert, garbled_circuit_interface.h:431-453); parity of the decoded logits is
pinned against the plaintext quantized evaluation (`plain_q_eval`)."""
import time

import numpy as np
import pytest

import dash_amd as d
from dash_amd.models import build_circuit, quantized_inputs
from dash_amd.serving import InferenceService, Watchdog, WatchdogTimeout


@pytest.fixture(scope="module")
def small():
    from dash_amd.ir.quant import QuantizationMethod as Q

    c = build_circuit("MODEL_B_POOL_REPL", Q.ScaleQuant, 3, seed=2)
    xs = quantized_inputs("MODEL_B_POOL_REPL", 7, Q.ScaleQuant, 3)
    return c, xs


def _ref(c, xs):
    from dash_amd.garbling import GarbledCircuit

    gc = GarbledCircuit(c, 8, 100.0, seed=b"r" * 16)
    return np.stack([gc.plain_q_eval(x) for x in xs])


@pytest.mark.parametrize("prefetch", [True, False])
def test_service_cpu_matches_plaintext(small, prefetch):
    c, xs = small
    with InferenceService(c, 8, 100.0, hardened=False, backend="cpu", slots_per_group=2, groups=2, prefetch=prefetch,
                          seed=b"p" * 16, insecure_fixed_seed=True) as svc:
        y = svc.infer(xs)          # 7 inputs -> 4 groups of <= 2 (pool cycles, re-garbled in the background)
        y2 = svc.infer(xs[:3])
        st = svc.stats.as_dict()
    np.testing.assert_array_equal(y, _ref(c, xs))
    np.testing.assert_array_equal(y2, _ref(c, xs[:3]))
    assert st["inferences"] == 10 and st["retries"] == 0 and st["integrity_failures"] == 0
    # every inference on its own GC; the pool was refilled after each batch
    assert st["gcs_garbled"] >= 10
    assert st["batch_latency_ms"]["p50"] is not None


def test_service_recovers_from_integrity_failures(small):
    c, xs = small
    hits = []

    def fault(i, attempt):  # corrupt the first attempt of inputs 1 and 4, and two attempts of input 5
        bad = (i in (1, 4) and attempt == 0) or (i == 5 and attempt < 2)
        if bad:
            hits.append((i, attempt))
        return bad

    with InferenceService(c, 8, 100.0, hardened=False, backend="cpu", slots_per_group=3, groups=2, fault_hook=fault,
                          max_retries=2, seed=b"f" * 16, insecure_fixed_seed=True) as svc:
        y = svc.infer(xs)
        st = svc.stats.as_dict()
    np.testing.assert_array_equal(y, _ref(c, xs))
    assert st["integrity_failures"] == 4 and st["retries"] == 4
    assert sorted(hits) == [(1, 0), (4, 0), (5, 0), (5, 1)]


def test_service_gives_up_after_max_retries(small):
    c, xs = small
    with InferenceService(c, 8, 100.0, hardened=False, backend="cpu", slots_per_group=2, groups=1, prefetch=False,
                          fault_hook=lambda i, a: i == 0, max_retries=1, seed=b"g" * 16, insecure_fixed_seed=True) as svc:
        with pytest.raises(d.IntegrityError):
            svc.infer(xs[:2])
        assert svc.stats.integrity_failures == 2


def test_watchdog_fires_and_passes():
    seen = []
    wd = Watchdog(on_timeout=lambda n, dt: seen.append(n), poll_s=0.01)
    try:
        with wd.guard("fast", 5.0):
            pass
        with pytest.raises(WatchdogTimeout):
            with wd.guard("slow", 0.05):
                time.sleep(0.3)
        assert seen == ["slow"] and wd.events[0][0] == "slow"
    finally:
        wd.close()


def test_dist_init_timeout_gloo(tmp_path):
    """Collectives get a finite timeout (RCCL/gloo) instead of hanging forever."""
    import os

    import torch.multiprocessing as mp

    port = 29500 + (os.getpid() % 1000)
    mp.spawn(_timeout_worker, args=(2, port), nprocs=2, join=True)


def _timeout_worker(rank, world, port):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from dash_amd.parallel import init_distributed, shutdown

    ctx = init_distributed(backend="gloo", use_gpu=False, timeout_s=5.0)
    try:
        # rank 1 never joins the second barrier: rank 0 must time out, not hang
        dist.barrier()
        if rank == 0:
            t = time.time()
            with pytest.raises(RuntimeError):
                dist.barrier()
            assert time.time() - t < 60
    finally:
        if rank == 1:
            time.sleep(8)
        shutdown(ctx)


@pytest.mark.gpu
@pytest.mark.parametrize("enc", ["device", "host"])
def test_service_hip_matches_plaintext_and_recovers(small, enc):
    c, xs = small
    with InferenceService(c, 8, 100.0, hardened=False, backend="hip", slots_per_group=2, groups=2, device=0, seed=b"h" * 16, insecure_fixed_seed=True,
                          fault_hook=lambda i, a: i == 2 and a == 0, step_timeout_s=60, input_encoding=enc) as svc:
        assert svc.device_encode == (enc == "device")
        y = svc.infer(xs)
        st = svc.stats.as_dict()
    np.testing.assert_array_equal(y, _ref(c, xs))
    assert st["integrity_failures"] == 1 and st["retries"] == 1 and st["timeouts"] == 0


@pytest.mark.gpu
def test_service_hip_concurrent_refill_no_spurious_failures(small):
    """Regression (HipEvaluator.load serialization, runtime.hip load_mu_): 4 refill workers loading slots of the
    same evaluators concurrently, no injected faults -> no integrity failure, no retry, exact outputs."""
    c, xs = small
    xs4 = [xs[i % len(xs)] for i in range(24)]
    with InferenceService(c, 8, 100.0, hardened=False, backend="hip", slots_per_group=4, groups=2, device=0, garble_workers=4,
                          seed=b"c" * 16, insecure_fixed_seed=True, step_timeout_s=60) as svc:
        ys = [svc.infer(xs4[i:i + 8]) for i in range(0, 24, 8)]
        st = svc.stats.as_dict()
    np.testing.assert_array_equal(np.concatenate(ys), _ref(c, xs4))
    assert st["integrity_failures"] == 0 and st["retries"] == 0 and st["timeouts"] == 0


@pytest.mark.gpu
def test_sink_model_orphaned_by_evaluator_raises(small):
    """A GC garbled into an evaluator slot (sink) aliases that evaluator's HBM: after the evaluator is gone its
    tables must refuse a host read instead of reading freed memory."""
    import gc as pygc

    from dash_amd.garbling import GarbledCircuit
    from dash_amd.runtime import HipEvaluator

    c, xs = small
    g0 = GarbledCircuit(c, 8, 100.0, seed=b"s" * 16, device=0)
    ev = HipEvaluator(template=g0.model, batch=1, device=0)
    g1 = GarbledCircuit(c, 8, 100.0, seed=b"t" * 16, device=0, sink=ev.sink(0))
    ev.load(0, g1.model)
    del ev
    pygc.collect()
    with pytest.raises(RuntimeError, match="destroyed HipEvaluator"):
        g1.model.serialize()


@pytest.mark.gpu
def test_hip_stream_wait_bounded():
    from dash_amd.native import native

    st = native().hip_stream_create(0)
    try:
        assert native().hip_stream_wait(st, 5.0)  # idle stream drains immediately
    finally:
        native().hip_stream_destroy(st)


def test_cli_run_service(capsys):
    from dash_amd.__main__ import main

    main(["run-service", "--model", "MODEL_A", "--scheme", "SIMPLE", "--backend", "cpu", "--batch", "2",
          "--groups", "2", "--inputs", "3", "--seed", "00" * 16, "--insecure-fixed-seed"])
    out = capsys.readouterr().out
    import json

    stats = json.loads(out.strip().splitlines()[-1])
    assert stats["inferences"] == 3 and stats["integrity_failures"] == 0


def test_cli_run_service_refuses_fixed_seed():
    from dash_amd.__main__ import main

    with pytest.raises(SystemExit):
        main(["run-service", "--model", "MODEL_A", "--scheme", "SIMPLE", "--backend", "cpu", "--inputs", "1",
              "--seed", "11" * 16])


def test_seed_bytes_accepts_json_decoded_digits():
    from dash_amd.config import DashConfig, _parse_value

    assert DashConfig(seed=_parse_value("11" * 16)).seed_bytes() == bytes([0x11]) * 16
    assert DashConfig(seed=_parse_value("0a" * 16)).seed_bytes() == bytes([0x0A]) * 16
    assert DashConfig(seed=7).seed_bytes() == bytes(15) + b"\x07"
    assert DashConfig(seed=None).seed_bytes() is None


def test_latency_history_is_bounded():
    from dash_amd.serving import LATENCY_WINDOW, ServiceStats

    st = ServiceStats()
    for i in range(LATENCY_WINDOW + 100):
        st.latencies_ms.append(float(i))
    assert len(st.latencies_ms) == LATENCY_WINDOW
    assert st.as_dict()["batch_latency_ms"]["max"] == float(LATENCY_WINDOW + 99)


def test_timeout_is_not_requeued_and_close_returns(small, monkeypatch):
    """A hung GPU step (faked: _run_group raises WatchdogTimeout) marks the service unhealthy; the hung group
    is not handed to the garbler (whose refill would block on the hung kernel) and close() returns."""
    import threading

    c, xs = small
    svc = InferenceService(c, 8, 100.0, hardened=False, backend="cpu", slots_per_group=2, groups=2, seed=b"t" * 16, insecure_fixed_seed=True)
    hang = threading.Event()
    refills = []

    def hung_refill(g):  # stands in for a refill stuck in hipDeviceSynchronize
        refills.append(g.idx)
        hang.wait()

    def timed_out(g, *a, **k):
        svc.stats.timeouts += 1
        svc.healthy = False
        raise WatchdogTimeout("faked GPU hang")

    monkeypatch.setattr(svc, "_refill", hung_refill)
    monkeypatch.setattr(svc, "_run_group", timed_out)
    with pytest.raises(WatchdogTimeout):
        svc.infer(xs[:2])
    with pytest.raises(RuntimeError, match="unhealthy"):
        svc.infer(xs[:2])
    t = time.time()
    svc.close()
    assert time.time() - t < 10
    assert refills == []  # never re-queued
    hang.set()


def test_garbler_failure_wakes_every_waiter(small, monkeypatch):
    """A dead background garbler fails every later infer() promptly instead of blocking on a group that
    will never be refilled."""
    c, xs = small
    svc = InferenceService(c, 8, 100.0, hardened=False, backend="cpu", slots_per_group=1, groups=3, seed=b"w" * 16, insecure_fixed_seed=True)

    def boom():
        raise OSError("garbler died")

    monkeypatch.setattr(svc, "_new_gc", boom)
    t = time.time()
    with pytest.raises(RuntimeError):
        svc.infer(xs[:6])  # 6 batches of 1 over 3 groups: needs refills
    with pytest.raises(RuntimeError):
        svc.infer(xs[:1])
    assert not svc.healthy
    assert time.time() - t < 30
    svc.close()
