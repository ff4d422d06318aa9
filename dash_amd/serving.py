"""Production serving engine: pipelined offline/online phases, watchdogs and
discard-and-re-garble recovery.

The reference has no serving loop, no health checks and no recovery
(SURVEY §5.3): its only failure detector is the decoding integrity check
(`garbled_circuit_interface.h:431-453`, which prints and asserts), and every
benchmark garbles one GC, evaluates it and throws it away
(`benchmarks/model_benchmarks/non_sgx/main.cpp:27-92`). This module turns the
same primitives into a long-running service on one MI355X:

* **GC slot pool.** A GC is single use (re-evaluating it with another input
  leaks the global offsets R_p), so the service keeps ``groups`` HIP evaluators
  of ``slots_per_group`` slots each; a slot holds one fresh garbled model whose
  tables live in HBM. The slots that received an input in a batch are spent
  and re-garbled; slots a short batch left unused keep their GC (never encoded,
  so nothing about it was revealed). Failed inputs join the next batch.
* **Offline/online pipeline.** A background garbler thread re-garbles stale
  groups (on the GPU garbler or the host garbler) and streams them into their
  HBM slots while the online path evaluates the other groups, so in steady
  state the online latency never waits for garbling unless the pool drains.
* **Watchdog.** Every online evaluation waits on its stream with a deadline
  (native ``hip_stream_wait``: hipStreamQuery polling with the GIL released)
  instead of an unbounded synchronize; a hung step raises ``WatchdogTimeout``
  and marks the service unhealthy (a hung GPU cannot be recovered in-process:
  the supervisor — torchrun elastic or the operator — restarts the rank).
  ``Watchdog`` additionally guards arbitrary host sections (e.g. collectives).
* **Recovery.** A decode integrity failure (``IntegrityError``: a corrupted
  table, label or message) discards the GC and resubmits the input on a fresh
  GC, up to ``max_retries`` times; failures and retries are counted.
* **Metrics.** Latency percentiles, throughput, retries, integrity failures and
  timeouts as one JSON-serialisable dict (``stats()``).

Backends: ``"hip"`` (MI355X, batched HIP evaluator) and ``"cpu"`` (the native
host evaluator, used by the CPU tests).
"""
from __future__ import annotations

import hashlib
import os
import queue
import threading
import time
from contextlib import contextmanager
from dataclasses import dataclass, field
from collections import deque
from typing import Callable, Deque, List, Optional, Sequence

import numpy as np

from .native import native


class WatchdogTimeout(RuntimeError):
    """A guarded section (GPU step, collective) exceeded its deadline."""


class Watchdog:
    """Deadline monitor for host-side sections.

    ``with wd.guard("allgather", 30): ...`` registers a deadline; a monitor
    thread calls ``on_timeout(name, elapsed_s)`` once if the section is still
    running after its deadline. The default handler records the event; pass
    ``abort_exit_code`` to terminate the process instead (the only way out of a
    call blocked inside the driver; ``os._exit`` does not exec, so it is safe
    after GPU initialisation)."""

    def __init__(self, on_timeout: Optional[Callable[[str, float], None]] = None, poll_s: float = 0.05,
                 abort_exit_code: Optional[int] = None):
        self.events: List[tuple] = []
        self._on_timeout = on_timeout
        self._abort = abort_exit_code
        self._poll = poll_s
        self._lock = threading.Lock()
        self._active: dict = {}
        self._next = 0
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="dash-watchdog", daemon=True)
        self._thread.start()

    def _run(self) -> None:
        while not self._stop.wait(self._poll):
            now = time.monotonic()
            fired = []
            with self._lock:
                for key, (name, t0, deadline) in list(self._active.items()):
                    if now > deadline:
                        fired.append((name, now - t0))
                        del self._active[key]
            for name, dt in fired:
                self.events.append((name, dt))
                if self._on_timeout is not None:
                    self._on_timeout(name, dt)
                if self._abort is not None:
                    os._exit(self._abort)

    @contextmanager
    def guard(self, name: str, timeout_s: float):
        with self._lock:
            key = self._next
            self._next += 1
            t0 = time.monotonic()
            self._active[key] = (name, t0, t0 + timeout_s)
        try:
            yield
        finally:
            with self._lock:
                fired = key not in self._active
                self._active.pop(key, None)
        if fired:
            raise WatchdogTimeout(f"{name} exceeded its {timeout_s:.3g} s deadline")

    def close(self) -> None:
        self._stop.set()
        self._thread.join(timeout=1.0)


def wait_stream(stream, timeout_s: float, what: str = "GPU step") -> None:
    """Bounded wait for a HIP stream (handle, torch stream or None = current)."""
    from .runtime import _stream_handle

    if not native().hip_stream_wait(_stream_handle(stream), float(timeout_s)):
        raise WatchdogTimeout(f"{what} still running after {timeout_s:.3g} s (GPU hang?)")


#: batch latencies kept for the percentiles (a long-running service must not grow without bound)
LATENCY_WINDOW = 4096


@dataclass
class ServiceStats:
    inferences: int = 0
    batches: int = 0
    retries: int = 0
    integrity_failures: int = 0
    timeouts: int = 0
    range_refusals: int = 0  # batches refused by the garbler's range guard (garbling/guard.py)
    gcs_garbled: int = 0
    garble_s: float = 0.0
    pool_waits_s: float = 0.0
    latencies_ms: Deque[float] = field(default_factory=lambda: deque(maxlen=LATENCY_WINDOW))
    t_start: float = field(default_factory=time.perf_counter)
    encoding: Optional[str] = None  # offline-message encoding of the served GCs: "hardened" | "reference"
    input_encoding: Optional[str] = None  # online message #1: "device" (garbler's device encoder) | "host"

    def as_dict(self) -> dict:
        lat = np.asarray(self.latencies_ms, dtype=np.float64)
        wall = time.perf_counter() - self.t_start

        def pct(q):
            return round(float(np.percentile(lat, q)), 3) if lat.size else None

        return {
            "inferences": self.inferences, "batches": self.batches, "retries": self.retries,
            "integrity_failures": self.integrity_failures, "timeouts": self.timeouts,
            "range_refusals": self.range_refusals,
            "gcs_garbled": self.gcs_garbled, "garble_s_per_gc": round(self.garble_s / max(1, self.gcs_garbled), 4),
            "pool_wait_s": round(self.pool_waits_s, 3),
            # percentiles over the last LATENCY_WINDOW batches
            "batch_latency_ms": {"p50": pct(50), "p90": pct(90), "p99": pct(99), "max": pct(100)},
            "inferences_per_s_wall": round(self.inferences / wall, 3) if wall > 0 else None,
            "encoding": self.encoding, "input_encoding": self.input_encoding,
        }


class _Group:
    """One evaluator (``slots`` GC slots) plus the garbler-side state of its GCs."""

    def __init__(self, idx: int, slots: int):
        self.idx = idx
        self.slots = slots
        self.ev = None          # HipEvaluator (hip backend)
        self.gcs: list = [None] * slots
        self.enc = None         # the garbler's device input encoder, one slot per GC slot (input_encoding="device")
        self.ready = threading.Event()
        self.stream = None
        self.runs = 0           # evaluations so far (run 2 captures the hipGraph)
        self.lock = threading.Lock()
        self.pending = 0        # spent slots still being refilled


class InferenceService:
    """Long-running garbled-inference service on one GPU (or the host).

    ``infer(xs)`` takes any number of quantized inputs and returns their
    decoded logits ``[len(xs), n_out]`` in order; each input is evaluated on a
    fresh GC. ``fault_hook(global_index, attempt) -> bool`` (tests / chaos
    runs) corrupts that attempt's output message before decoding, which the
    integrity check must catch and the service must recover from.

    Thread safety: ``infer`` may be called from several request threads; calls
    are serialized by an internal lock (one batch at a time reaches the GPU
    groups, whose slot state is not shared across callers)."""

    def __init__(self, circuit, crt, mrs=None, *, max_modulus: int = 0, slots_per_group: int = 4, groups: int = 2,
                 backend: str = "hip", device: int = 0, garble_device: Optional[bool] = None, max_retries: int = 2,
                 step_timeout_s: float = 120.0, seed: Optional[bytes] = None, prefetch: bool = True,
                 fault_hook: Optional[Callable[[int, int], bool]] = None, nthreads: int = 0,
                 rescale: str = "auto", relu: str = "auto", fused_sign: bool = True,
                 insecure_fixed_seed: bool = False, garble_workers: Optional[int] = None,
                 input_encoding: Optional[str] = None, hardened: Optional[bool] = None):
        if backend not in ("hip", "cpu"):
            raise ValueError("backend must be 'hip' or 'cpu'")
        if seed is not None and not insecure_fixed_seed:
            # a fixed seed replays the same GC label / offset sequence after every restart, on new inputs
            raise ValueError("InferenceService(seed=...) reuses garbling randomness across restarts; pass "
                             "insecure_fixed_seed=True to accept that (tests / reproducible benchmarks only)")
        if backend == "hip" and native().hip_device_count() == 0:
            raise RuntimeError("InferenceService(backend='hip') needs a visible MI355X")
        self.circuit, self.crt, self.mrs, self.max_modulus = circuit, crt, mrs, max_modulus
        self.backend, self.device = backend, device
        self.garble_device = (backend == "hip") if garble_device is None else bool(garble_device)
        # online message #1: "device" = the garbler's device encoder writes each slot's input labels on the GPU
        # (GarbledCircuit.device_input_encoder, re-armed per GC); "host" = compressed labels + H2D + GPU unpack
        enc = input_encoding or os.environ.get("DASH_SERVE_INPUT_ENCODING", "device")
        if enc not in ("device", "host"):
            raise ValueError("input_encoding must be 'device' or 'host'")
        self.device_encode = backend == "hip" and enc == "device"
        self.max_retries, self.step_timeout_s = max_retries, step_timeout_s
        self.fault_hook = fault_hook
        self.nthreads = nthreads
        # gadget constructions (GarbledCircuit): the serving default is the fastest measured one
        # hardened=None: the hardened encoding whenever the constructions allow it; the reference encoding
        # (R_p recoverable from its constant labels, docs/SECURITY.md §1.1) only when asked for explicitly
        if hardened is None:
            from .garbling.gc import hardened_supported, resolve_constructions
            from .ir.bases import first_primes

            base = first_primes(crt) if isinstance(crt, int) else [int(p) for p in crt]
            r, _ = resolve_constructions(circuit, base, rescale, relu, fused_sign, None)
            if not hardened_supported(circuit, fused_sign, r):
                raise ValueError("InferenceService: these constructions (fused_sign=%s, rescale=%s) only have the "
                                 "reference encoding, whose constant labels reveal R_p (docs/SECURITY.md §1.1); pass "
                                 "hardened=False to serve it anyway" % (fused_sign, r))
        self.gc_kw = dict(rescale=rescale, relu=relu, fused_sign=fused_sign, hardened=hardened)
        self._seed = seed if seed is not None else os.urandom(16)
        self._ctr = 0
        self.stats = ServiceStats()
        self.stats.input_encoding = "device" if self.device_encode else ("host" if backend == "hip" else "labels")
        self.healthy = True
        self.groups = [_Group(g, slots_per_group) for g in range(groups)]
        # background refill workers: with the GPU garbler eight GCs garble at once on eight streams of the device
        # (garble_gpu.hip DevCtx pool), filling each other's kernel-launch gaps and latency stalls
        # (served inf/s with 5 % faults, 2 / 3 / 4 workers: 88 / 104 / 110, profiles/r03_serving_workers_*.json;
        # round 6, bench served phase, 4 / 6 / 8 / 12 / 16 workers: 172-178 / 181-193 / 190-201 / 188-192 /
        # 188-190, profiles/ab/r6/r06z{c,d}_*.json)
        self.garble_workers = max(1, int(garble_workers if garble_workers is not None else
                                         int(os.environ.get("DASH_GARBLE_WORKERS", "0")) or
                                         (8 if self.garble_device else 1)))
        self._ctr_lock = threading.Lock()
        self._next_group = 0
        self._err: Optional[BaseException] = None
        # hipGraph capture (a group's 2nd run) must not overlap the garbler thread's device-wide syncs and
        # allocations, which would invalidate the capture; replays and eager runs need no lock
        self._capture_lock = threading.Lock()
        self._infer_lock = threading.Lock()
        self._q: "queue.Queue" = queue.Queue()  # (group, slot) refill items; None stops a worker
        if backend == "hip":
            import torch

            torch.cuda.set_device(device)
            self._streams = [native().hip_stream_create(0) for _ in range(groups)]
            for g, st in zip(self.groups, self._streams):
                g.stream = st
        # fill the pool once synchronously (first GC also sizes the evaluators), then refill in the background
        for g in self.groups:
            self._refill(g)
        if backend == "hip":
            self._prime_graphs()
        self._workers: List[threading.Thread] = []
        if prefetch:
            for w in range(self.garble_workers):
                t = threading.Thread(target=self._garbler_loop, name=f"dash-garbler-{w}", daemon=True)
                t.start()
                self._workers.append(t)

    @property
    def _worker(self):  # the first refill worker (None without prefetch)
        return self._workers[0] if self._workers else None

    # ------------------------------------------------------------ offline
    def _new_gc(self, sink=None):
        from .garbling import GarbledCircuit

        with self._ctr_lock:
            seed = hashlib.sha256(self._seed + self._ctr.to_bytes(8, "little")).digest()[:16]
            self._ctr += 1
        t = time.perf_counter()
        gc = GarbledCircuit(self.circuit, self.crt, self.mrs, max_modulus=self.max_modulus, seed=seed,
                            nthreads=self.nthreads, device=self.device if self.garble_device else None,
                            sink=sink if self.garble_device else None, **self.gc_kw)
        with self._ctr_lock:
            self.stats.garble_s += time.perf_counter() - t
            self.stats.gcs_garbled += 1
        return gc

    def _prime_graphs(self) -> None:
        """Capture every group's hipGraph now, before the background garbler starts.

        A group's first run is eager and its second run captures the graph; the
        capture must not overlap the garbler thread's device-wide syncs and
        allocations. Doing both runs here (no input is encoded, so no GC is
        spent: the activations hold zeros) means the online path never takes
        the capture lock, and a refill never stalls an online step."""
        for g in self.groups:
            for _ in range(2):
                g.ev.run(g.stream)
            g.runs = 2
            wait_stream(g.stream, self.step_timeout_s, f"group {g.idx} graph capture")

    def _refill_slot(self, g: _Group, b: int) -> None:
        if self.backend == "hip":
            from .runtime import HipEvaluator

            if g.ev is None:
                with self._capture_lock:  # first fill: evaluator allocation and its device-wide setup
                    gc = self._new_gc()
                    if g.ev is None:
                        g.ev = HipEvaluator(template=gc.model, batch=g.slots, device=self.device)
            else:
                # the GPU garbler writes the tables straight into the slot (zero-copy load) on its own stream:
                # no device-wide synchronization, so refills overlap the other groups' evaluations
                gc = self._new_gc(g.ev.sink(b))
            g.ev.load(b, gc.model)
            gc.model = None  # tables live in HBM now
            if self.device_encode:  # the garbler's input state of this GC to the GPU (offline, with its tables)
                if g.enc is None:  # arms only slot b (this GC's evaluator slot); the others load their own GCs
                    g.enc = gc.device_input_encoder(self.device, g.slots, slot=b)
                else:
                    g.enc.load(gc.garbler, b)
        else:
            gc = self._new_gc()
        g.gcs[b] = gc
        if self.stats.encoding is None:
            self.stats.encoding = "hardened" if gc.hardened else "reference"

    def _refill(self, g: _Group) -> None:
        for b in range(g.slots):
            if g.gcs[b] is None:  # a non-None GC was never encoded: still fresh
                self._refill_slot(g, b)
        g.ready.set()

    def _garbler_loop(self) -> None:
        while True:
            item = self._q.get()
            if item is None or not self.healthy:
                return
            g, b = item
            try:
                self._refill_slot(g, b)
                with g.lock:
                    g.pending -= 1
                    done = g.pending == 0
                if done:
                    g.ready.set()
            except BaseException as e:  # surfaced by the next infer()
                self._err = e
                self.healthy = False
                for other in self.groups:  # wake every waiter: none of them will be refilled
                    other.ready.set()
                return

    def _take_group(self) -> _Group:
        g = self.groups[self._next_group]
        self._next_group = (self._next_group + 1) % len(self.groups)
        if not g.ready.is_set():
            if self._worker is None:
                self._refill(g)
            else:
                t = time.perf_counter()
                while not g.ready.wait(0.5):  # re-check for a dead garbler thread
                    if self._err is not None:
                        break
                self.stats.pool_waits_s += time.perf_counter() - t
        if self._err is not None:
            raise RuntimeError("background garbler failed") from self._err
        return g

    def _release(self, g: _Group, used: int) -> None:
        # only the slots that received an input are spent; an unused slot was never encoded for its GC (its
        # staging still holds labels of an older, unrelated GC), so its GC stays valid for the next batch
        for b in range(used):
            g.gcs[b] = None
        g.ready.clear()
        # an unhealthy service (hung GPU step or dead garbler) never refills: the refill would block on the
        # hung kernel
        if self._workers and self.healthy:
            with g.lock:
                g.pending = used
            for b in range(used):  # one item per spent slot: the workers garble a group's slots in parallel
                self._q.put((g, b))

    # ------------------------------------------------------------- online
    def _run_group(self, g: _Group, xs: Sequence[np.ndarray], idx: Sequence[int], attempts: Sequence[int]):
        """Evaluate len(xs) <= slots inputs on group g. Returns per-input logits or None on integrity failure."""
        from . import IntegrityError

        out: list = [None] * len(xs)
        t = time.perf_counter()
        if self.backend == "hip":
            ev = g.ev
            if self.device_encode:  # unused slots are not encoded (see _release)
                ev.encode_device_into(0, g.enc, np.stack([np.asarray(x).reshape(-1) for x in xs]), g.stream)
            else:
                for b in range(len(xs)):
                    ev.encode_compressed_into(b, g.gcs[b], xs[b], guarded=True)  # batch guard below
                ev.upload_inputs_compressed(g.stream)
            ev.run(g.stream)  # graph replay: captured in _prime_graphs
            g.runs += 1
            # the garbler's exact range guard (mixed-radix wrap band, CRT overflow) on a side stream, overlapping
            # the evaluation: a refused input raises RangeGuardError before any result of the batch is released
            gc0 = g.gcs[0]
            pend = gc0.guard.submit(xs) if gc0.guard_enabled else None
            try:
                wait_stream(g.stream, self.step_timeout_s, f"group {g.idx} evaluation")
            except WatchdogTimeout:
                self.stats.timeouts += 1
                self.healthy = False
                raise
            ev.fetch_outputs(g.stream)
            for b in range(len(xs)):
                msg = np.array(ev.outputs_compressed(b), copy=True)
                if self.fault_hook is not None and self.fault_hook(idx[b], attempts[b]):
                    msg[0, 0, 0] ^= np.uint64(1) << np.uint64(9)
                try:
                    out[b] = np.asarray(g.gcs[b].decode_compressed(msg))
                except IntegrityError:
                    self.stats.integrity_failures += 1
            if pend is not None:
                try:
                    pend.raise_if_bad()
                except ValueError:
                    self.stats.range_refusals += 1
                    raise
        else:
            for b, x in enumerate(xs):
                gc = g.gcs[b]
                labels = gc.cpu_evaluate(gc.garble_inputs(x), self.nthreads)
                if self.fault_hook is not None and self.fault_hook(idx[b], attempts[b]):
                    p, arr = labels[0]
                    arr = np.array(arr, copy=True)
                    arr.flat[0] = (int(arr.flat[0]) + 1) % int(p)
                    labels = [(p, arr)] + list(labels[1:])
                try:
                    out[b] = np.asarray(gc.decode_outputs(labels))
                except IntegrityError:
                    self.stats.integrity_failures += 1
        self.stats.latencies_ms.append(1000.0 * (time.perf_counter() - t))
        self.stats.batches += 1
        return out

    def infer(self, xs: Sequence[np.ndarray]) -> np.ndarray:
        with self._infer_lock:
            return self._infer(xs)

    def _infer(self, xs: Sequence[np.ndarray]) -> np.ndarray:
        from . import IntegrityError

        if self._err is not None:
            raise RuntimeError("background garbler failed; restart the rank") from self._err
        if not self.healthy:
            raise RuntimeError("service is unhealthy (a GPU step timed out); restart the rank")
        xs = [np.asarray(x, dtype=np.int64).reshape(-1) for x in xs]
        results: list = [None] * len(xs)
        pending = deque((i, 0) for i in range(len(xs)))  # (input, attempt); retries join later batches
        slots = self.groups[0].slots
        while pending:
            batch = [pending.popleft() for _ in range(min(slots, len(pending)))]
            g = self._take_group()
            try:
                out = self._run_group(g, [xs[i] for i, _ in batch], [i for i, _ in batch], [a for _, a in batch])
            finally:
                self._release(g, len(batch))  # single use: the GCs that saw an input are discarded, then re-garbled
            for (i, a), y in zip(batch, out):
                if y is not None:
                    results[i] = y
                    self.stats.inferences += 1
                elif a + 1 > self.max_retries:
                    raise IntegrityError(f"input {i} failed the integrity check {a + 1} times")
                else:
                    self.stats.retries += 1
                    pending.append((i, a + 1))
        return np.stack(results)

    def close(self, join_timeout_s: float = 30.0) -> None:
        """Stop the garbler thread and free the GPU state.

        An unhealthy service (a hung GPU step) only drops its references to the
        pool: freeing device memory or destroying streams would block on the
        hung kernel. The garbler thread is a daemon, so the process can still
        exit (non-zero) and the supervisor restarts the rank."""
        if self._workers:
            while True:  # drop pending refills: the pool is going away
                try:
                    self._q.get_nowait()
                except queue.Empty:
                    break
            for _ in self._workers:
                self._q.put(None)
            for t in self._workers:
                t.join(timeout=join_timeout_s if self.healthy else 1.0)
            self._workers = []
        if not self.healthy:
            self._abandoned = (self.groups, getattr(self, "_streams", []))  # never freed, see above
            self.groups, self._streams = [], []
            return
        for g in self.groups:
            g.ev = None
            g.gcs = [None] * g.slots
        if self.backend == "hip":
            if self.garble_device:
                native().gpu_table_cache_trim()
            for st in self._streams:
                native().hip_stream_destroy(st)
            self._streams = []

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
