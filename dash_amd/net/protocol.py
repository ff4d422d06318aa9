"""Garbler/evaluator protocol over a `Channel`.

Messages (tags):
  HELO  client -> server  JSON {"version", "batch"};   server -> client JSON {"backend", "device"}
  MODL  client -> server  flags = slot, payload = GarbledModel.serialize()      (offline)
  MODS  client -> server  flags = slot, payload = JSON {"name", "size"}: the same offline message in a shared
                          memory segment of the garbler's ring (same-host split; the evaluator ACKs once it has
                          loaded it, after which the garbler reuses the segment)
  TMPL  client -> server  payload = skeleton of one GC (GarbledModel.serialize_skeleton(all_device=True)): the
                          HIP evaluator is built from it; server -> client IPCH = JSON [[layer, table, bytes per
                          slot, IPC handle hex], ...] of its table arenas (device transport "ipc")
  MODX  client -> server  flags = slot, payload = skeleton of a GC whose tables the garbler's GPU wrote straight
                          into that slot through the IPC handles (same node: same device or a peer over xGMI)
  INPT  client -> server  flags = n, payload = n x (k, N, 2) uint64 compressed input labels   (online #1)
  OUTP  server -> client  payload = n x (k, n_out, 2) uint64 compressed output labels          (online #2)
  BYE_  either side
  ERR!  server -> client  UTF-8 error text

A garbled model is single use (reusing its labels on a second input would
leak the offsets R_p): the server drops every slot after one
INPT round and refuses a second round on the same slots. The online traffic
per inference is exactly input_size*k*16 B + n_out*k*16 B plus framing, the
"single online round" of the reference's communication model
(benchmarks/evaluation.ipynb:895-950).
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional, Sequence

import numpy as np

from ..native import native
from .channel import Channel, ChannelClosed, connect

VERSION = 1
# Largest table arena the ipc transport exports: importing a bigger dmabuf-backed allocation
# (hipIpcOpenMemHandle) never returned on the MI355X lease (MiniONN at batch 4 and 8: 2.2 and 4.5 GB arenas),
# while 1.1 GB arenas open at once. The server refuses a larger one with a clear error instead of a hang.
IPC_MAX_ARENA = 2 << 30
_DEBUG = os.environ.get("DASH_NET_DEBUG") == "1"


def _dbg(msg: str) -> None:
    if _DEBUG:
        import sys

        print(f"[dash.net {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


class EvaluatorServer:
    """Evaluator party: receives garbled models, evaluates online rounds on
    the CPU oracle (`backend="cpu"`) or the HIP evaluator (`backend="hip"`)."""

    def __init__(self, backend: str = "cpu", device: int = 0, nthreads: int = 0, tamper: bool = False):
        assert backend in ("cpu", "hip")
        self.backend, self.device, self.nthreads = backend, device, nthreads
        self.tamper = tamper  # fault injection: flip one output bit (tests)
        self.input_digests: list = []  # sha256 of every online message #1 received (seed-reuse audits, tests)
        self._reset()

    def _reset(self):
        self.models: dict = {}
        self.ev = None
        self.batch = 1
        self.rounds = 0
        self._close_shm()

    def _close_shm(self):
        for mm in getattr(self, "_shm", {}).values():
            try:
                mm.close()
            except (OSError, BufferError):
                pass
        self._shm: dict = {}

    def _segment(self, name: str):
        """Read-only map of the garbler's POSIX shared-memory segment (its owner creates and unlinks it; mapped
        directly so that no resource tracker of this process claims it)."""
        mm = self._shm.get(name)
        if mm is None:
            import mmap

            if "/" in name.strip("/") or not name.strip("/"):
                raise ValueError("bad shared-memory segment name")
            fd = os.open("/dev/shm/" + name.strip("/"), os.O_RDONLY)
            try:
                mm = mmap.mmap(fd, 0, prot=mmap.PROT_READ)
            finally:
                os.close(fd)
            self._shm[name] = mm
        return mm

    def serve(self, ch: Channel) -> None:
        n = native()
        try:
            while True:
                try:
                    tag, flags, buf = ch.recv()
                except ChannelClosed:
                    return
                try:
                    if tag == b"HELO":
                        hello = json.loads(buf.decode())
                        if hello.get("version") != VERSION:
                            raise ValueError(f"protocol version {hello.get('version')} != {VERSION}")
                        self._reset()
                        self.batch = int(hello.get("batch", 1))
                        ch.send(b"HELO", json.dumps({"backend": self.backend, "device": self.device}).encode())
                    elif tag == b"TMPL":
                        if self.backend != "hip":
                            raise ValueError("the ipc transport needs the HIP evaluator")
                        from ..runtime import HipEvaluator

                        skel = n.GarbledModel.deserialize_skeleton(buf)
                        _dbg("server: TMPL received, building the evaluator")
                        if self.ev is None:
                            self.ev = HipEvaluator(template=skel, batch=self.batch, device=self.device)
                        ex = self.ev.ipc_export()
                        big = max((int(nb) * self.batch for _, _, nb, _ in ex), default=0)
                        if big >= IPC_MAX_ARENA:
                            raise ValueError(f"ipc transport: a {big / 2**30:.2f} GiB table arena (batch {self.batch}) is "
                                             f"above the {IPC_MAX_ARENA >> 30} GiB this transport opens; use a smaller "
                                             f"batch or transport 'shm'")
                        hs = [[int(l), str(t), int(nb), bytes(h).hex()] for l, t, nb, h in ex]
                        _dbg(f"server: exported {len(hs)} table arenas")
                        ch.send(b"IPCH", json.dumps(hs).encode())
                    elif tag == b"MODX":
                        slot = flags
                        if not 0 <= slot < self.batch:
                            raise ValueError(f"slot {slot} out of range")
                        if self.ev is None:
                            raise ValueError("MODX before TMPL: the evaluator has no table arenas yet")
                        self.ev.load(slot, n.GarbledModel.deserialize_skeleton(buf))
                        _dbg(f"server: MODX slot {slot} loaded")
                        del buf
                        self.models[slot] = True
                        ch.send(b"ACK_")
                    elif tag in (b"MODL", b"MODS"):
                        slot = flags
                        if not 0 <= slot < self.batch:
                            raise ValueError(f"slot {slot} out of range")
                        if tag == b"MODL":
                            m = n.GarbledModel.deserialize_buffer(buf)  # parsed in place, no bytes() copy
                        else:
                            ref = json.loads(buf.decode())
                            seg = self._segment(str(ref["name"]))
                            size = int(ref["size"])
                            if not 0 < size <= len(seg):
                                raise ValueError("shared-memory model size out of range")
                            view = memoryview(seg)[:size]
                            try:
                                m = n.GarbledModel.deserialize_buffer(view)
                            finally:
                                view.release()
                        del buf
                        if self.backend == "hip":
                            from ..runtime import HipEvaluator

                            if self.ev is None:
                                self.ev = HipEvaluator(template=m, batch=self.batch, device=self.device)
                            self.ev.load(slot, m)
                            self.models[slot] = True
                        else:
                            self.models[slot] = m
                        ch.send(b"ACK_")
                    elif tag == b"INPT":
                        ch.send(b"OUTP", self._round(flags, buf))
                    elif tag == b"BYE_":
                        self._close_shm()
                        return
                    else:
                        raise ValueError(f"unknown message {tag!r}")
                except Exception as e:  # report every failure to the peer, keep serving
                    ch.send(b"ERR!", f"{type(e).__name__}: {e}".encode())
        finally:
            self._close_shm()
            ch.close()

    def _round(self, nb: int, buf: bytearray) -> bytes:
        n = native()
        if nb != self.batch or len(self.models) != self.batch:
            raise ValueError(f"online round needs all {self.batch} slots garbled (have {sorted(self.models)})")
        import hashlib

        self.input_digests.append(hashlib.sha256(bytes(buf)).hexdigest())
        raw = np.frombuffer(buf, dtype=np.uint64)
        per = raw.size // nb
        outs = []
        if self.backend == "hip":
            ev = self.ev
            k = ev._h.crt_size()
            N = ev._h.input_size()
            assert per == k * N * 2, "input size mismatch"
            for b in range(nb):
                ev.set_input_compressed(b, raw[b * per:(b + 1) * per].reshape(k, N, 2))
            ev.upload_inputs_compressed()
            ev.run()
            ev.fetch_outputs()
            outs = [ev.outputs_compressed(b) for b in range(nb)]
        else:
            for b in range(nb):
                m = self.models[b]
                k = len(m.crt)
                N = int(np.prod(m.in_dims))
                assert per == k * N * 2, "input size mismatch"
                labels = n.decompress_labels(raw[b * per:(b + 1) * per].reshape(k, N, 2), list(m.crt))
                out = n.cpu_evaluate(m, labels, self.nthreads)
                outs.append(n.compress_labels(out))
        self.models.clear()  # single use
        self.rounds += 1
        payload = np.concatenate([o.reshape(-1) for o in outs])
        if self.tamper:
            payload = payload.copy()
            payload[0] ^= np.uint64(1)
        return payload.tobytes()


def serve_once(sock, backend: str = "cpu", device: int = 0, tamper: bool = False) -> None:
    """Accept one client on a listening socket and serve it to completion."""
    conn, _ = sock.accept()
    EvaluatorServer(backend, device, tamper=tamper).serve(Channel(conn))


class GarblerClient:
    """Garbler party: owns the circuit, garbles fresh GCs (offline), encodes
    inputs and decodes outputs (online).

    device: garble on this GPU (the garbler's own device; byte-identical to the host garbler), else on the
    host CPU. pipeline: garble GC b + 1 while GC b is serialized onto the wire and loaded by the evaluator
    (a bounded producer thread; the evaluator's ACKs are collected after the last model instead of after each
    one). gc_kw: GarbledCircuit construction options (rescale / relu / fused_sign)."""

    def __init__(self, host: str, port: int, circuit, crt, mrs=None, batch: int = 1, max_modulus: int = 0,
                 seed: Optional[bytes] = None, timeout: float = 600.0, device: Optional[int] = None,
                 pipeline: bool = True, transport: str = "tcp", **gc_kw):
        """transport: "tcp" ships the offline message over the channel (any host); "shm" writes it into a ring
        of shared-memory segments of this host and sends only their names (same-host split, e.g. the trusted
        garbler beside its evaluator); "ipc" garbles on this process's GPU straight into the HIP evaluator's
        table slots through their IPC handles (same node; the garbler's device and the evaluator's may differ,
        writes then go peer-to-peer over xGMI) and sends only each model's skeleton; online messages always
        use the channel."""
        if transport not in ("tcp", "shm", "ipc"):
            raise ValueError("transport must be 'tcp', 'shm' or 'ipc'")
        if transport == "ipc" and device is None:
            raise ValueError("transport='ipc' garbles on a GPU: pass device=")
        self.circuit, self.crt, self.mrs = circuit, crt, mrs
        self.batch, self.max_modulus = batch, max_modulus
        self.device, self.pipeline, self.gc_kw = device, pipeline, gc_kw
        self.transport = transport
        self._ring: list = []  # shared-memory segments (shm transport)
        self._ipc = None  # the evaluator's table slots, opened (ipc transport)
        self._seed = seed
        self._ctr = 0
        self.ch = connect(host, port, timeout=timeout)
        self.ch.send(b"HELO", json.dumps({"version": VERSION, "batch": batch}).encode())
        _, _, buf = self.ch.recv(b"HELO")
        self.server_info = json.loads(buf.decode())
        self.gcs: list = []
        self._bufs: list = []
        self.stats = {"offline_bytes": 0, "online_bytes": 0, "garble_s": 0.0, "serialize_s": 0.0, "offline_s": 0.0,
                      "online_s": [], "gcs": 0}

    def _next_seed(self) -> Optional[bytes]:
        if self._seed is None:
            return None
        import hashlib

        self._ctr += 1
        return hashlib.sha256(self._seed + self._ctr.to_bytes(8, "little")).digest()[:16]

    def _garble_one(self, seed):
        """One fresh GC and its offline message (a reused send buffer); the garbler keeps only the encoder and
        decoder secrets."""
        from ..garbling import GarbledCircuit

        t = time.perf_counter()
        gc = GarbledCircuit(self.circuit, self.crt, self.mrs, max_modulus=self.max_modulus, seed=seed,
                            device=self.device, **self.gc_kw)
        self.stats["encoding"] = "hardened" if gc.hardened else "reference"
        t1 = time.perf_counter()
        n = gc.model.serialized_size()
        try:
            buf = self._bufs.pop()  # a buffer whose send has completed (appended by the sending thread)
        except IndexError:
            buf = None
        if buf is None or buf.size < n:
            buf = np.empty(n, dtype=np.uint8)
        gc.model.serialize_into(buf)
        gc.model = None
        t2 = time.perf_counter()
        return gc, buf, n, t1 - t, t2 - t1

    # ---- shared-memory ring (transport="shm")
    _RING = 3

    def _ring_ensure(self, size: int) -> None:
        from multiprocessing import shared_memory

        if self._ring and self._ring[0].size >= size:
            return
        self._ring_close()
        # tmpfs accepts an ftruncate past its free space and then SIGBUSes the writer (the native serializer
        # runs without the GIL, so the garbler process dies instead of raising): check the space up front
        need = self._RING * size
        try:
            st = os.statvfs("/dev/shm")
            free = st.f_bavail * st.f_frsize
        except OSError:
            free = None
        if free is not None and free < need:
            raise RuntimeError(f"transport='shm' needs {need / 2**30:.2f} GiB in /dev/shm for {self._RING} ring "
                               f"segments but only {free / 2**30:.2f} GiB are free; use transport='tcp'")
        self._ring = []
        try:
            for _ in range(self._RING):
                seg = shared_memory.SharedMemory(create=True, size=size)
                self._ring.append(seg)
                if hasattr(os, "posix_fallocate"):  # reserve the pages now: a full tmpfs fails here, not in a write
                    os.posix_fallocate(seg._fd, 0, size)
        except OSError as e:
            self._ring_close()
            raise RuntimeError(f"transport='shm': cannot reserve {size} bytes in /dev/shm ({e}); "
                               "use transport='tcp'") from e

    def _ring_close(self) -> None:
        for seg in self._ring:
            try:
                seg.close()
                seg.unlink()
            except (OSError, BufferError):
                pass
        self._ring = []

    def _offline_shm(self, seeds) -> None:
        """Offline phase through the shared-memory ring: the producer garbles GC b + 1 and serializes it into a
        free segment while GC b's segment is being loaded by the evaluator; a segment is reused after its ACK."""
        import collections
        import queue
        import threading

        first = self._garble_gc(seeds[0])
        n = first.model.serialized_size()
        self._ring_ensure(n)
        free: "queue.Queue" = queue.Queue()
        for i in range(len(self._ring)):
            free.put(i)
        ready: "queue.Queue" = queue.Queue()
        err: list = []

        def produce():
            try:
                for b in range(self.batch):
                    gc = first if b == 0 else self._garble_gc(seeds[b])
                    i = free.get()
                    if i < 0:  # the sending side gave up
                        return
                    t = time.perf_counter()
                    got = gc.model.serialize_into(np.ndarray((self._ring[i].size,), np.uint8, buffer=self._ring[i].buf))
                    gc.model = None
                    self.stats["serialize_s"] += time.perf_counter() - t
                    ready.put((gc, i, got))
            except BaseException as e:  # surfaced on the sending thread
                err.append(e)
                ready.put(None)

        if not self.pipeline:  # one GC at a time: garble, serialize into segment 0, ship, wait for its ACK
            for b in range(self.batch):
                gc = first if b == 0 else self._garble_gc(seeds[b])
                t = time.perf_counter()
                got = gc.model.serialize_into(np.ndarray((self._ring[0].size,), np.uint8, buffer=self._ring[0].buf))
                gc.model = None
                self.stats["serialize_s"] += time.perf_counter() - t
                self.ch.send(b"MODS", json.dumps({"name": self._ring[0].name, "size": got}).encode(), flags=b)
                self.stats["offline_bytes"] += got
                self.ch.recv(b"ACK_")
                self.gcs.append(gc)
            return
        th = threading.Thread(target=produce, name="dash-garbler", daemon=True)
        th.start()
        pending: "collections.deque" = collections.deque()
        try:
            for b in range(self.batch):
                item = ready.get()
                if item is None:
                    raise err[0]
                gc, i, got = item
                self.ch.send(b"MODS", json.dumps({"name": self._ring[i].name, "size": got}).encode(), flags=b)
                self.stats["offline_bytes"] += got  # the offline message (in the segment) + its frame below
                pending.append(i)
                self.gcs.append(gc)
                if len(pending) >= len(self._ring):
                    self.ch.recv(b"ACK_")
                    free.put(pending.popleft())
            while pending:
                self.ch.recv(b"ACK_")
                free.put(pending.popleft())
        finally:
            for _ in range(len(self._ring)):  # unblock a producer waiting for a segment if sending failed
                free.put(-1)
            th.join()

    def _offline_ipc(self, seeds) -> None:
        """Offline phase over the device transport: GC b is garbled on this process's GPU straight into the
        evaluator's slot b (opened once from its IPC handles); its skeleton follows on the channel. Slots are
        distinct, so GC b + 1 is garbled while the evaluator loads GC b's constants; the ACKs are collected last."""
        if self._ipc is None:
            tmpl = self._garble_gc(None)  # a template for the evaluator's build (tables stay here, discarded)
            _dbg("client: template garbled")
            self.ch.send(b"TMPL", tmpl.model.serialize_skeleton(all_device=True))
            del tmpl
            _, _, buf = self.ch.recv(b"IPCH")
            hs = [(int(l), str(t), int(nb), bytes.fromhex(h)) for l, t, nb, h in json.loads(buf.decode())]
            _dbg(f"client: {len(hs)} IPC handles received")
            self._ipc = native().IpcTables(int(self.device), hs, self.batch)
            _dbg("client: handles opened")
        for b in range(self.batch):
            gc = self._garble_gc(seeds[b], sink=self._ipc.sink(b))
            _dbg(f"client: GC {b} garbled into the evaluator's slot")
            t = time.perf_counter()
            skel = gc.model.serialize_skeleton()
            gc.model = None
            self.stats["serialize_s"] += time.perf_counter() - t
            self.ch.send(b"MODX", skel, flags=b)
            self.gcs.append(gc)
        for _ in range(self.batch):
            self.ch.recv(b"ACK_")

    def _garble_gc(self, seed, sink=None):
        from ..garbling import GarbledCircuit

        t = time.perf_counter()
        gc = GarbledCircuit(self.circuit, self.crt, self.mrs, max_modulus=self.max_modulus, seed=seed,
                            device=self.device, sink=sink, **self.gc_kw)
        self.stats["garble_s"] += time.perf_counter() - t
        self.stats["encoding"] = "hardened" if gc.hardened else "reference"
        return gc

    def offline(self) -> None:
        """Garble `batch` fresh circuits and ship them (offline phase)."""
        import queue
        import threading

        if self.transport == "ipc":
            t0 = time.perf_counter()
            sent0 = self.ch.bytes_sent
            seeds = [self._next_seed() for _ in range(self.batch)]
            self.gcs = []
            self._offline_ipc(seeds)
            self.stats["gcs"] += self.batch
            self.stats["offline_bytes"] += self.ch.bytes_sent - sent0
            self.stats["offline_s"] += time.perf_counter() - t0
            return
        if self.transport == "shm":
            t0 = time.perf_counter()
            sent0 = self.ch.bytes_sent
            seeds = [self._next_seed() for _ in range(self.batch)]
            self.gcs = []
            self._offline_shm(seeds)
            self.stats["gcs"] += self.batch
            self.stats["offline_bytes"] += self.ch.bytes_sent - sent0
            self.stats["offline_s"] += time.perf_counter() - t0
            return
        t0 = time.perf_counter()
        sent0 = self.ch.bytes_sent
        seeds = [self._next_seed() for _ in range(self.batch)]
        self.gcs = []
        if not self.pipeline or self.batch == 1:
            for b in range(self.batch):
                gc, buf, n, tg, ts = self._garble_one(seeds[b])
                self.stats["garble_s"] += tg
                self.stats["serialize_s"] += ts
                self.ch.send(b"MODL", memoryview(buf)[:n], flags=b)
                self.ch.recv(b"ACK_")
                self._bufs.append(buf)
                self.gcs.append(gc)
        else:
            q: "queue.Queue" = queue.Queue(maxsize=2)  # at most two models in flight beside the one on the wire
            err: list = []
            stop = threading.Event()

            def put(item) -> bool:
                # bounded put that gives up once the sending side has stopped (a failed send must not leave the
                # producer blocked on a full queue forever)
                while not stop.is_set():
                    try:
                        q.put(item, timeout=0.1)
                        return True
                    except queue.Full:
                        continue
                return False

            def produce():
                try:
                    for b in range(self.batch):
                        if stop.is_set() or not put(self._garble_one(seeds[b])):
                            return
                except BaseException as e:  # surfaced on the sending thread
                    err.append(e)
                    put(None)

            th = threading.Thread(target=produce, name="dash-garbler", daemon=True)
            th.start()
            try:
                for b in range(self.batch):
                    item = q.get()
                    if item is None:
                        raise err[0]
                    gc, buf, n, tg, ts = item
                    self.stats["garble_s"] += tg
                    self.stats["serialize_s"] += ts
                    self.ch.send(b"MODL", memoryview(buf)[:n], flags=b)
                    self._bufs.append(buf)
                    self.gcs.append(gc)
                for _ in range(self.batch):  # the evaluator acknowledges every load, in order
                    self.ch.recv(b"ACK_")
            finally:
                stop.set()
                while True:  # drain: a producer blocked in put() sees the stop flag within 0.1 s
                    try:
                        q.get_nowait()
                    except queue.Empty:
                        break
                th.join()
        self.stats["gcs"] += self.batch
        self.stats["offline_bytes"] += self.ch.bytes_sent - sent0
        self.stats["offline_s"] += time.perf_counter() - t0

    def infer(self, xs: Sequence) -> list:
        """One online round for `batch` inputs -> decoded outputs."""
        if len(self.gcs) != self.batch:
            raise RuntimeError("no fresh garbled circuits: call offline() first (GCs are single use)")
        assert len(xs) == self.batch
        t0 = time.perf_counter()
        b0, r0 = self.ch.bytes_sent, self.ch.bytes_recv
        msg = np.concatenate([gc.garble_inputs_compressed(x).reshape(-1) for gc, x in zip(self.gcs, xs)])
        self.ch.send(b"INPT", msg, flags=self.batch)
        _, _, buf = self.ch.recv(b"OUTP")
        raw = np.frombuffer(buf, dtype=np.uint64)
        per = raw.size // self.batch
        outs = []
        for b, gc in enumerate(self.gcs):
            k = len(gc.decoder.moduli)
            outs.append(gc.decode_compressed(raw[b * per:(b + 1) * per].reshape(k, -1, 2)))
        self.gcs = []
        self.stats["online_bytes"] += (self.ch.bytes_sent - b0) + (self.ch.bytes_recv - r0)
        self.stats["online_s"].append(time.perf_counter() - t0)
        return outs

    def close(self) -> None:
        try:
            self.ch.send(b"BYE_")
        except OSError:
            pass
        self.ch.close()
        self._ring_close()
        self._ipc = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
