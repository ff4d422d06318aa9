"""Headline benchmark engine (bench.py and the multi-rank tests share it).

Metric: online garbled inferences/sec for the MiniONN-style CIFAR-10 CNN
(MODEL_F_MINIONN_POOL_REPL, DASH config: ScaleQuant l=5, k=7 CRT base {2..17},
ReLU accuracy 100 % -> MRS {86,7,6,6,5}), BASELINE.json.

Timed region per step (the reference's GPU model benchmark,
benchmarks/model_benchmarks/sgx/Enclave/Enclave.cpp:177-183):
    garble_inputs -> H2D -> evaluate -> D2H -> decode_outputs
for B independent garbled circuits per GPU (one fresh input per GC per step).
Offline garbling and the table upload are excluded, as in the reference, and
reported separately. The B GCs of the online phase are garbled once and
re-encoded every step; a step's work (encode, H2D, evaluate, D2H, decode for B
inferences) is the same as on fresh GCs. (A rolling per-group pipeline of the
steps, each group's decode and next encode overlapping the others' runs, measured
no faster: 2246 vs 2300 inf/s, the GPU is the bound.) Two further phases run after the
timed loop and are reported beside the headline, never instead of it:

* ``reference``: the same loop with the reference's gadget constructions
  (legacy l-fold sign-base-extension rescale rescale_gadget.h:115-242,
  approximate-sign ReLU garbled_relu.h:119-179, explicit cast gates
  sign_gadget.h:456-546) -> ``reference_constructions_value``;
* ``served``: fresh GC per inference (GCs are single use), offline garbling
  pipelined against online evaluation (dash_amd.serving.InferenceService)
  -> ``served_inf_per_s``, garbling included.

Multi-GPU: one process per GPU (torchrun), batch data parallel; every rank
garbles and evaluates its own GCs; the slowest rank defines the step time;
per-rank records (device, PCI bus id, ms/step, host encode+decode time) are
all-gathered over the job's process group (RCCL) and printed by rank 0.

``--backend cpu`` runs the identical driver on the native host evaluator
(tests: gloo, world 2/4, no GPU).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import sys
import time
from typing import List, Optional

import numpy as np

BASELINE_LATENCY_MS = 1443.0  # RTX 4090, DASH GPU, MiniONN, batch 1, fresh GC
BASELINE_INF_PER_S = 1000.0 / BASELINE_LATENCY_MS

CONSTRUCTIONS = {
    # the framework's fastest exact-on-the-guarded-range constructions (headline)
    "flagship": dict(sign="fused", rescale="mrs", relu="joint"),
    # the reference's constructions
    "reference": dict(sign="reference", rescale="legacy", relu="approx", hardened=False),
}


def log(*a):
    print(f"[bench {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def host_thread_budget(requested: int = 0) -> int:
    """Host worker threads per rank: the rank's share of the visible CPUs
    (cores / ranks on this node), capped by OMP_NUM_THREADS when set."""
    if requested > 0:
        return requested
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        ncpu = os.cpu_count() or 1
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    t = max(1, ncpu // local)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        t = min(t, int(omp))
    return t


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU). Without a launcher (WORLD_SIZE unset) bench.py starts N fresh ranks "
                         "itself; with one, WORLD_SIZE must equal N")
    ap.add_argument("--rehearse-shared-device", action="store_true",
                    default=os.environ.get("DASH_BENCH_REHEARSAL", "") == "1",
                    help="allow more ranks than visible GPUs (ranks share devices over gloo). A rehearsal of the "
                         "multi-rank path, never a scaling measurement; the record says so")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("DASH_BENCH_BATCH", "0")),
                    help="GCs evaluated together per GPU (0: as many as HBM holds, a multiple of --streams)")
    ap.add_argument("--constructions", default=os.environ.get("DASH_BENCH_CONSTRUCTIONS", "flagship"),
                    choices=sorted(CONSTRUCTIONS), help="gadget constructions of the headline phase")
    ap.add_argument("--sign", default=None, choices=["fused", "reference"], help="override the sign construction")
    ap.add_argument("--rescale", default=None, choices=["mrs", "legacy"], help="override the rescale construction")
    ap.add_argument("--relu", default=None, choices=["mrs", "approx", "joint"], help="override the ReLU sign")
    # 3 groups with the steps pipelined: 3230 / 3225 / 3240 / 3229 inf/s (165 GCs) against 3065-3085 with 4, 3158-3174
    # with 5, 3018-3021 with 6, 3004-3007 with 8 and 2799-2813 with 2, with the box's 4 hardware queues or 8
    # (profiles/ab/r6/r06z{,p,r}_*.json); the reference constructions' 10 GB GCs take 2 groups
    ap.add_argument("--streams", type=int, default=int(os.environ.get("DASH_BENCH_STREAMS", "3")),
                    help="independent GC groups per GPU, each on its own HIP stream")
    ap.add_argument("--ref-streams", type=int, default=int(os.environ.get("DASH_BENCH_REF_STREAMS", "2")),
                    help="GC groups of the reference-constructions phase")
    ap.add_argument("--model", default="MODEL_F_MINIONN_POOL_REPL")
    ap.add_argument("--config", default="DASH", choices=["DASH", "REDASH_OPT", "REDASH_CPM"])
    ap.add_argument("--backend", default="hip", choices=["hip", "cpu"])
    ap.add_argument("--no-mfma", action="store_true")
    ap.add_argument("--profile", action="store_true", help="print per-layer GPU times")
    ap.add_argument("--threads", type=int, default=0, help="host threads per rank (0: cores / local ranks)")
    ap.add_argument("--verify", type=int, default=1)
    ap.add_argument("--pipeline", type=int, default=int(os.environ.get("DASH_BENCH_PIPELINE", "1")),
                    help="1: a group's next step is encoded and launched as soon as its outputs of the current step "
                         "are fetched and decoded (the other groups keep the GPU busy meanwhile); 0: step by step")
    ap.add_argument("--garble-device", type=int, default=int(os.environ.get("DASH_BENCH_GARBLE_DEVICE", "1")),
                    help="garble on this rank's GPU (byte-identical to the host garbler)")
    ap.add_argument("--phases",
                    default=os.environ.get("DASH_BENCH_PHASES", "main,threads,latency,latency_ref,reference,served"),
                    help="comma list of main, threads, latency (flagship, batch 1: device and wire-form input "
                         "encoding), latency_ref (batch 1, the reference's constructions and encoding, wire-form "
                         "input: the like-for-like comparison with its 1443 ms), reference, served (main is always "
                         "run)")
    ap.add_argument("--thread-sweep", default="4,8",
                    help="host thread budgets of the threads phase (headline loop re-timed at each)")
    ap.add_argument("--latency-gcs", type=int, default=8, help="fresh GCs timed one by one in the latency phase")
    ap.add_argument("--input-encoding", default=os.environ.get("DASH_BENCH_INPUT_ENCODING", "device"),
                    choices=["device", "host"],
                    help="online message #1 (hip): the garbler's device encoder (GarbledCircuit.device_input_encoder,"
                         " one launch per group) or host-encoded compressed labels + H2D + GPU unpack")
    ap.add_argument("--ref-batch", type=int, default=0, help="GCs per GPU of the reference phase (0: auto)")
    ap.add_argument("--ref-steps", type=int, default=0, help="timed steps of the reference phase (0: --steps)")
    # with 8 concurrent garblings, small groups keep the pool ahead of the requests: 2 slots x 8 groups 226-241
    # served inf/s (p50 batch 3.4-4 ms) against 193-211 for 16 x 3 (profiles/ab/r6/r06z{f,g,h,i}_*.json)
    ap.add_argument("--served-slots", type=int, default=2)
    ap.add_argument("--served-groups", type=int, default=8)
    ap.add_argument("--served-requests", type=int, default=64, help="online batches of the served phase")
    ap.add_argument("--served-min-s", type=float, default=10.0,
                    help="the served phase keeps issuing requests until it has run this long (steady state)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------------------- rank launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpus() -> int:
    """Visible GPU count without initialising HIP in this process (a parent that starts ranks must not).

    Read from the KFD topology in sysfs (parallel/dist.py kfd_gpus), filtered by the *_VISIBLE_DEVICES
    variables: torch.cuda.device_count() falls back to hipGetDeviceCount when amdsmi is missing, which would
    initialise the HIP runtime here. Raises when the topology cannot be read (no silent guess)."""
    from .parallel.dist import kfd_gpus, visible_indices

    gpus = kfd_gpus()
    return len(visible_indices(len(gpus), None, gpus))


def spawn_ranks(args, argv: List[str]) -> int:
    """``bench.py --gpus N`` with no launcher: start N fresh rank processes (torch.distributed.run, one per GPU,
    rendezvous on 127.0.0.1) and forward rank 0's JSON line. This parent never makes a HIP call and never
    execs; it exits with the launcher's code (non-zero when any rank failed). The reference is single-device
    (benchmarks/model_benchmarks/non_sgx/main.cpp:27-92); batch DP over the node is this framework's scale-out."""
    import subprocess

    n = args.gpus
    if args.backend == "hip":
        try:
            avail = visible_gpus()
        except RuntimeError as e:
            if not args.rehearse_shared_device:
                log(f"--gpus {n}: {e}; refusing")
                return 2
            avail = 0
        if avail < n and not args.rehearse_shared_device:
            log(f"--gpus {n} requested but only {avail} GPU(s) visible: refusing (a scaling run needs one GPU per "
                f"rank; --rehearse-shared-device runs the multi-rank path on shared devices, clearly labelled)")
            return 2
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if args.rehearse_shared_device:
        env["DASH_BENCH_REHEARSAL"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(root, "bench.py"), *argv]
    log(f"starting {n} ranks: {' '.join(cmd[1:6])} ...")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True)
    record = None
    for line in proc.stdout:
        if line.lstrip().startswith("{") and '"metric"' in line:
            record = line.strip()
        else:
            sys.stderr.write(line)
    rc = proc.wait()
    if record is not None:
        print(record, flush=True)
    if rc == 0 and record is None:
        log("ranks exited 0 but rank 0 printed no record")
        return 1
    return rc


def check_world(args, ctx, recs: list, rehearsal: bool) -> None:
    """Rank 0's guard before it prints: the job really is N ranks, over RCCL, on N distinct GPUs."""
    if ctx.world != args.gpus:
        raise RuntimeError(f"--gpus {args.gpus} but the job has {ctx.world} rank(s)")
    if args.backend != "hip" or ctx.world == 1 or rehearsal:
        return
    if ctx.backend != "nccl":
        raise RuntimeError(f"multi-GPU bench must run over nccl (RCCL), got {ctx.backend}")
    buses = {r.get("pci_bus_id") for r in recs}
    if len(buses) != ctx.world:
        raise RuntimeError(f"{ctx.world} ranks but {len(buses)} distinct GPU(s) (PCI bus ids {sorted(buses)})")


# ----------------------------------------------------------------------------------------- evaluator slots
class _HipGroup:
    """``per`` GC slots evaluated together by one HipEvaluator on one stream.

    Online message #1 (``device_encode``): the garbler's device input encoder of the group (one encoder slot per
    GC slot, armed when the GC is loaded, offline) writes every slot's input labels with one H2D of the plaintext
    inputs and one launch; otherwise the host encodes 16-B compressed labels (a reused GC's codebook lookup) that
    are copied to the GPU and unpacked there."""

    def __init__(self, template, per: int, device: int, mfma: bool, profile: bool, stream, device_encode=False):
        from .runtime import HipEvaluator

        self.ev = HipEvaluator(template=template, batch=per, device=device, mfma=mfma, profile=profile)
        self.stream = stream
        self.per, self.device = per, device
        self.device_encode = device_encode
        self.enc = None

    def load(self, b, gc):
        self.ev.load(b, gc.model)  # a GC garbled into this slot (sink) only copies its small constants
        gc.model = None  # tables live in HBM now
        if self.device_encode:  # the garbler's input state of this GC to the GPU (offline, with its tables)
            if self.enc is None:  # arms only slot b; every slot is armed by its own GC
                self.enc = gc.device_input_encoder(self.device, self.per, slot=b)
            else:
                self.enc.load(gc.garbler, b)

    def sink(self, b):
        return self.ev.sink(b)

    def encode_batch(self, gcs, xs):
        if self.device_encode:
            self.ev.encode_device_into(0, self.enc, np.stack([np.asarray(x).reshape(-1) for x in xs]), self.stream)
        else:
            for b, (gc, x) in enumerate(zip(gcs, xs)):
                self.ev.encode_compressed_into(b, gc, x, guarded=True)  # the step's batch guard (_Bench)

    def launch(self):
        if not self.device_encode:
            self.ev.upload_inputs_compressed(self.stream)
        self.ev.run(self.stream)

    def fetch(self):
        self.ev.fetch_outputs(self.stream)  # online message #2 (synchronizes this group's stream)

    def decode(self, b, gc):
        return self.ev.decode(b, gc)


class _CpuGroup:
    """Host-evaluator stand-in with the same interface (tests, no GPU)."""

    def __init__(self, template, per: int, threads: int):
        self.per, self.threads = per, threads
        self.models = [None] * per
        self.inputs = [None] * per
        self.outputs = [None] * per

    def load(self, b, gc):
        self.models[b] = gc

    def sink(self, b):
        return None

    def encode_batch(self, gcs, xs):
        for b, (gc, x) in enumerate(zip(gcs, xs)):
            self.inputs[b] = gc.garble_inputs(x)

    def launch(self):
        for b, gc in enumerate(self.models):
            self.outputs[b] = gc.cpu_evaluate(self.inputs[b], self.threads)

    def fetch(self):
        pass

    def decode(self, b, gc):
        return gc.decode_outputs(self.outputs[b])


# ----------------------------------------------------------------------------------------- phases
class _Bench:
    def __init__(self, args, ctx):
        self.args, self.ctx = args, ctx
        from .ir.quant import QuantizationMethod
        from .models import BENCH_CONFIGS, build_circuit, canonical

        self.model = canonical(args.model)
        cfg = BENCH_CONFIGS.get(f"{self.model}/{args.config}") or BENCH_CONFIGS["MODEL_F_MINIONN_POOL_REPL/DASH"]
        self.cfg = cfg
        self.qm, self.qp = QuantizationMethod(cfg["q_method"]), cfg["q_parameter"]
        self.circuit = build_circuit(self.model, self.qm, self.qp, seed=0)  # public model, identical on every rank
        # range calibration (reference layer.h range tracking): arms the mixed-radix rescale's wrap-band guard
        # (garbling.resolve_constructions refuses rescale="mrs" when a tracked rescale input enters the band)
        from .models import quantized_inputs

        self.circuit.calibrate(quantized_inputs(self.model, 32, self.qm, self.qp, seed=0), svc_modulus(cfg["crt"]))
        self.hip = args.backend == "hip"
        self.device_encode = self.hip and getattr(args, "input_encoding", "device") == "device"
        self.device = ctx.device if (self.hip and ctx.device is not None) else 0
        if self.hip:
            import torch

            self.device = torch.cuda.current_device()

    # ---- one GC (sink: the evaluator slot the GPU garbler writes the tables into)
    def garble(self, tag: str, b: int, cons: dict, sink=None):
        from .garbling import GarbledCircuit

        seed = hashlib.sha256(f"dash-bench/{tag}/{self.ctx.rank}/{b}/{os.getpid()}".encode()).digest()[:16]
        dev = self.device if (self.hip and self.args.garble_device) else None
        return GarbledCircuit(self.circuit, self.cfg["crt"], self.cfg["mrs"], seed=seed, device=dev,
                              fused_sign=cons["sign"] == "fused", rescale=cons["rescale"], relu=cons["relu"],
                              hardened=cons.get("hardened"), nthreads=self.threads,
                              sink=sink if dev is not None else None)

    # ---- offline: garble B GCs into G groups of evaluator slots
    def offline(self, tag: str, cons: dict, batch: int, streams: int = 0):
        from .parallel import all_reduce_min

        args, ctx = self.args, self.ctx
        B = batch if batch > 0 else (256 if self.hip else 2)
        G = max(1, min(streams or args.streams, B))
        B -= B % G
        per = B // G
        gcs: list = []
        groups: list = [None] * G
        st = dict(garble_s=0.0, upload_s=0.0, table_gb=0.0)
        free0 = None
        if self.hip:
            import torch

            free0 = torch.cuda.mem_get_info(self.device)[0]
            streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(G - 1)]
        else:
            streams = [None] * G
        t_off = time.perf_counter()

        def new_group(gc, g, per_):
            if self.hip:
                from .native import native

                native().gpu_table_cache_trim()  # the new group's table arena needs the garbler's cached blocks
                return _HipGroup(gc.model, per_, self.device, not args.no_mfma, args.profile, streams[g],
                                 device_encode=self.device_encode)
            return _CpuGroup(gc.model, per_, self.threads)

        b = 0
        while b < B:
            try:
                t = time.perf_counter()
                grp = groups[b // per] if b > 0 and b // per < len(groups) else None
                gc = self.garble(tag, b, cons, sink=grp.sink(b % per) if grp is not None else None)
                st["garble_s"] += time.perf_counter() - t
                if b == 0:
                    if self.hip:
                        # HBM guard: every GC's tables stay resident. Size B from the real device footprint of
                        # one GC (tables + evaluator scratch) plus one GC in flight in the garbler.
                        from .runtime import HipEvaluator

                        probe = HipEvaluator(template=gc.model, batch=1, device=self.device, mfma=not args.no_mfma)
                        per_gc = probe.device_bytes() * 1.01
                        del probe
                        fit = int((free0 - gc.table_bytes - 2.5e9) // per_gc)
                        log(f"[{tag}] rank {ctx.rank}: {free0 / 1e9:.1f} GB HBM free, {per_gc / 1e9:.2f} GB per GC "
                            f"({gc.table_bytes / 1e9:.2f} GB tables): fits {fit}")
                        if fit < B:
                            B = max(G, fit - fit % G)
                            log(f"[{tag}] rank {ctx.rank}: batch {'sized' if batch <= 0 else 'reduced'} to {B}")
                    B = int(all_reduce_min(ctx, float(B)))  # every rank evaluates the same number of GCs
                    G = max(1, min(G, B))
                    B -= B % G
                    per = B // G
                    # every group's arena up front (template: this GC), so later GCs garble straight into slots
                    groups = []
                    for g in range(G):
                        try:
                            groups.append(new_group(gc, g, per))
                        except RuntimeError as e:  # fragmentation near full HBM: keep the groups that fit
                            if "out of memory" not in str(e) or g == 0:
                                raise
                            from .native import native

                            native().hip_clear_last_error()
                            log(f"[{tag}] rank {ctx.rank}: HBM holds {g} of {G} groups")
                            break
                    G = len(groups)
                    B = G * per
                t = time.perf_counter()
                g = b // per
                st["table_gb"] = gc.table_bytes / 1e9
                groups[g].load(b % per, gc)
                st["upload_s"] += time.perf_counter() - t
                gcs.append(gc)
                if b < 3 or (b + 1) % 16 == 0 or b + 1 == B:
                    log(f"[{tag}] rank {ctx.rank}: garbled+uploaded GC {b + 1}/{B} ({st['table_gb']:.2f} GB tables)")
            except RuntimeError as e:
                # HBM ran out before the estimate said it would: keep this rank's complete groups; the
                # all-reduce below makes every rank agree on the smallest batch
                if "out of memory" not in str(e) or b < per:
                    raise
                from .native import native

                native().gpu_table_cache_trim()
                native().hip_clear_last_error()  # the handled OOM must not resurface in the next launch check
                log(f"[{tag}] rank {ctx.rank}: out of HBM at GC {b + 1}")
                B = b
                break
            b += 1
        # ranks agree on B after the loop too (one rank's out-of-memory fallback shrinks only its own batch)
        B_all = int(all_reduce_min(ctx, float(B - B % per)))
        G = B_all // per
        groups, gcs, streams = groups[:G], gcs[:G * per], streams[:G]
        B = G * per
        if self.hip:
            from .native import native

            native().gpu_table_cache_trim()
        st["offline_s"] = time.perf_counter() - t_off
        return gcs, groups, B, G, per, st

    # ---- online: timed steps over the loaded groups
    def online(self, gcs, groups, B, per, steps, warmup, seed_base, verify):
        from .models import quantized_inputs
        from .parallel import all_reduce_max, barrier

        ctx = self.ctx
        inputs = quantized_inputs(self.model, B * (steps + warmup), self.qm, self.qp, seed=seed_base + ctx.rank)
        host = [0.0]

        guard = gcs[0].guard if (self.hip and gcs[0].guard_enabled) else None

        def step(i: int, check: bool = False):
            xs = inputs[i * B:(i + 1) * B]
            # online message #1 (device encoder, or wire form: 16-B compressed labels -> pinned staging -> H2D ->
            # GPU unpack); the G groups run concurrently on their own streams
            for g, grp in enumerate(groups):
                t = time.perf_counter()
                grp.encode_batch(gcs[g * per:(g + 1) * per], xs[g * per:(g + 1) * per])
                host[0] += time.perf_counter() - t
                grp.launch()
            # the garbler's exact range guard of the step's inputs (mixed-radix wrap band, CRT overflow): one
            # batched check on its own stream, submitted after the evaluations (its host-side submit is then off
            # their critical path) and overlapping them; no result is released before it passes
            pend = guard.submit(xs) if guard is not None else None
            dec = []
            for g, grp in enumerate(groups):
                grp.fetch()
                t = time.perf_counter()
                dec += [grp.decode(b, gcs[g * per + b]) for b in range(per)]
                host[0] += time.perf_counter() - t
            if pend is not None:
                pend.raise_if_bad()
            if check:
                self.verify(xs, dec)
            return dec

        # DASH_BENCH_ORDER=completion: the pipelined loop takes the groups in the order their steps finish
        # (a HIP event per launch, polled) instead of in index order
        by_completion = os.environ.get("DASH_BENCH_ORDER", "index") == "completion" and self.hip
        done_ev = [None] * len(groups)

        def launch_group(g, grp, i):
            xs = inputs[i * B:(i + 1) * B]
            t = time.perf_counter()
            grp.encode_batch(gcs[g * per:(g + 1) * per], xs[g * per:(g + 1) * per])
            host[0] += time.perf_counter() - t
            grp.launch()
            if by_completion:
                import torch

                done_ev[g] = torch.cuda.Event()
                done_ev[g].record(grp.stream)

        def group_order():
            left = list(range(len(groups)))
            while left:
                g = next((x for x in left if done_ev[x] is None or done_ev[x].query()), left[0]) if by_completion \
                    else left[0]
                left.remove(g)
                yield g

        def steps_pipelined(first: int, n: int, check_first: bool = False):
            """Steps first .. first + n - 1 with the groups pipelined across steps: group g's step i + 1 is
            encoded and launched right after its step-i outputs are fetched and decoded, while the other groups
            still run step i. Every step's range check still passes before its outputs are released."""
            for g, grp in enumerate(groups):
                launch_group(g, grp, first)
            pend = guard.submit(inputs[first * B:(first + 1) * B]) if guard is not None else None
            dec = None
            for i in range(first, first + n):
                more = i + 1 < first + n
                parts = [None] * len(groups)
                for g in group_order():
                    grp = groups[g]
                    grp.fetch()
                    t = time.perf_counter()
                    parts[g] = [grp.decode(b, gcs[g * per + b]) for b in range(per)]
                    host[0] += time.perf_counter() - t
                    if more:
                        launch_group(g, grp, i + 1)
                dec = [y for part in parts for y in part]
                nxt = guard.submit(inputs[(i + 1) * B:(i + 2) * B]) if (guard is not None and more) else None
                if pend is not None:
                    pend.raise_if_bad()
                if check_first and i == first:
                    self.verify(inputs[i * B:(i + 1) * B], dec)
                pend = nxt
            return dec

        pipelined = bool(getattr(self.args, "pipeline", 0))
        verified = False
        if pipelined and warmup > 0:
            steps_pipelined(0, warmup, check_first=bool(verify))
            verified = bool(verify)
        else:
            for w in range(warmup):
                step(w, check=bool(verify) and w == 0)
                verified = verified or bool(verify)
        self.sync()
        barrier(ctx)
        self.sync()
        host[0] = 0.0
        t0 = time.perf_counter()
        last = None
        if pipelined and steps > 0:
            last = steps_pipelined(warmup, steps)
        else:
            for s in range(steps):
                last = step(warmup + s)
        self.sync()
        barrier(ctx)
        self.sync()
        local = time.perf_counter() - t0
        elapsed = all_reduce_max(ctx, local)  # slowest rank defines the step time
        # after the timer: the last timed step's decoded outputs against the exact plaintext model
        last_ok = None
        if verify and steps > 0:
            i = warmup + steps - 1
            self.verify(inputs[i * B:(i + 1) * B], last)
            last_ok = True
        return dict(elapsed=elapsed, local=local, host_ms=1000.0 * host[0] / max(1, steps), last=last,
                    verified=verified, verified_last_step=last_ok, step=step)

    def verify(self, xs, ys) -> None:
        """Decoded garbled outputs == the exact quantized plaintext model (CRT semantics), batched on this rank's
        GPU (garbling/guard.py RangeGuard.outputs; numpy per input on the cpu backend)."""
        from .garbling.guard import guard_for

        ref = guard_for(self.circuit, svc_modulus(self.cfg["crt"]), True, self.device if self.hip else None).outputs(xs)
        for k, (r, y) in enumerate(zip(ref, ys)):
            if not np.array_equal(r, np.asarray(y)):
                raise RuntimeError(f"garbled output mismatch at input {k}: {list(y)} vs {list(r)}")

    def sync(self):
        if self.hip:
            import torch

            torch.cuda.synchronize()

    # ---- served: fresh GC per inference, garbling pipelined against evaluation
    def served(self, cons: dict) -> dict:
        from .models import quantized_inputs
        from .parallel import all_reduce_max, barrier
        from .serving import InferenceService

        a, ctx = self.args, self.ctx
        slots, groups, reqs = a.served_slots, a.served_groups, a.served_requests
        pool = quantized_inputs(self.model, slots * 8, self.qm, self.qp, seed=5000 + ctx.rank)
        t0 = time.perf_counter()
        svc = InferenceService(self.circuit, self.cfg["crt"], self.cfg["mrs"],
                               backend="hip" if self.hip else "cpu", device=self.device, slots_per_group=slots,
                               groups=groups, garble_device=bool(self.hip and a.garble_device),
                               rescale=cons["rescale"], relu=cons["relu"], fused_sign=cons["sign"] == "fused",
                               hardened=cons.get("hardened"), nthreads=self.threads)
        fill_s = time.perf_counter() - t0
        try:
            barrier(ctx)
            svc.stats.t_start = time.perf_counter()
            t1 = time.perf_counter()
            ok = True
            M = svc_modulus(self.cfg["crt"])
            r = 0
            # steady state: at least `reqs` requests AND at least served_min_s seconds (the pool's initial fill
            # is drained within the first few requests; after that every inference waits on fresh garbling)
            while True:
                k = r % 8
                batch = pool[k * slots:(k + 1) * slots]
                y = svc.infer(batch)
                if r < 8:
                    ok = ok and all(np.array_equal(y[i], self.circuit.plain_q_eval(x, track=False, crt_modulus=M))
                                    for i, x in enumerate(batch))
                r += 1
                # every rank stops after the same number of requests (agreed by rank 0's clock)
                if r >= reqs:
                    done = all_reduce_max(ctx, float(time.perf_counter() - t1 >= a.served_min_s))
                    if done > 0:
                        break
            local = time.perf_counter() - t1
            st = svc.stats.as_dict()
        finally:
            svc.close()
        barrier(ctx)
        elapsed = all_reduce_max(ctx, local)
        n = slots * r
        return dict(value=ctx.world * n / elapsed, local_inf_per_s=n / local, pool_fill_s=fill_s,
                    garble_s_per_gc=st["garble_s_per_gc"], pool_wait_s=st["pool_wait_s"],
                    batch_latency_ms=st["batch_latency_ms"], verified=ok, slots=slots, groups=groups,
                    requests=r, duration_s=round(local, 2),
                    note=("one-process simulation: garbler and evaluator share this rank's process and GPU (the "
                          "reference's non-SGX benches do the same); benchmarks/two_party.py measures the split"))

    # ---- batch-1 latency on fresh GCs (the reference's timed region, one image at a time)
    def latency(self, cons: dict, device_encode: Optional[bool] = None) -> dict:
        """garble_inputs -> H2D -> evaluate -> D2H -> decode for one inference on a fresh GC each
        (benchmarks/model_benchmarks/sgx/Enclave/Enclave.cpp:177-183); garbling and the table upload are
        outside the timed region, as there. device_encode=False: online message #1 in wire form (the garbler
        encodes 16-B compressed labels on the host, H2D, GPU unpack), as between two parties."""
        from .models import quantized_inputs

        dev_enc = self.device_encode if device_encode is None else (bool(device_encode) and self.hip)

        n = max(2, self.args.latency_gcs)
        xs = quantized_inputs(self.model, n, self.qm, self.qp, seed=7000 + self.ctx.rank)
        ev, grp, times, ok = None, None, [], True
        for i in range(n + 1):  # one untimed warm-up GC (first launch, graph build)
            if self.hip:
                if grp is None:
                    gc = self.garble("lat", i, cons)
                    from .native import native

                    native().gpu_table_cache_trim()
                    grp = _HipGroup(gc.model, 1, self.device, not self.args.no_mfma, False, None,
                                    device_encode=dev_enc)
                else:
                    gc = self.garble("lat", i, cons, sink=grp.sink(0))
            else:
                gc = self.garble("lat", i, cons)
                grp = grp or _CpuGroup(gc.model, 1, self.threads)
            grp.load(0, gc)
            x = xs[max(0, i - 1)]
            self.sync()
            t = time.perf_counter()
            grp.encode_batch([gc], [x])
            grp.launch()
            # the garbler's range guard on its own stream, overlapping the evaluation (the cpu backend guards
            # inside garble_inputs)
            pend = gc.guard.submit([x]) if (self.hip and gc.guard_enabled) else None
            grp.fetch()
            y = grp.decode(0, gc)
            if pend is not None:
                pend.raise_if_bad()
            dt = time.perf_counter() - t
            if i > 0:
                times.append(1000.0 * dt)
                ok = ok and bool(np.array_equal(y, gc.plain_q_eval(x)))
        del grp
        if self.hip:
            from .native import native

            native().gpu_table_cache_trim()
        ts = sorted(times)
        return dict(latency_b1_ms=round(float(np.median(ts)), 3), min_ms=round(ts[0], 3), max_ms=round(ts[-1], 3),
                    gcs=n, fresh_gc_per_inference=True, verified=ok,
                    input_encoding="device" if dev_enc else "host", constructions=gc.effective_constructions())

    # ---- per-rank evidence
    def rank_record(self, ms_step: float, inf_s: float, host_ms: float, B: int) -> dict:
        rec = dict(rank=self.ctx.rank, local_rank=self.ctx.local_rank, host=socket.gethostname(), pid=os.getpid(),
                   threads=self.threads, gcs=B, ms_per_step=round(ms_step, 3), inf_per_s=round(inf_s, 3),
                   host_encode_decode_ms_per_step=round(host_ms, 3))
        # the GPU this rank owns by LOCAL_RANK, from sysfs (what init_distributed bound it to)
        from .parallel.dist import rank_gpu

        plan = rank_gpu(self.ctx.local_rank)
        rec["gpu_plan"] = plan
        if self.hip:
            from .native import native

            rec["device"] = int(self.device)
            rec["pci_bus_id"] = native().hip_device_pci_bus_id(int(self.device))
            if plan is not None:
                rec["pci_matches_plan"] = rec["pci_bus_id"].lower() == plan["pci"].lower()
                if not rec["pci_matches_plan"] and os.environ.get("DASH_DEBUG_DEVICE") == "1":
                    raise RuntimeError(f"rank {self.ctx.rank}: LOCAL_RANK {self.ctx.local_rank} should own "
                                       f"{plan['pci']} but runs on {rec['pci_bus_id']}")
        else:
            rec["device"] = "cpu"
        return rec


def svc_modulus(crt) -> int:
    from .ir.bases import crt_modulus, first_primes

    return crt_modulus(crt if isinstance(crt, list) else first_primes(crt))


def run(argv=None) -> Optional[dict]:
    """Run the benchmark in this process (one rank); rank 0 returns (and bench.py prints) the JSON record,
    other ranks None."""
    args = parse_args(argv)
    from .native import native
    from .parallel import all_gather_array, all_gather_object, init_distributed, shutdown

    hip = args.backend == "hip"
    rehearsal = bool(args.rehearse_shared_device)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        raise RuntimeError(f"--gpus {args.gpus} but WORLD_SIZE={world_env}: start the bench with "
                           f"'python bench.py --gpus N' (it launches the ranks) or under torchrun with N ranks")
    if hip:
        # one process per GPU; backend nccl (= RCCL over xGMI). More ranks than GPUs only as a labelled rehearsal
        # (ranks share devices over gloo; RCCL refuses two ranks on one device).
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        ndev = visible_gpus()
        if world_env > ndev:
            if not rehearsal:
                raise RuntimeError(f"{world_env} ranks but {ndev} visible GPU(s); pass --rehearse-shared-device "
                                   f"for a (labelled) shared-device rehearsal")
            os.environ["LOCAL_RANK"] = str(int(os.environ.get("LOCAL_RANK", "0")) % max(1, ndev))
    backend = os.environ.get("DASH_DIST_BACKEND") or None
    if rehearsal and world_env > 1 and backend is None:
        backend = "gloo"
    if backend not in (None, "nccl") and hip and world_env > 1 and not rehearsal:
        raise RuntimeError(f"DASH_DIST_BACKEND={backend}: a GPU scaling run uses nccl (RCCL)")
    ctx = init_distributed(backend=backend, use_gpu=hip)
    world, rank = ctx.world, ctx.rank
    bench = _Bench(args, ctx)
    bench.threads = host_thread_budget(args.threads)
    native().set_num_threads(bench.threads)
    phases = {p.strip() for p in args.phases.split(",") if p.strip()} | {"main"}

    cons = dict(CONSTRUCTIONS[args.constructions])
    for key in ("sign", "rescale", "relu"):
        if getattr(args, key):
            cons[key] = getattr(args, key)

    # ---------------- main (headline) phase
    gcs, groups, B, G, per, off = bench.offline("main", cons, args.batch)
    resolved = gcs[0].effective_constructions()
    resolved_guard = gcs[0].guard_enabled
    free_b = total_b = None
    if hip:
        import torch

        free_b, total_b = torch.cuda.mem_get_info(bench.device)
    r = bench.online(gcs, groups, B, per, args.steps, args.warmup, 1000, args.verify)
    elapsed = r["elapsed"]
    gathered = all_gather_array(ctx, np.stack(r["last"]))  # decoded logits of the last step onto every rank
    assert gathered.shape[0] == world
    total_inf = world * B * args.steps
    value = total_inf / elapsed
    ms_step = 1000.0 * elapsed / args.steps
    recs = all_gather_object(ctx, bench.rank_record(1000.0 * r["local"] / args.steps,
                                                    B * args.steps / r["local"], r["host_ms"], B))
    prof = op_ms = None
    if args.profile and hip:
        r["step"](0)
        prof = {k: round(v, 3) for k, v in groups[0].ev.layer_times().items()}
        op_ms = [[n, round(v, 4)] for n, v in groups[0].ev.op_times()]
    verified = r["verified"]
    r_last_ok = r["verified_last_step"]

    # ---------------- threads phase: the same loop at smaller host thread budgets (an 8-rank node gives each
    # rank cores / 8); the step time must not depend on the host encode/decode
    threads = None
    if "threads" in phases:
        threads = {str(bench.threads): dict(ms_per_step=round(ms_step, 3), host_encode_decode_ms_per_step=round(
            r["host_ms"], 3))}
        for t in sorted({int(v) for v in args.thread_sweep.split(",") if v.strip()} - {bench.threads}):
            native().set_num_threads(t)
            rt = bench.online(gcs, groups, B, per, args.steps, 1, 2000 + t, 0)
            rt.pop("step")  # the closure holds the groups (all of the phase's HBM)
            threads[str(t)] = dict(ms_per_step=round(1000.0 * rt["elapsed"] / args.steps, 3),
                                   host_encode_decode_ms_per_step=round(all_reduce_max_(ctx, rt["host_ms"]), 3))
        native().set_num_threads(bench.threads)
        log(f"[threads] {threads}")
    r.pop("step")
    del gcs, groups, r

    # ---------------- latency phase: batch 1, fresh GC per inference (the reference's metric)
    lat = lat_host = lat_ref = None
    if "latency" in phases:
        lat = bench.latency(cons)
        log(f"[latency] {lat}")
        if bench.device_encode:  # the same with online message #1 in wire form (garbler and evaluator apart)
            lat_host = bench.latency(cons, device_encode=False)
            log(f"[latency host-encoded] {lat_host}")
    if "latency_ref" in phases and hip:
        # the reference's configuration exactly: its gadget constructions, its (wire-compatible, fixed-key AES)
        # encoding, inputs encoded on the host and shipped as labels, fresh GC, batch 1
        lat_ref = bench.latency(CONSTRUCTIONS["reference"], device_encode=False)
        log(f"[latency reference] {lat_ref}")

    # ---------------- reference-constructions phase (same driver, the reference's gadgets)
    ref = None
    if "reference" in phases and args.constructions != "reference":
        rc = CONSTRUCTIONS["reference"]
        rsteps = args.ref_steps or args.steps
        g2, grp2, B2, G2, per2, off2 = bench.offline("reference", rc, args.ref_batch, args.ref_streams)
        r2 = bench.online(g2, grp2, B2, per2, rsteps, max(1, min(args.warmup, 2)), 3000, args.verify)
        ref = dict(value=round(world * B2 * rsteps / r2["elapsed"], 3),
                   ms_per_step=round(1000.0 * r2["elapsed"] / rsteps, 3), gcs_per_gpu=B2, streams=G2, steps=rsteps,
                   constructions=g2[0].effective_constructions(), verified_vs_plaintext=r2["verified"],
                   verified_last_timed_step=r2["verified_last_step"],
                   gc_reuse=True,
                   offline={"garble_s_per_gc": round(off2["garble_s"] / max(1, B2), 3),
                            "table_gb_per_gc": round(off2["table_gb"], 3)})
        del g2, grp2, r2

    # ---------------- served phase (fresh GC per inference, garbling included)
    served = None
    if "served" in phases:
        served = bench.served(cons)

    out = None
    if rank == 0:
        check_world(args, ctx, recs, rehearsal)
        out = {
            "metric": ("online garbled inferences/sec (MiniONN CIFAR-10 CNN)"
                       if bench.model == "MODEL_F_MINIONN_POOL_REPL" else f"online garbled inferences/sec ({bench.model})"),
            "value": round(value, 3),
            "unit": "inferences/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "ms_per_inference": round(1000.0 * elapsed / (B * args.steps), 3),
            "latency_ms_per_batch": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            # like-for-like: the reference's 1443 ms is a batch-1 latency on a fresh GC, so vs_baseline divides it
            # by this framework's batch-1 latency (flagship constructions); the batched-throughput ratio and the
            # reference-constructions ratio are reported beside it
            "vs_baseline": (round(BASELINE_LATENCY_MS / lat["latency_b1_ms"], 1) if lat is not None
                            else round(value / BASELINE_INF_PER_S, 2)),
            "vs_baseline_throughput": round(value / BASELINE_INF_PER_S, 2),
            "dtype": "uint8 label components / int8 MFMA (exact modular arithmetic)",
            "data": f"synthetic {'CIFAR-10' if bench.circuit.input_dims[0] == 3 else 'MNIST'}-shaped inputs, random-init weights",
            "config": {
                "model": bench.model,
                "scheme": args.config,
                "crt_base": bench.cfg["crt"] if isinstance(bench.cfg["crt"], list) else native().first_primes(bench.cfg["crt"]),
                "mrs": bench.cfg["mrs"],
                "global_batch": world * B,
                "gcs_per_gpu": B,
                "streams": G,
                "constructions": args.constructions,
                "requested_constructions": cons,
                "sign_construction": resolved["sign"],
                "rescale_construction": resolved["rescale"],
                "relu_construction": resolved["relu"],
                # offline-message encoding (docs/SECURITY.md): "hardened" = no constant labels shipped and a
                # tweaked pad per table entry; "reference" = the reference's wire format
                "encoding": resolved.get("encoding", "reference"),
                "seq_len": None,
                "input_shape": list(bench.circuit.input_dims),
                "parallelism": f"dp{world}",
                "backend": args.backend,
            },
            # the headline's GCs are garbled once and re-encoded every step: an online-phase rate (a step's
            # work equals that of fresh GCs); served_inf_per_s is the protocol-valid fresh-GC rate
            "gc_reuse": True,
            "pipelined_steps": bool(args.pipeline),
            "gc_reuse_note": ("the timed steps re-encode fresh inputs under GCs garbled once; "
                              + ("online message #1 comes from the garbler's device encoder (W0 + x R per label, "
                                 "the same work for a fresh GC; no codebook)" if bench.device_encode else
                                 "a reused GC also builds a per-GC input codebook on its second encode "
                                 "(host_encode_decode_ms_per_step)")
                              + "; GCs are single use in the protocol: served_inf_per_s (fresh GC per inference, "
                              "garbling included) and latency_b1_ms (fresh GC, batch 1) measure that"),
            "input_encoding": "device" if bench.device_encode else "host",
            "input_encoding_note": ("device: the garbler's input state of each GC (base labels W0, offsets R) sits on "
                                    "the evaluator's GPU, written by the garbler's encoder; the in-process / same-node "
                                    "form of online message #1 (it does not exist in wire form). Two separate parties "
                                    "use the host (wire-form) path: latency_b1_host_encoded_ms and "
                                    "latency_b1_reference_ms measure it") if bench.device_encode else
                                   "host: online message #1 in wire form (16-B compressed labels, H2D, GPU unpack)",
            "vs_baseline_note": ("vs_baseline = 1443 ms / latency_b1_ms (batch 1, fresh GC, flagship constructions, "
                                 "hardened encoding); vs_baseline_b1_reference = 1443 ms / latency_b1_reference_ms "
                                 "(the reference's constructions and encoding, host-encoded input labels: the exact "
                                 "like-for-like); vs_baseline_throughput = value / (1 / 1.443 s), batched throughput "
                                 "over the reference's batch-1 rate"),
            "dist_backend": ctx.backend if ctx.distributed else "none",
            "world_size": world,
            "rehearsal_shared_device": rehearsal and world > 1,
            "threads_per_rank": bench.threads,
            "ranks": recs,
            "offline": {"garble_s_per_gc": round(off["garble_s"] / max(1, B), 3),
                        "upload_s_per_gc": round(off["upload_s"] / max(1, B), 3),
                        "table_gb_per_gc": round(off["table_gb"], 3), "offline_total_s": round(off["offline_s"], 1)},
            "verified_vs_plaintext": verified,
            "verified_last_timed_step": r_last_ok,
            # the garbler's exact per-input range check (garbling/guard.py, csrc/hip/guard.hip) inside the timed
            # steps, on its own stream beside the evaluation
            "range_guard": bool(resolved_guard),
        }
        if hip:
            out["hbm_gb"] = {"used": round((total_b - free_b) / 1e9, 1), "total": round(total_b / 1e9, 1)}
        if threads is not None:
            out["host_thread_sweep"] = threads
        if lat is not None:
            out["latency_b1_ms"] = lat["latency_b1_ms"]
            out["latency_b1"] = lat
        if lat_host is not None:
            out["latency_b1_host_encoded_ms"] = lat_host["latency_b1_ms"]
            out["latency_b1_host_encoded"] = lat_host
        if lat_ref is not None:
            out["latency_b1_reference_ms"] = lat_ref["latency_b1_ms"]
            out["latency_b1_reference"] = lat_ref
            out["vs_baseline_b1_reference"] = round(BASELINE_LATENCY_MS / lat_ref["latency_b1_ms"], 1)
        if ref is not None:
            out["reference_constructions_value"] = ref["value"]
            out["reference_constructions"] = ref
        if served is not None:
            out["served_inf_per_s"] = round(served["value"], 3)
            out["served"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in served.items() if k != "value"}
        if prof:
            out["layer_ms"] = prof
            out["op_ms"] = op_ms
    shutdown(ctx)
    return out


def all_reduce_max_(ctx, v: float) -> float:
    from .parallel import all_reduce_max

    return all_reduce_max(ctx, v)


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args, argv))  # parent: starts the ranks, never touches the GPU
    out = run(argv)
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
