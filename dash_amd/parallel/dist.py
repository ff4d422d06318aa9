"""Batch data parallelism over GPUs (one process per GPU, RCCL over xGMI).

The reference is single-device (DP over inferences is "No").
Garbled inference has no cross-inference dependency, so the natural MI355X
scale-out is batch DP: every rank garbles and evaluates its own single-use
GCs with all tables resident in its own HBM, and the only collectives are

* a broadcast of the public model from rank 0 (weights are public to the
  evaluator in the DASH setting), and
* one all-gather of decoded logits per batch (10 int64 per inference),

both tiny, so scaling is bound by per-GPU throughput, not by xGMI.
Backend: ``nccl`` (= RCCL on ROCm) when a GPU is present, ``gloo`` otherwise
(CPU tests, world_size > 1 on one host).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np


KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def kfd_gpus(root: Optional[str] = None) -> list:
    """GPU agents of the KFD topology, in KFD node order (the order HIP enumerates devices), read from sysfs
    without touching the HIP runtime. Each entry: {"node", "pci" (dddd:bb:dd.f), "gfx"}. Raises when the
    topology is missing: callers must not guess a device count. ``DASH_KFD_TOPOLOGY`` overrides the sysfs root
    (tests use a synthetic topology)."""
    root = root or os.environ.get("DASH_KFD_TOPOLOGY") or KFD_TOPOLOGY
    if not os.path.isdir(root):
        raise RuntimeError(f"KFD topology {root} not readable: cannot count GPUs without initialising HIP")
    out = []
    for name in sorted(os.listdir(root), key=lambda s: int(s) if s.isdigit() else 1 << 30):
        if not name.isdigit():
            continue
        props = {}
        try:
            with open(os.path.join(root, name, "properties")) as f:
                for line in f:
                    parts = line.split()
                    if len(parts) == 2 and parts[1].lstrip("-").isdigit():
                        props[parts[0]] = int(parts[1])
        except OSError:
            continue
        if props.get("simd_count", 0) <= 0 or props.get("gfx_target_version", 0) == 0:
            continue  # CPU agent
        loc, dom = props.get("location_id", 0), props.get("domain", 0)
        pci = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"
        out.append({"node": int(name), "pci": pci, "gfx": props.get("gfx_target_version", 0),
                    "unique_id": props.get("unique_id"), "render_minor": props.get("drm_render_minor")})
    return _accessible(out)


def _accessible(gpus: list) -> list:
    """The GPUs whose DRM render node this process may open (HIP enumerates only those; sysfs is not namespaced,
    so a container sees every GPU of the host there). Unfiltered when no render node can be checked at all
    (no /dev/dri, or no node lists its render minor): never guess a smaller count from missing information."""
    dri = os.environ.get("DASH_DRI_DIR", "/dev/dri")
    if not os.path.isdir(dri) or not any(g.get("render_minor") is not None for g in gpus):
        return gpus
    ok = [g for g in gpus if g.get("render_minor") is None
          or os.access(os.path.join(dri, f"renderD{g['render_minor']}"), os.R_OK | os.W_OK)]
    return ok if ok else gpus


def visible_indices(n: int, env: Optional[dict] = None, gpus: Optional[list] = None) -> list:
    """Indices (into the KFD GPU list) a HIP process started with `env` would see: ROCR_VISIBLE_DEVICES
    filters first, then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES index into what remains. Entries are
    ordinals or (ROCR_VISIBLE_DEVICES) UUIDs ``GPU-<16 hex digits of the KFD unique_id>``, matched against
    `gpus` (kfd_gpus entries); an entry that matches nothing ends the list, as in HIP."""
    env = os.environ if env is None else env
    idx = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is None:
            continue
        v = v.strip()
        if v == "":
            return []
        sel = []
        for tok in v.split(","):
            tok = tok.strip()
            if tok.isdigit() and int(tok) < len(idx):
                sel.append(idx[int(tok)])
            elif tok.upper().startswith("GPU-") and gpus is not None:
                want = tok[4:].lower()
                hit = [i for i in idx if gpus[i].get("unique_id") is not None
                       and f"{gpus[i]['unique_id']:016x}" == want.rjust(16, "0")]
                if not hit:
                    break
                sel.append(hit[0])
            else:
                break  # HIP stops at the first invalid entry
        idx = sel
    return idx


def rank_gpu(local_rank: int, env: Optional[dict] = None) -> Optional[dict]:
    """The GPU a rank with this LOCAL_RANK owns, from sysfs only (no HIP call): HIP device index = LOCAL_RANK
    within the visible devices, plus the KFD node and PCI address behind it. None when the topology is unknown
    or LOCAL_RANK is beyond the visible GPUs (a shared-device rehearsal maps ranks modulo the GPU count first)."""
    try:
        gpus = kfd_gpus()
    except RuntimeError:
        return None
    vis = visible_indices(len(gpus), env, gpus)
    if not 0 <= local_rank < len(vis):
        return None
    g = gpus[vis[local_rank]]
    return {"device": local_rank, "kfd_node": g["node"], "pci": g["pci"]}


def gpu_local_cpus(local_rank: int) -> Optional[set]:
    """CPUs of the NUMA node closest to the GPU a rank with this LOCAL_RANK uses (PCI local_cpulist), or None
    when unknown. Sysfs only: safe before the first HIP call."""
    try:
        gpus = kfd_gpus()
    except RuntimeError:
        return None
    vis = visible_indices(len(gpus), None, gpus)
    if local_rank >= len(vis):
        return None
    path = f"/sys/bus/pci/devices/{gpus[vis[local_rank]]['pci']}/local_cpulist"
    try:
        with open(path) as f:
            spec = f.read().strip()
    except OSError:
        return None
    cpus = set()
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus or None


def bind_rank_affinity(local_rank: int) -> Optional[list]:
    """Pin this process to the CPUs local to its GPU (intersected with the CPUs it may use) before HIP starts,
    so host encode / decode / garbling threads of 8 ranks do not cross NUMA nodes. Returns the CPU list set, or
    None when the topology is unknown or the intersection is empty (affinity unchanged)."""
    cpus = gpu_local_cpus(local_rank)
    if not cpus or not hasattr(os, "sched_setaffinity"):
        return None
    allowed = os.sched_getaffinity(0)
    mine = sorted(cpus & allowed)
    if not mine:
        return None
    os.sched_setaffinity(0, mine)
    return mine


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: Optional[int] = None

    @property
    def distributed(self) -> bool:
        return self.world > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_distributed(backend: Optional[str] = None, use_gpu: Optional[bool] = None,
                     timeout_s: Optional[float] = None) -> DistContext:
    """Initialise torch.distributed from the torchrun environment (RANK,
    WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT). Single process -> no-op.

    Failure detection (the reference has none): collectives time
    out after ``timeout_s`` (default ``DASH_DIST_TIMEOUT_S`` or 600 s) instead
    of hanging forever, and RCCL async error handling tears the process group
    down on a timed-out or failed collective so the rank exits and the
    launcher (torchrun elastic) can restart it."""
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and os.environ.get("DASH_NUMA_BIND", "1") != "0":
        bind_rank_affinity(local)  # sysfs only, before torch.cuda touches HIP
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    dev = None
    if use_gpu:
        torch.cuda.set_device(local)
        dev = local
    if world <= 1:
        return DistContext(rank, 1, local, "none", dev)
    import torch.distributed as dist

    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    if not dist.is_initialized():
        import datetime

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        if timeout_s is None:
            timeout_s = float(os.environ.get("DASH_DIST_TIMEOUT_S", "600"))
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s))
    return DistContext(dist.get_rank(), dist.get_world_size(), local, backend, dev)


def shutdown(ctx: DistContext) -> None:
    if ctx.distributed:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()


def broadcast_object(ctx: DistContext, obj=None, src: int = 0):
    """Broadcast a picklable object (e.g. the public Circuit) from `src`.
    Objects only ever come from ranks of the same job, never from files."""
    if not ctx.distributed:
        return obj
    import torch.distributed as dist

    box = [obj if ctx.rank == src else None]
    dist.broadcast_object_list(box, src=src)
    return box[0]


def _tensor_device(ctx: DistContext):
    import torch

    return torch.device("cuda", ctx.device) if ctx.backend == "nccl" else torch.device("cpu")


def all_gather_array(ctx: DistContext, a: np.ndarray) -> np.ndarray:
    """All-gather equally shaped int64 arrays -> stacked [world, ...]."""
    a = np.ascontiguousarray(a, dtype=np.int64)
    if not ctx.distributed:
        return a[None]
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(a).to(_tensor_device(ctx))
    out = [torch.empty_like(t) for _ in range(ctx.world)]
    dist.all_gather(out, t)
    return np.stack([o.cpu().numpy() for o in out])


def all_reduce_max(ctx: DistContext, v: float) -> float:
    if not ctx.distributed:
        return float(v)
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(v)], dtype=torch.float64, device=_tensor_device(ctx))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_min(ctx: DistContext, v: float) -> float:
    return -all_reduce_max(ctx, -float(v))


def all_gather_object(ctx: DistContext, obj) -> list:
    """Gather one small picklable record per rank (rank order). Records come
    only from ranks of this job."""
    if not ctx.distributed:
        return [obj]
    import torch.distributed as dist

    out = [None] * ctx.world
    dist.all_gather_object(out, obj)
    return out


def barrier(ctx: DistContext) -> None:
    if ctx.distributed:
        import torch.distributed as dist

        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device])
        else:
            dist.barrier()


def shard(n: int, ctx: DistContext) -> range:
    """Contiguous shard of n items for this rank (sizes differ by at most 1)."""
    base, rem = divmod(n, ctx.world)
    start = ctx.rank * base + min(ctx.rank, rem)
    return range(start, start + base + (1 if ctx.rank < rem else 0))


class BatchDataParallel:
    """Data-parallel garbled inference: each rank owns `per_rank` fresh GCs per
    round and evaluates them on its GPU (`backend="hip"`) or on the CPU
    oracle (`backend="cpu"`); outputs are all-gathered in global order.

    Every round garbles new circuits (GCs are single use). With the ``hip``
    backend they are garbled on the rank's own GPU (byte-identical to the host
    garbler), so N ranks never compete for the shared host cores; the gadget
    constructions default to GarbledCircuit's ("auto": the mixed-radix rescale
    and joint ReLU where the CRT base and tracked ranges allow)."""

    def __init__(self, ctx: DistContext, circuit, crt, mrs=None, per_rank: int = 1, backend: str = "hip",
                 max_modulus: int = 0, seed: Optional[bytes] = None, garble_device: Optional[bool] = None,
                 **gc_kw):
        self.ctx, self.circuit, self.crt, self.mrs = ctx, circuit, crt, mrs
        self.per_rank, self.backend, self.max_modulus = per_rank, backend, max_modulus
        self.seed = seed
        self.garble_device = (backend == "hip") if garble_device is None else bool(garble_device)
        self.gc_kw = gc_kw
        self.round = 0
        self.ev = None

    def _seed(self, b: int) -> Optional[bytes]:
        if self.seed is None:
            return None
        import hashlib

        return hashlib.sha256(self.seed + f"/{self.ctx.rank}/{self.round}/{b}".encode()).digest()[:16]

    def infer(self, inputs: Sequence) -> np.ndarray:
        """inputs: exactly world * per_rank quantized inputs (global batch) -> [global, n_out]."""
        from ..garbling import GarbledCircuit

        ctx = self.ctx
        assert len(inputs) == ctx.world * self.per_rank, "global batch must be world * per_rank"
        mine = inputs[ctx.rank * self.per_rank:(ctx.rank + 1) * self.per_rank]
        dev = (ctx.device or 0) if self.garble_device else None
        if self.backend == "hip":
            # the bench's path (benchcore._HipGroup): GCs garbled straight into the evaluator's slots (sink),
            # online message #1 from the garbler's device encoder, the garbler's range guard beside the run
            from ..benchcore import _HipGroup

            gcs = []
            for b in range(self.per_rank):
                sink = self.ev.sink(b) if (self.ev is not None and dev is not None) else None
                gc = GarbledCircuit(self.circuit, self.crt, self.mrs, max_modulus=self.max_modulus,
                                    seed=self._seed(b), device=dev, sink=sink, **self.gc_kw)
                if self.ev is None:
                    self.ev = _HipGroup(gc.model, self.per_rank, ctx.device or 0, True, False, None,
                                        device_encode=True)
                self.ev.load(b, gc)
                gcs.append(gc)
            self.round += 1
            self.ev.encode_batch(gcs, mine)
            self.ev.launch()
            pend = gcs[0].guard.submit(mine) if gcs[0].guard_enabled else None
            self.ev.fetch()
            outs = np.stack([self.ev.decode(b, gc) for b, gc in enumerate(gcs)])
            if pend is not None:
                pend.raise_if_bad()  # no result leaves the rank before the garbler's range check passed
        else:
            gcs = [GarbledCircuit(self.circuit, self.crt, self.mrs, max_modulus=self.max_modulus, seed=self._seed(b),
                                  device=dev, **self.gc_kw)
                   for b in range(self.per_rank)]
            self.round += 1
            outs = np.stack([gc.decode_outputs(gc.cpu_evaluate(gc.garble_inputs(x))) for gc, x in zip(gcs, mine)])
        return all_gather_array(ctx, outs).reshape(ctx.world * self.per_rank, -1)
