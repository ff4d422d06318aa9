"""Batch-DP over torch.distributed with the gloo backend, world_size 2, 4 and 8 (CPU).
The same code path runs with nccl (RCCL) on GPUs (bench.py, --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as tmp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from dash_amd.garbling import GarbledCircuit
    from dash_amd.models import build_circuit, quantized_inputs
    from dash_amd.parallel import BatchDataParallel, broadcast_object, init_distributed, shard, shutdown

    ctx = init_distributed(use_gpu=False)
    circuit = broadcast_object(ctx, build_circuit("MODEL_A") if ctx.rank == 0 else None)
    xs = broadcast_object(ctx, quantized_inputs("MODEL_A", world * 2) if ctx.rank == 0 else None)
    dp = BatchDataParallel(ctx, circuit, 7, 100.0, per_rank=2, backend="cpu", seed=b"dp-test")
    out = dp.infer(xs)
    ref = np.stack([GarbledCircuit(circuit, 7, 100.0, seed=bytes(16), garble_me=False).plain_q_eval(x) for x in xs])
    q.put((rank, bool(np.array_equal(out, ref)), list(shard(5, ctx))))
    shutdown(ctx)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_batch_dp_gloo(world):
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res)
    # contiguous balanced shards of 5 items: the first 5 % world ranks get one extra
    sizes = [len(r[2]) for r in res]
    assert sum(sizes) == 5 and max(sizes) - min(sizes) <= 1
    assert [i for r in res for i in r[2]] == list(range(5))


def _bench_worker(rank, world, port, q, local_rank=None, env=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank if local_rank is None else local_rank),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **(env or {}))
    from dash_amd import benchcore

    out = benchcore.run(["--backend", "cpu", "--gpus", str(world), "--model", "MODEL_A", "--batch", "2", "--streams",
                         "1", "--steps", "2", "--warmup", "1", "--phases", "main,served", "--served-slots", "2",
                         "--served-groups", "2", "--served-requests", "1", "--served-min-s", "0"])
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_driver_gloo(world):
    """bench.py's own driver (dash_amd.benchcore) over gloo: the ranks agree on the batch, the JSON carries the
    backend, world size and one record per rank, and every rank's outputs match the plaintext evaluation."""
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out = res[0]
    assert all(res[r] is None for r in range(1, world))
    assert out["n_gpus"] == world and out["world_size"] == world and out["dist_backend"] == "gloo"
    assert out["config"]["global_batch"] == 2 * world and out["config"]["parallelism"] == f"dp{world}"
    assert [r["rank"] for r in out["ranks"]] == list(range(world))
    assert all(r["gcs"] == 2 and r["ms_per_step"] > 0 and r["host_encode_decode_ms_per_step"] >= 0
               for r in out["ranks"])
    assert out["verified_vs_plaintext"] and out["served"]["verified"]
    assert out["value"] > 0 and out["served_inf_per_s"] > 0
    # the headline value is the whole-job rate over the slowest rank's time
    assert abs(out["value"] - world * 2 * 2 / (out["ms_per_step"] * 2 / 1000.0)) / out["value"] < 0.01


def _fake_kfd(root, n_gpus, ids=False):
    """A KFD topology like an MI355X node's: node 0 a CPU agent, nodes 1..n GPUs on distinct PCI buses (ids: with
    unique_id and drm_render_minor 128 + i)."""
    os.makedirs(os.path.join(root, "0"))
    with open(os.path.join(root, "0", "properties"), "w") as f:
        f.write("cpu_cores_count 96\nsimd_count 0\ngfx_target_version 0\n")
    buses = []
    for i in range(n_gpus):
        bus = 0x05 + 0x20 * i
        os.makedirs(os.path.join(root, str(i + 1)))
        with open(os.path.join(root, str(i + 1), "properties"), "w") as f:
            f.write(f"simd_count 1024\ngfx_target_version 90500\nlocation_id {bus << 8}\ndomain 0\n")
            if ids:
                f.write(f"unique_id {0x1234abcd0000 + i}\ndrm_render_minor {128 + i}\n")
        buses.append(f"0000:{bus:02x}:00.0")
    return buses


def test_visible_gpus_uuid_and_render_nodes(tmp_path, monkeypatch):
    """ROCR_VISIBLE_DEVICES may name GPUs by UUID (GPU-<unique_id hex>); sysfs lists every GPU of the host, but
    only those whose render node this process can open are enumerated by HIP (a container's share)."""
    from dash_amd.parallel.dist import kfd_gpus, rank_gpu, visible_indices

    buses = _fake_kfd(str(tmp_path / "kfd"), 8, ids=True)
    monkeypatch.setenv("DASH_KFD_TOPOLOGY", str(tmp_path / "kfd"))
    dri = tmp_path / "dri"
    dri.mkdir()
    monkeypatch.setenv("DASH_DRI_DIR", str(dri))
    for i in (2, 5):  # this "container" owns GPUs 2 and 5
        (dri / f"renderD{128 + i}").write_text("")
    gpus = kfd_gpus()
    assert [g["pci"] for g in gpus] == [buses[2], buses[5]]
    uid5 = f"GPU-{0x1234abcd0000 + 5:016x}"
    assert visible_indices(len(gpus), {"ROCR_VISIBLE_DEVICES": uid5}, gpus) == [1]
    assert visible_indices(len(gpus), {"ROCR_VISIBLE_DEVICES": f"{uid5},GPU-ffff"}, gpus) == [1]  # stops at a miss
    assert rank_gpu(0, {"ROCR_VISIBLE_DEVICES": uid5})["pci"] == buses[5]
    # nothing checkable (no render node accessible): the full list, never a guessed smaller count
    for f in dri.iterdir():
        f.unlink()
    assert len(kfd_gpus()) == 8


def test_rank_gpu_follows_local_rank(tmp_path):
    """LOCAL_RANK (not RANK) picks the GPU, inside the visible set, from sysfs alone."""
    from dash_amd.parallel.dist import rank_gpu

    buses = _fake_kfd(str(tmp_path / "kfd"), 8)
    env = {"DASH_KFD_TOPOLOGY": str(tmp_path / "kfd")}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        assert rank_gpu(3, {}) == {"device": 3, "kfd_node": 4, "pci": buses[3]}
        # HIP_VISIBLE_DEVICES=4,5,6,7: device 3 of the rank is the node's 8th GPU
        assert rank_gpu(3, {"HIP_VISIBLE_DEVICES": "4,5,6,7"})["pci"] == buses[7]
        assert rank_gpu(4, {"HIP_VISIBLE_DEVICES": "4,5,6,7"}) is None
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_bench_driver_records_local_rank_gpu(tmp_path):
    """The bench driver over gloo with LOCAL_RANK permuted against RANK (rank r has LOCAL_RANK 3 - r): every
    rank records the GPU of its LOCAL_RANK (device index, KFD node, PCI address) from a synthetic 4-GPU topology."""
    buses = _fake_kfd(str(tmp_path / "kfd"), 4)
    world = 4
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env = {"DASH_KFD_TOPOLOGY": str(tmp_path / "kfd"), "DASH_NUMA_BIND": "0", "HIP_VISIBLE_DEVICES": "0,1,2,3"}
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q, world - 1 - r, env)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    recs = res[0]["ranks"]
    assert [r["rank"] for r in recs] == [0, 1, 2, 3]
    for r in recs:
        assert r["local_rank"] == world - 1 - r["rank"]
        assert r["gpu_plan"] == {"device": r["local_rank"], "kfd_node": r["local_rank"] + 1,
                                 "pci": buses[r["local_rank"]]}


def test_single_process_context():
    from dash_amd.parallel import all_gather_array, init_distributed

    ctx = init_distributed(use_gpu=False)
    assert ctx.world == 1 and not ctx.distributed
    np.testing.assert_array_equal(all_gather_array(ctx, np.arange(3)), [[0, 1, 2]])


@pytest.mark.gpu
def test_batch_dp_hip_single_rank():
    from dash_amd.garbling import GarbledCircuit
    from dash_amd.models import build_circuit, quantized_inputs
    from dash_amd.parallel import BatchDataParallel, init_distributed

    ctx = init_distributed(use_gpu=True)
    c = build_circuit("MODEL_A")
    xs = quantized_inputs("MODEL_A", 3)
    dp = BatchDataParallel(ctx, c, 7, 100.0, per_rank=3, backend="hip")
    for _ in range(2):  # fresh GCs every round, evaluator reused
        out = dp.infer(xs)
        ref = GarbledCircuit(c, 7, 100.0, garble_me=False)
        np.testing.assert_array_equal(out, np.stack([ref.plain_q_eval(x) for x in xs]))


def _run_bench_cli(args, timeout=600):
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    return subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=root)


def test_bench_cli_spawns_ranks():
    """`python bench.py --gpus 4` with no launcher starts 4 fresh ranks itself (no torchrun by the caller) and
    prints rank 0's record with world size 4 and one record per rank."""
    import json

    p = _run_bench_cli(["--backend", "cpu", "--gpus", "4", "--model", "MODEL_A", "--batch", "2", "--streams", "1",
                        "--steps", "2", "--warmup", "1", "--phases", "main,latency", "--latency-gcs", "2"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["world_size"] == 4 and out["dist_backend"] == "gloo"
    assert [r["rank"] for r in out["ranks"]] == [0, 1, 2, 3]
    assert len({r["pid"] for r in out["ranks"]}) == 4
    assert out["gc_reuse"] is True and out["latency_b1"]["verified"] and out["latency_b1_ms"] > 0
    assert out["config"]["rescale_construction"] in ("mrs", "legacy", "none")


def test_bench_cli_refuses_world_mismatch():
    """Under a launcher, --gpus must equal WORLD_SIZE (a 1-rank job never reports itself as N GPUs)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--backend", "cpu", "--gpus", "2",
                        "--model", "MODEL_A", "--batch", "2", "--steps", "1", "--phases", "main"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_bench_cli_refuses_missing_gpus():
    """--gpus N on a host with fewer visible GPUs fails loudly unless the shared-device rehearsal is asked for."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("host has 2+ GPUs")
    p = _run_bench_cli(["--gpus", "2", "--steps", "1"], timeout=300)
    assert p.returncode == 2 and "refusing" in p.stderr


@pytest.mark.parametrize("pipeline", [0, 1])
def test_bench_pipelined_groups_verified(pipeline, monkeypatch):
    """The online loop with two groups, stepped (0) or with each group's next step launched as soon as its outputs
    are decoded (1): the first and the last timed step both match the plaintext model."""
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    from dash_amd import benchcore

    out = benchcore.run(["--backend", "cpu", "--gpus", "1", "--model", "MODEL_A", "--batch", "4", "--streams", "2",
                         "--steps", "3", "--warmup", "2", "--phases", "main", "--pipeline", str(pipeline)])
    assert out["pipelined_steps"] == bool(pipeline)
    assert out["config"]["streams"] == 2 and out["config"]["global_batch"] == 4
    assert out["verified_vs_plaintext"] and out["verified_last_timed_step"]
