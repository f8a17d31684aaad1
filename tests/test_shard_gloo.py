"""CPU, world_size 2 over gloo: the batch-sharded (data-parallel) hot path gives the same
result as one process over the whole batch, and the helpers' collectives behave.

The per-shard compute here is the CPU oracle (tests may use it as the checker); on GPUs the
same sharding runs the HIP path (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pwcnet_amd.shard import broadcast_module, gather_to, max_over_ranks, shard, shard_bounds


def test_shard_bounds_partition():
    for total in (0, 1, 7, 8, 64, 65):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi = shard_bounds(total, world, r)
                assert 0 <= lo <= hi <= total
                seen.extend(range(lo, hi))
            assert seen == list(range(total))
    with pytest.raises(ValueError):
        shard_bounds(8, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _hot_path_cpu(x1, x2, flow):
    """warp -> Correlation(9,1,9,1,2) on the oracle (the checker, CPU)."""
    from oracle import oracle as O
    w = O.warp_forward(x2, flow, dtype=np.float32)
    return O.corr_forward(x1, w, 9, 1, 9, 1, 2, dtype=np.float32)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        B, C, H, W = 5, 8, 12, 14  # odd batch: shards of 3 and 2
        x1 = torch.randn(B, C, H, W, generator=g)
        x2 = torch.randn(B, C, H, W, generator=g)
        fl = torch.randn(B, 2, H, W, generator=g) * 2
        out = torch.from_numpy(_hot_path_cpu(shard(x1, world, rank).numpy(),
                                             shard(x2, world, rank).numpy(),
                                             shard(fl, world, rank).numpy()))
        full = gather_to(out, dst=0)
        m = torch.nn.Linear(3, 2)
        torch.manual_seed(100 + rank)  # ranks start different ...
        torch.nn.init.normal_(m.weight)
        broadcast_module(m, src=0)      # ... and end equal to rank 0
        wsum = float(m.weight.sum())
        mx = max_over_ranks(float(rank + 1))
        if rank == 0:
            ref = _hot_path_cpu(x1.numpy(), x2.numpy(), fl.numpy())
            q.put(("ok", float(np.abs(full.numpy() - ref).max()), tuple(full.shape), wsum, mx))
        else:
            q.put(("rank1", wsum, mx))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_hot_path_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0 = [r for r in res if r[0] == "ok"][0]
    r1 = [r for r in res if r[0] == "rank1"][0]
    assert r0[1] == 0.0 and r0[2] == (5, 81, 12, 14)  # bit-identical: same per-item arithmetic
    assert r0[3] == r1[1]                               # parameters broadcast from rank 0
    assert r0[4] == r1[2] == 2.0                        # max over ranks


def test_bench_launcher_two_ranks_cpu_rehearsal():
    """bench.py --gpus 2 starts its own two ranks (torch.distributed.run child), shards the
    checked pairs, broadcasts the Net harness weights from rank 0 and verifies every rank's
    per-pair checksums against rank 0's recomputation (launcher rehearsal on gloo, with the
    torch-CPU stand-in for the per-shard op)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--device", "cpu",
                        "--gpus", "2", "--height", "128", "--width", "128", "--batch", "2",
                        "--steps", "2", "--warmup", "1"], capture_output=True, text=True,
                       timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 4
    assert d["checks"]["replay"] is True
    assert d["checks"]["shards"] == {"pairs": 4, "ranks": 2, "ok": True, "bad_ranks": []}
    assert d["checks"]["weights_broadcast"]["ok"] is True
    assert d["checks"]["weights_broadcast"]["bytes"] == 20475776
    assert d["checks"]["weights_broadcast"]["seconds"] >= 0
    # every rank's own step time, the headline being their MAX
    assert len(d["per_rank_ms_per_step"]) == 2
    assert abs(max(d["per_rank_ms_per_step"]) - d["ms_per_step"]) <= 1e-4 * d["ms_per_step"] + 1e-4


def test_bench_rejects_gpus_world_mismatch():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--device", "cpu",
                        "--gpus", "2"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
