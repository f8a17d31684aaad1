"""The N > 1 path on a one-GPU box: bench.py --gpus 2 with both ranks on cuda:0
and the collectives over gloo on CPU copies -- the launcher (torch.distributed.run child), the
batch sharding, the HIP hot path per shard, the weight broadcast and the per-pair shard check
(rank 0 recomputes every rank's pairs) together.  The production N > 1 path is the same code
with --dist-backend nccl (RCCL) and one GPU per rank (main.py:43,141 is single-device; SURVEY
§8e)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_on_one_gpu_over_gloo():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend",
           "gloo", "--same-device", "--steps", "5", "--warmup", "2", "--sets", "1",
           "--no-cpu-baseline", "--no-pmc", "--no-net-forward", "--no-corr4",
           "--grouped-mode", "off"]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 16
    assert d["config"]["parallelism"].startswith("REHEARSAL")
    assert d["checks"]["shards"] == {"pairs": 16, "ranks": 2, "ok": True, "bad_ranks": []}
    assert d["checks"]["weights_broadcast"]["ok"] is True
    assert d["checks"]["replay"] is True
    assert len(d["per_rank_ms_per_step"]) == 2 and d["value"] > 0
