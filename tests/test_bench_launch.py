"""bench.py's rank plumbing (CPU): ``--gpus N`` without a torchrun environment starts N ranks
itself and the line reports the ranks that ran; ``--gpus`` disagreeing with WORLD_SIZE is an
error; the row split of BASELINE.md §2's multi-GPU synthetic.  The GPU legs themselves run in
tests/test_bench_gpu.py (2 gloo ranks sharing the one card) and in the driver's N-GPU runs."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-check"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    line = lines[0]
    assert line["n_gpus"] == n and line["ranks_seen"] == n
    assert sorted(x["rank"] for x in line["ranks"]) == list(range(n))
    assert sorted(x["local_rank"] for x in line["ranks"]) == list(range(n))
    assert len({x["pid"] for x in line["ranks"]}) == n


def test_gpus_mismatch_with_world_size_fails():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 7, 8, 16])
def test_row_blocks_cover_the_weight(world):
    import bench
    blocks, blk = bench.row_blocks(bench.ROWS, world)
    assert blk % 8 == 0 and len(blocks) == world
    assert blocks[0][0] == 0 and blocks[-1][1] == bench.ROWS
    for (a0, a1), (b0, _) in zip(blocks, blocks[1:]):
        assert a1 == b0
    for r0, r1 in blocks:
        assert 0 <= r1 - r0 <= blk and r0 % 8 == 0
