"""bench.py's multi-rank legs on the GPU: ``--gpus 2`` starts two ranks itself; on the one-GPU
box they share cuda:0 over gloo (QZ_BENCH_BACKEND=gloo -- RCCL refuses two ranks on one
device), which runs the same code as the driver's N-GPU RCCL runs: barriers, max-over-ranks
timing, the row-sharded synthetic with its all-gather (checked bit for bit against one
whole-weight quantize) and the sharded whole-model plan with gather_state."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_gloo(cuda):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["QZ_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--no-extras", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = lines[0]
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2
    rs = line["row_sharded_synthetic_11008x4096"]
    assert rs["gathered_equals_single_gpu"] is True
    assert rs["kernel_only"]["params_per_s"] > 0 and rs["end_to_end"]["params_per_s"] > 0
    st = line["strong_scaling_qwen3_4b_sharded"]
    assert st["units_total"] == 252 and st["end_to_end"]["tensors_on_every_rank"] == 2 * 252
