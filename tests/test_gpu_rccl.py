"""bench.py's N > 1 path through RCCL on the GPU box's one GPU.

RCCL refuses two ranks on one device, so one rank runs under
torch.distributed.run with backend nccl and RTMI_DIST_FORCE=1: every
collective of the N-GPU run goes through RCCL — the per-context process
groups, each step's gather on its context's CU-masked stream, the barriers
and max-over-ranks reductions, the gather check against rank 0's own frame
(bit for bit), the one-shot render's gather.  What one GPU cannot show (xGMI
traffic, rank skew) is the driver's 8-GPU run."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


@pytest.mark.gpu
def test_n_rank_path_through_rccl_at_one_rank(tmp_path):
    import bench

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                                                           "RTMI_DIST_BACKEND", "RTMI_BENCH_STUB")}
    env.update(RTMI_DIST_FORCE="1", RTMI_DIST_TIMEOUT_S="120")
    cmd = bench.launch_command(1, ["--gpus", "1", "--steps", "3", "--warmup", "3", "--no-cpu-baseline", "--no-exec-counts"],
                               bench.free_port())
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = p.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout[-2000:]
    d = json.loads(lines[0])
    assert "stub" not in d and d["n_gpus"] == 1 and "RTMI_DIST_FORCE" in d["config"]["dist_rehearsal"]
    assert d["dist"]["backend"] == "nccl" and d["dist"]["world_size"] == 1
    assert d["config"]["pipeline"] == 3 and d["config"]["gather"].startswith("inline")
    assert d["dist"]["segments_per_rank"] == [d["roofline"]["segments_per_launch"]]
    gc = d["gather_check"]
    assert gc["rows"] == 800 and gc["bit_exact_vs_1gpu_frame"] is True and gc["max_abs_diff"] == 0.0
    assert d["one_shot"]["wall_ms_max_rank"] > 0 and d["one_shot_msamples_per_s"] > 0
    assert d["value"] > 0
