"""bench.py's N > 1 path on the CPU (VERDICT r03 "make the first real N > 1
run boring"): `bench.py --gpus N` starts N ranks itself through
torch.distributed.run (launch()), each rank joins the process group
(dist_setup(), gloo), renders its interleaved strip, the strips meet on rank 0
in one gather, rank 0 checks the un-permuted image against its own whole-frame
render and prints the line.  The renderer is bench.StubRenderer (each pixel
holds its image coordinates: partition-invariant like the product's RNG keys;
RTMI_BENCH_STUB=1), so this rehearses everything but the GPU.  The line's
schema is what the driver's SCALE run reads."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n,pipeline", [(2, None), (3, 2), (2, 1), (8, None)])
def test_bench_n_ranks_line_schema(n, pipeline, tmp_path):
    """The steps alternate over the render contexts (3 by default when they
    gather, each with two strip buffers); 7 timed steps reuse buffers after
    their gathers."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(RTMI_DIST_BACKEND="gloo", RTMI_BENCH_STUB="1", OMP_NUM_THREADS="1")
    steps = 7
    pa = ["--pipeline", str(pipeline)] if pipeline else []
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", str(steps), "--warmup", "1",
                        *pa], capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    pipeline = pipeline or 3
    assert p.returncode == 0, p.stderr[-3000:]
    lines = p.stdout.splitlines()
    # rank 0 prints ONE line and nothing else reaches stdout (gloo's start-up
    # chatter included: bench.init_group)
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["stub"] is True and d["data"].startswith("STUB")
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == 1 and d["scaling"] == "strong"
    assert d["config"]["pipeline"] == pipeline
    assert d["unit"] == "Msamples/s" and d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["partition"] == "interleaved rows, one RCCL gather"
    assert d["config"]["gather"].startswith("inline")  # per-context process groups (the default)
    di = d["dist"]
    assert di["backend"] == "gloo" and di["world_size"] == n
    for key in ("kernel_ms_per_rank", "gather_ms_per_rank", "segments_per_rank", "wall_s_per_rank"):
        assert len(di[key]) == n, key
    # every pixel-sample of the 1200x800x500 frame exactly once over the ranks
    # (800 rows are ragged over 3 ranks: padded strips count nothing)
    assert sum(di["segments_per_rank"]) == 1200 * 800 * 500
    assert di["kernel_imbalance"] >= 1.0
    # timed steps: gather k on its context's stream, render k+1 on the other's
    assert ("while step k+1 renders on the other context" if pipeline > 1 else "between renders k and k+1") in di["gather_note"]
    gc = d["gather_check"]
    assert gc["rows"] == 800 and gc["bit_exact_vs_1gpu_frame"] is True and gc["max_abs_diff"] == 0.0
    assert "cpu_baseline" not in d  # rank 0 at N = 1 only
    assert d["roofline"]["kernel_ms_max_rank"] == max(di["kernel_ms_per_rank"])
    # the single-render figure beside the pipelined value —
    # one render of the whole frame plus its blocking gather, max over ranks
    os_ = d["one_shot"]
    assert os_["wall_ms_max_rank"] > 0 and "max over ranks" in os_["note"]
    assert d["one_shot_msamples_per_s"] == os_["msamples_per_s"]
    assert abs(os_["msamples_per_s"] - 1200 * 800 * 500 / (os_["wall_ms_max_rank"] * 1e-3) / 1e6) <= 1e-3 * os_["msamples_per_s"] + 1e-3


def test_stub_requires_gloo():
    env = dict(os.environ, RTMI_BENCH_STUB="1", RTMI_DIST_BACKEND="nccl")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "1"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert p.returncode != 0 and "needs RTMI_DIST_BACKEND=gloo" in p.stderr


def test_stalled_rank_fails_fast_with_rank_and_collective_named(tmp_path):
    """a rank that stalls past the collective timeout
    (here rank 1 sleeps 120 s before its first gather, the timeout is 4 s)
    ends the whole run non-zero well inside the stall, with the failing rank
    and the collective named on stderr and nothing on stdout (no partial
    line).  Replaces the reference's error behaviour, check_cuda's exit(99)
    (accelerated-rt-cuda/final.cu:13-24)."""
    import time

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(RTMI_DIST_BACKEND="gloo", RTMI_BENCH_STUB="1", OMP_NUM_THREADS="1", RTMI_DIST_TIMEOUT_S="4",
               RTMI_BENCH_STALL_RANK="1", RTMI_BENCH_STALL_S="120")
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=110, env=env, cwd=str(tmp_path))
    took = time.monotonic() - t0
    assert p.returncode != 0
    assert took < 100, took  # not the stall's 120 s, nor torch's 10-minute default
    assert p.stdout.strip() == "", p.stdout[-2000:]
    assert "bench: rank 0 of 2: collective failed (timeout 4 s): gather of step 1's strips" in p.stderr, p.stderr[-3000:]


def test_forced_one_rank_runs_the_n_rank_path(tmp_path):
    """RTMI_DIST_FORCE=1 under the launcher at world size 1: the process group
    and every collective of the N > 1 path run with one rank (the GPU box's
    one-rank RCCL rehearsal, tools/gpu_rccl_one_rank.sh); the line says so and
    carries the dist fields, the gather check and the one-shot wall figure."""
    sys.path.insert(0, REPO)
    import bench

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(RTMI_DIST_BACKEND="gloo", RTMI_BENCH_STUB="1", OMP_NUM_THREADS="1", RTMI_DIST_FORCE="1")
    cmd = bench.launch_command(1, ["--gpus", "1", "--steps", "3", "--warmup", "1"], bench.free_port())
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = p.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and "RTMI_DIST_FORCE" in d["config"]["dist_rehearsal"]
    assert d["config"]["partition"] == "interleaved rows, one RCCL gather"
    assert d["dist"]["world_size"] == 1 and d["dist"]["segments_per_rank"] == [1200 * 800 * 500]
    assert d["gather_check"]["bit_exact_vs_1gpu_frame"] is True
    assert d["one_shot"]["wall_ms_max_rank"] > 0
    assert "cpu_baseline" not in d


def test_force_without_launcher_is_the_plain_path(tmp_path):
    """RTMI_DIST_FORCE without a launcher environment changes nothing."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(RTMI_DIST_BACKEND="gloo", RTMI_BENCH_STUB="1", OMP_NUM_THREADS="1", RTMI_DIST_FORCE="1")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.splitlines()[-1])
    assert "dist" not in d and "dist_rehearsal" not in d["config"] and d["config"]["partition"] == "single GPU"



@pytest.mark.parametrize("n,mode", [(2, "side"), (3, "side")])
def test_side_gathers(n, mode, tmp_path):
    """RTMI_BENCH_GATHER=side: the gathers as async collectives of the default
    group (the default, inline, is what test_bench_n_ranks_line_schema runs);
    the line and the gather check are the same."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(RTMI_DIST_BACKEND="gloo", RTMI_BENCH_STUB="1", OMP_NUM_THREADS="1", RTMI_BENCH_GATHER=mode)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.splitlines()[-1])
    assert d["config"]["gather"].startswith("side")
    assert d["dist"]["world_size"] == n and sum(d["dist"]["segments_per_rank"]) == 1200 * 800 * 500
    assert d["gather_check"]["bit_exact_vs_1gpu_frame"] is True
