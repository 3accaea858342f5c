"""bench.py host logic (CPU): workload table, the Next-Week work-equivalent
FLOP count over the flattened scenes, and the strip partition it uses."""
import os
import sys
import pytest


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
import a_dive_into_ray_tracing_amd.nextweek as nw  # noqa: E402


def test_rtiow_workloads_are_baseline_configs():
    assert bench.RTIOW_WORKLOADS["config2"] == (1200, 800, 500)
    assert bench.RTIOW_WORKLOADS["config4"] == (1200, 800, 5000)
    assert bench.RTIOW_WORKLOADS["config5"] == (3840, 2160, 2000)


def test_nw_flop_per_segment_counts_every_object():
    earth = nw.load_image(os.path.join(REPO, "tests", "golden", "earthmap.jpeg"))
    final, _ = nw.preset(8, image=earth, aspect=1.0)
    blur, _ = nw.preset(1, aspect=1.5)
    # final scene: 1005 spheres (1000 cluster + 5), 1 moving sphere, 1 xz rect
    # (light), 400 boxes, 2 media on sphere boundaries, 1 instance
    assert bench.nw_flop_per_segment(final.flat()) == 1005 * 18 + 30 + 6 + 400 * 36 + 2 * (2 * 18 + 4) + 15
    # motion blur: 105 static spheres, 383 moving spheres
    assert bench.nw_flop_per_segment(blur.flat()) == 105 * 18 + 383 * 30


def test_flop_kinds_cover_the_object_kinds():
    # every non-medium kind of rtmi_nw_types.h ObjKind has a cost
    assert sorted(bench.NW_FLOP) == [0, 1, 2, 3, 4, 5]
    assert all(v > 0 for v in bench.NW_FLOP.values())


def test_auto_tile_w_rule():
    """The automatic tile shape (rtmi_device.hip auto_tile_w, mirrored by
    rt.auto_tile_w for reporting): 8x8 unless 16x4 leaves fewer idle lanes."""
    import a_dive_into_ray_tracing_amd as rt

    assert rt.auto_tile_w(1200, 800) == 8  # whole frame: both fill every tile
    assert rt.auto_tile_w(1200, 100) == 16  # 1/8 strip: 12.5 rows of 8x8 tiles, 25 of 16x4
    assert rt.auto_tile_w(1200, 400) == 8 and rt.auto_tile_w(1200, 200) == 8
    assert rt.auto_tile_w(3840, 270) == 8  # 1/8 of 2160 rows: 270 = 4 * 67 + 2, no shape fills it
    assert rt.auto_tile_w(1204, 8) == 8  # columns: 8 wastes 4 per row of tiles, 16 wastes 12
    assert rt.auto_tile_w(29, 19) in (8, 16)


def test_launch_command_starts_n_ranks_of_this_script():
    cmd = bench.launch_command(8, ["--gpus", "8", "--steps", "3"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-port=29555" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_gpus_beyond_visible_fails_loudly():
    """`bench.py --gpus 2` on a box with fewer GPUs must refuse (exit 2),
    never report a 1-GPU run as 2 (this container has no GPU)."""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "RTMI_DIST_BACKEND")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 2, (p.returncode, p.stderr[-500:])
    assert "2 GPUs asked" in p.stderr and p.stdout.strip() == ""


def test_world_size_mismatch_fails_loudly():
    import subprocess

    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0 and "launcher started 4 ranks" in p.stderr


def test_socket_cpus_prefers_socket0_one_per_core():
    # 2 sockets x 4 cores x 2 threads: cpu c -> core c % 8, socket (c % 8) // 4
    topo = {c: ((c % 8) // 4, c % 8) for c in range(16)}
    assert bench.socket_cpus(topo, set(range(16))) == [0, 1, 2, 3, 8, 9, 10, 11]
    # only socket-1 CPUs allowed: that socket
    assert bench.socket_cpus(topo, {4, 5, 12}) == [4, 5, 12]
    assert bench.socket_cpus({}, {3, 1}) == [1, 3]


def test_executed_flop_counts_nodes_leaves_and_big_spheres():
    c = {"segments": 10, "node_visits": 100, "leaf_sphere_tests": 30, "big_spheres": 4}
    assert bench.executed_flop(c) == 100 * 25 + (30 + 40) * 18
    assert bench.executed_flop(c, "grid") == 10 * 25 + 100 * 5 + (30 + 40) * 18


def test_busy_ms_per_launch_unions_overlapping_launches():
    """roofline.kernel_ms under --pipeline 2: launches on two streams overlap;
    the per-launch GPU time is the union of their intervals / count."""

    class Ev:
        def __init__(self, t):
            self.t = t

        def elapsed_time(self, other):
            return other.t - self.t

    pairs = lambda iv: [(Ev(a), Ev(b)) for a, b in iv]  # noqa: E731
    assert bench.busy_ms_per_launch(pairs([(0, 10), (10, 20), (20, 30)])) == 10
    assert bench.busy_ms_per_launch(pairs([(0, 20), (1, 21), (20, 40), (21, 41)])) == 41 / 4
    assert bench.busy_ms_per_launch(pairs([(5, 6), (0, 2)])) == 1.5  # a gap is not counted; any order


LIB = os.path.join(REPO, "a_dive_into_ray_tracing_amd", "lib", "librtmi.so")


def test_timed_kernel_symbol_names_the_instantiation():
    frame = {"tile_w": 8, "items_per_tile": 4, "tail_items_per_tile": 0, "persistent": 0, "bvh": 2}
    assert bench.timed_kernel_symbol(frame, flat=True) == "render_kernelILi8ELb1ELi3E"
    assert bench.timed_kernel_symbol(frame, flat=False) == "render_kernelILi8ELb1ELi2E"
    assert bench.timed_kernel_symbol(dict(frame, items_per_tile=1), flat=True) == "render_kernelILi8ELb0ELi3E"
    assert bench.timed_kernel_symbol(dict(frame, persistent=3, tile_w=16), flat=True) == "render_residentILi16ELi3E"
    assert bench.timed_kernel_symbol(dict(frame, bvh=4), flat=True) == "render_kernelILi8ELb1ELi5E"
    assert bench.timed_kernel_symbol(dict(frame, persistent=2), flat=True) is None
    assert bench.timed_kernel_symbol(None, flat=True) is None


@pytest.mark.skipif(not os.path.exists(LIB), reason="needs the built library")
def test_pmc_records_are_quoted_only_for_the_kernel_they_measured():
    """roofline.traffic / roofline.pmc come from committed
    PMC records; bench.py quotes them only while the timed kernel's gfx950
    code hashes as the record says, and reports why otherwise."""
    import json

    from a_dive_into_ray_tracing_amd import codeobj

    sym = "render_kernelILi8ELb1ELi3E"
    full, h = codeobj.kernel_sha1(LIB, sym)
    assert full and sym in full and len(h) == 40
    rec = {"symbol": sym, "code_sha1": h, "hbm_bytes_per_launch": 1}
    assert bench.pmc_guard(rec, LIB, sym) == (rec, None)
    # a perturbed hash (the kernel was rebuilt since the record): not quoted
    got, why = bench.pmc_guard(dict(rec, code_sha1="0" * 40), LIB, sym)
    assert got is None and "changed" in why
    # another kernel timed: not quoted
    got, why = bench.pmc_guard(rec, LIB, "render_residentILi8ELi3E")
    assert got is None and "render_residentILi8ELi3E" in why
    # no hash at all: not quoted
    got, why = bench.pmc_guard({"hbm_bytes_per_launch": 1}, LIB, sym)
    assert got is None and "no kernel code hash" in why
    # the committed records name a kernel of this library by its current code
    for path, key in (("pmc_valu.json", None), ("pmc_traffic.json", "grid")):
        d = json.load(open(os.path.join(REPO, "profiles", path)))
        d = d[key] if key else d
        assert codeobj.kernel_sha1(LIB, d["symbol"])[1] is not None
