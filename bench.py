#!/usr/bin/env python3
"""bench.py — Msamples/s on the RTIOW final scene (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One step = one full render of the config-2 workload: the final random-spheres
scene (487 spheres, glibc seed 1 as the reference), 1200x800, 500 spp, depth
50.  At N > 1 the image is split over ranks by interleaved rows (row j -> rank
j % N), each rank renders its strip on its own GPU, and the strips are
gathered to rank 0 with ONE RCCL gather (torch.distributed "nccl" = RCCL)
inside the timed region.  Total work is fixed as N grows: scaling "strong".
value = W*H*spp*K / max-over-ranks(wall time of K steps) / 1e6.
Steps alternate over render contexts, each on a HIP stream with a hardware
queue of its own (--pipeline; 2 by default, 3 at N > 1): step k+1's render is
independent of step k's, so its first blocks fill the CUs that step k's last
blocks leave idle (the end-of-dispatch drain).  At N > 1 each
step's gather runs on its context's stream right after the render, over a
process group of that context's own.  Every step still renders the whole
workload; --pipeline 1 runs them one after another on one context.
RTMI_DIST_FORCE=1 under a launcher runs the N > 1 path at world size 1 (a
one-rank RCCL rehearsal).
`--gpus N` without a launcher environment starts the N ranks itself (a
torch.distributed.run child of a parent that never touches the GPU) and
refuses to run when fewer than N GPUs are visible.  After the timed region
rank 0 renders the whole frame alone and checks the gathered image against
it bit for bit ("gather_check").

Closest hits go through the uniform grid by default (--accel grid; --accel
bvh the BVH): the same closest hit as the brute-force loop, bit for bit
(tests/test_gpu_parity.py), so the same image.  --accel none times the
brute-force kernel.

roofline (FP32 VALU): `achieved` = the EXECUTED algorithmic FLOP
of the timed kernel's launch / its mean duration (HIP events on the launch
stream).  With the grid or BVH the executed work is counted exactly by the
RTMI_STATS build of the same kernel (librtmi_stats.so, one extra untimed
render of the same rows in a child process; same paths, same image):
every lane's sphere miss tests (cell / leaf spheres and the brute-force big
spheres) x 18 FLOP (sphere.h:21-55) plus, for the grid, one
grid-box slab test per segment x 25 (6 FMA + 12 min/max + 1 compare) and its
DDA cell steps x 5, for the BVH its node slab tests x 25.  Brute force
executes segments x N x 18.
peak = 157.3 TFLOP/s FP32 vector.  `work_equivalent_*` keeps SURVEY §8(d)'s
brute-force-equivalent figure (segments x 487 x 18 over the BVH time, which
can exceed 1) and `brute_force_*` the brute-force kernel's own roofline from
one more untimed launch of the same rows.
cpu_baseline (BASELINE.md §4, rank 0, N = 1): host facts (CPU model, sockets,
cores per socket, the CPU share this job may load), every run pinned with
taskset to one physical core per thread on one socket: (ii) the reference's
worker() at -O2 with threads = the CPU share (the reported value), (i) the as-shipped -O0 build with
the reference's 16 threads, (iii) this build's C restatement (fast mode,
OpenMP) at -O3 -march=native — each on a bounded sample.

--workload config4 / config5 time BASELINE's other final-scene configs
(1200x800 at 5000 spp; 3840x2160 at 2000 spp).  It also selects the
Next-Week lines (not the headline): nw_motion_blur = the
Next-Week random scene with moving spheres at 1200x800x500 (the reference's
only published Next-Week number, rt_next_week/cuda/README.md:167-174: 37.88 s),
nw_final = the Next-Week final scene at 800x800 (main.cu:517-524; --nw-spp,
default 1024).  Same row partition and gather as the headline.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

W, H, SPP, DEPTH, SEED = 1200, 800, 500, 50, 1984
FLOP_PER_SPHERE_TEST = 18  # oc 3, hb 5, |oc|^2-r^2 7, disc 3
FLOP_PER_NODE_TEST = 25  # slab test as executed: 6 FMA (12) + 12 min/max + 1 compare
FLOP_PER_CELL_STEP = 5  # grid DDA step: min of 3 face parameters (2) + compare (1) + the next face's fma (2)
PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 vector (MI355X_MICROARCH.md)
PUBLISHED_CPU_MSPS = 0.1189  # README.md:16-19: rt_in_one_weekend, 1200x800x500, 16 threads, 4036.1 s
METRIC = "Msamples/sec (pixels x spp) on RTIOW final scene"
# BASELINE.json configs on the final scene: config2 = the headline (1 GPU,
# 1200x800x500); config4 = the same at 5000 spp; config5 = 3840x2160 (16:9
# camera) at 2000 spp (quoted for 8 GPUs; the final scene has the
# reference's defocus blur, aperture 0.1).
RTIOW_WORKLOADS = {"config2": (1200, 800, 500), "config4": (1200, 800, 5000), "config5": (3840, 2160, 2000)}
STATS_LIB = os.path.join(REPO, "a_dive_into_ray_tracing_amd", "lib", "librtmi_stats.so")


# ----------------------------------------------------------------- launch ----
def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(gpus, argv, port):
    """The torch.distributed.run command that starts `gpus` ranks of this
    script with the same arguments (one process per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def visible_gpus():
    """GPUs this process could use, counted without initialising the GPU
    (torch.cuda.device_count() does not create a context on this image)."""
    import torch

    return torch.cuda.device_count()


def launch(args, argv):
    """--gpus N > 1 without a launcher environment: check that N GPUs are
    visible, then run N ranks as a torch.distributed.run child and exit with
    its status.  This process never touches the GPU (no exec after GPU init)."""
    backend = os.environ.get("RTMI_DIST_BACKEND", "nccl")
    n = 0 if STUB else visible_gpus()
    if backend == "nccl" and n < args.gpus:
        print(f"bench: {args.gpus} GPUs asked, {n} visible — refusing to report a {n}-GPU run as {args.gpus}",
              file=sys.stderr, flush=True)
        return 2
    cmd = launch_command(args.gpus, argv, free_port())
    print(f"bench: launching {args.gpus} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


# Collective timeout (s) of the process group: a rank that stalls (a hung
# first RCCL gather, a dead peer) ends the run within this bound instead of
# torch's default 10 minutes.  It covers rank 0's untimed side renders while
# the other ranks wait at a barrier (the whole-frame gather check: 0.7 s at
# config 5 on one GPU) and RCCL's communicator set-up in the first collective.
# RTMI_DIST_TIMEOUT_S overrides it (tests use a few seconds).
DIST_TIMEOUT_S = float(os.environ.get("RTMI_DIST_TIMEOUT_S", "60"))


class CollectiveError(RuntimeError):
    """A collective of the process group failed or timed out on this rank."""


def collective(name, fn, *a, **kw):
    """Run one torch.distributed call; a failure (gloo: a timeout raises here;
    RCCL: torch's watchdog aborts the process and names the work itself)
    becomes a CollectiveError naming the collective."""
    try:
        return fn(*a, **kw)
    except Exception as e:
        raise CollectiveError(f"{name}: {type(e).__name__}: {str(e).splitlines()[0] if str(e) else ''}") from e


class stdout_to_stderr:
    """The process's fd 1 pointed at fd 2 meanwhile: a backend's own start-up
    chatter (gloo prints its peer connections to stdout from C++) must not
    reach stdout, which carries only the JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def init_group(dist, backend, **kw):
    """init_process_group with stdout quiet (stdout_to_stderr); every
    collective of the group times out after DIST_TIMEOUT_S."""
    from datetime import timedelta

    with stdout_to_stderr():
        collective("init_process_group", dist.init_process_group, backend,
                   timeout=timedelta(seconds=DIST_TIMEOUT_S), **kw)


def dist_setup(torch, dist):
    """One process per GPU (torch.distributed.run env).  RCCL ("nccl") is the
    product path.  RTMI_DIST_BACKEND=gloo is a rehearsal mode for a box with
    fewer GPUs than ranks: ranks share devices (local_rank % device count) and
    the collectives run on host copies; the timed region then includes those
    copies, so it is never a reported number."""
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("RTMI_DIST_BACKEND", "nccl")
    if STUB:  # CPU rehearsal: no device at all
        if backend != "gloo":
            raise SystemExit("bench: RTMI_BENCH_STUB=1 needs RTMI_DIST_BACKEND=gloo")
        if world_size > 1 or FORCE_DIST:
            init_group(dist, "gloo")
        cpu = torch.device("cpu")
        return world_size, rank, -1, cpu, cpu
    ndev = torch.cuda.device_count()
    if backend == "nccl" and local_rank >= ndev:
        raise SystemExit(f"bench: rank {rank} needs GPU {local_rank}, {ndev} visible")
    device = local_rank % max(1, ndev) if backend == "gloo" else local_rank
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    if world_size > 1 or FORCE_DIST:
        if backend == "gloo":
            init_group(dist, "gloo")
        else:
            init_group(dist, "nccl", device_id=dev)
    coll = dev if backend == "nccl" else torch.device("cpu")
    return world_size, rank, device, dev, coll


# ------------------------------------------------- CPU rehearsal (stub) ----
# RTMI_BENCH_STUB=1 (with RTMI_DIST_BACKEND=gloo): the whole launch / rank
# setup / timed loop / gather / gather-check / line assembly path on the CPU,
# with a stand-in renderer that writes each pixel's image coordinates.  Used
# by tests/test_bench_dist.py to rehearse N > 1 where no GPU exists; the line
# it prints is marked "stub" and is never a measurement.
STUB = os.environ.get("RTMI_BENCH_STUB") == "1"
# tests/test_bench_dist.py only (stub runs): rank RTMI_BENCH_STALL_RANK sleeps
# RTMI_BENCH_STALL_S seconds before each gather, past the collective timeout
# RTMI_DIST_FORCE=1 under a launcher (WORLD_SIZE set): the process group and
# every collective of the N > 1 path run at world size 1 too (a one-rank
# RCCL rehearsal of the exact calls the N-GPU run makes on one GPU; RCCL
# refuses two ranks on one device).  The line says so (config.dist_rehearsal).
FORCE_DIST = os.environ.get("RTMI_DIST_FORCE") == "1" and "WORLD_SIZE" in os.environ
# Where a timed step's gather runs (RTMI_BENCH_GATHER=inline|side).
# "inline" (the default) issues it as a synchronous collective, which this
# torch runs on the caller's current stream — the render's own stream and
# hardware queue, right after the render — over a process group of that
# context's own: one communicator per stream (NCCL forbids one communicator's
# collectives on two streams, whose kernels could then run out of issue
# order).  "side" issues it as an async collective of the default group on
# torch's NCCL stream, joined by a stream wait before its buffer is rendered
# into again: the cross-stream waits between a context's renders cost the
# overlap of consecutive launches.  One-rank RCCL run
# (profiles/r06/rccl_one_rank/ab_gather_mode2.txt): one rank's 1/8 strip 2.60-2.62
# (inline) vs 2.69 (side) vs 2.54-2.55 ms without gathers; the frame 19.00-19.01 vs
# 19.08-19.12 vs 18.98-18.99.
GATHER_INLINE = os.environ.get("RTMI_BENCH_GATHER", "inline") == "inline"
DIST_REHEARSAL = ("RTMI_DIST_FORCE: one rank through every collective of the N > 1 path (gathers, barriers, max "
                  "over ranks, gather check, one-shot)")
STALL_RANK = int(os.environ.get("RTMI_BENCH_STALL_RANK", "-1")) if STUB else -1
STALL_S = float(os.environ.get("RTMI_BENCH_STALL_S", "0"))


class StubRenderer:
    """Stand-in for rt.Renderer (CPU): pixel (i, j) channel c of the strip =
    (j * W + i) * 3 + c, so the value depends only on the image coordinates
    (partition-invariant, like the product's RNG keys)."""

    def __init__(self):
        self._segs = 0

    def render_rows(self, cam, W_, H_, S, D, seed, row0, row_step, nrows, buf):
        import torch

        j = row0 + row_step * np.arange(nrows)
        v = (j[:, None] * W_ + np.arange(W_)[None, :])[:, :, None] * 3 + np.arange(3)[None, None, :]
        buf.copy_(torch.from_numpy(np.where((j < H_)[:, None, None], v, 0).astype(np.float32)))
        self._segs = int((j < H_).sum()) * W_ * S

    def last_segments(self):
        return self._segs

    def __getattr__(self, name):  # set_schedule / set_kernel / set_accel / set_ordering / close
        if name.startswith("set_") or name == "close":
            return lambda *a, **k: None
        raise AttributeError(name)


def hw_queue_streams(torch, dev, n):
    """n HIP streams, each on a hardware queue of its own: created with
    hipExtStreamCreateWithCUMask and every CU enabled (the runtime gives a
    CU-masked stream its own queue; plain streams created after torch's stream
    pool share queues, and two streams on one queue run their kernels one after
    another, measured in profiles/r05/pipeline/).  Returns (torch streams,
    destroy function)."""
    import ctypes as C

    # the HIP runtime this process already uses (torch's), not a second copy
    with open("/proc/self/maps") as f:
        path = next((ln.split()[-1] for ln in f if "libamdhip64" in ln), "libamdhip64.so")
    hip = C.CDLL(path)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = [0] * ((ncu + 31) // 32)
    for c in range(ncu):
        words[c // 32] |= 1 << (c % 32)
    mask = (C.c_uint32 * len(words))(*words)
    raw = []
    for _ in range(n):
        h = C.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(C.byref(h), C.c_uint32(len(words)), mask)
        if rc != 0:
            break
        raw.append(h.value)

    def destroy():
        torch.cuda.synchronize(dev)
        # torch's current stream is one of these (an ExternalStream): point it
        # back at the default stream before the handles are freed
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
        for x in raw:
            hip.hipStreamDestroy(C.c_void_p(x))

    if len(raw) < n:  # the same steps on plain streams (correct; they may share a queue and not overlap)
        print(f"bench: hipExtStreamCreateWithCUMask failed ({rc}): plain streams instead", file=sys.stderr, flush=True)
        destroy()
        return [torch.cuda.Stream(dev) for _ in range(n)], None
    return [torch.cuda.ExternalStream(x, device=dev) for x in raw], destroy


def busy_ms_per_launch(events):
    """Mean GPU time per launch over (start, end) event pairs that may
    overlap (launches on two streams): the union of their intervals / count."""
    base = events[0][0]
    iv = sorted((base.elapsed_time(a), base.elapsed_time(b)) for a, b in events)
    total, cur_s, cur_e = 0.0, iv[0][0], iv[0][1]
    for a, b in iv[1:]:
        if a > cur_e:
            total += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    return (total + cur_e - cur_s) / len(events)


class StubEvent:
    """torch.cuda.Event stand-in (host clock)."""

    def __init__(self, **_):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


# ------------------------------------------------------- executed work ----
def executed_counts_child(argv):
    """--exec-counts child (RTMI_LIBRARY = the RTMI_STATS build): render the
    given rows once and print the exact per-lane work counters as JSON."""
    import ctypes as C

    import torch

    import a_dive_into_ray_tracing_amd as rt

    Wc, Hc, S, row0, row_step, nrows = (int(x) for x in argv[:6])
    accel = argv[6]
    kernel = argv[7] if len(argv) > 7 else "auto"
    L = rt.load()
    L.rt_ctx_debug_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    L.rt_ctx_debug_counters.restype = C.c_int
    world = rt.random_scene()
    r = rt.Renderer(world, 0)
    r.set_accel(accel)
    r.set_kernel(kernel)
    strip = torch.empty((nrows, Wc, 3), dtype=torch.float32, device="cuda:0")
    r.render_rows(rt.final_camera(Wc / Hc), Wc, Hc, S, DEPTH, SEED, row0, row_step, nrows, strip.data_ptr(), 0)
    r.synchronize()
    v = (C.c_uint64 * 8)()
    rt.check(L.rt_ctx_debug_counters(r._h, v), "rt_ctx_debug_counters")
    nbig, nnodes = r.accel_info()
    print(json.dumps({"segments": v[0], "node_visits": v[5], "leaf_sphere_tests": v[6], "node_iterations_wave": v[1],
                      "leaf_sphere_iterations_wave": v[2], "root_resolutions_wave": v[4],
                      "wave_passes": v[7] & ((1 << 63) - 1), "big_spheres": nbig,
                      "bvh_nodes": nnodes, "checksum": float(strip.double().sum().item())}), flush=True)
    r.close()


def executed_counts(Wc, Hc, S, row0, row_step, nrows, accel="bvh", kernel="auto"):
    """Run the RTMI_STATS build on the same rows (same kernel) in a child process."""
    if not os.path.exists(STATS_LIB):
        return None, f"{STATS_LIB} not built"
    env = dict(os.environ, RTMI_LIBRARY=STATS_LIB)
    try:
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--exec-counts", str(Wc), str(Hc), str(S),
                              str(row0), str(row_step), str(nrows), accel, kernel],
                             capture_output=True, text=True, timeout=240, env=env, check=True).stdout
        return json.loads(out.strip().splitlines()[-1]), None
    except Exception as e:  # reported, never replaced by another figure
        return None, f"stats child failed: {e}"


def executed_flop(c, accel="bvh"):
    """Executed algorithmic FLOP of one BVH / grid launch from the stats
    counters ("node_visits" / "leaf_sphere_tests" count grid cells / cell
    sphere tests for the grid, whose every segment also clips the ray to the
    grid box: one slab test)."""
    spheres = (c["leaf_sphere_tests"] + c["segments"] * c["big_spheres"]) * FLOP_PER_SPHERE_TEST
    if accel == "grid":
        return c["segments"] * FLOP_PER_NODE_TEST + c["node_visits"] * FLOP_PER_CELL_STEP + spheres
    return c["node_visits"] * FLOP_PER_NODE_TEST + spheres


# ------------------------------------------------ committed PMC records ----
def timed_kernel_symbol(sched, flat):
    """Mangled-name fragment of the render kernel a launch ran, from its
    schedule (Renderer.last_schedule) and whether the grid is one y layer."""
    if not sched:
        return None
    tw, kind, acc = sched["tile_w"], sched["persistent"], sched["bvh"]
    a = {2: 3 if flat else 2, 4: 5 if flat else 4}.get(acc, acc)  # (last_schedule folds the one-layer kinds)
    if kind == 3:
        return f"render_residentILi{tw}ELi{a}E"
    if kind == 0:
        chunked = int(sched["items_per_tile"] + sched["tail_items_per_tile"] > 1)
        return f"render_kernelILi{tw}ELb{chunked}ELi{a}E"
    return None  # (the persistent kernel: no committed record)


def pmc_guard(record, lib_path, symbol):
    """(record, None) when a committed PMC record (profiles/pmc_*.json) was
    measured on the very kernel code this run timed — its "symbol" is the
    timed kernel and its "code_sha1" the sha1 of that kernel's gfx950 code in
    the loaded library — else (None, why).  A rebuilt kernel, another kernel
    shape or a record without a hash is never quoted."""
    from a_dive_into_ray_tracing_amd import codeobj

    if not record or "code_sha1" not in record or "symbol" not in record:
        return None, "record carries no kernel code hash"
    if symbol != record["symbol"]:
        return None, f"record measured on {record['symbol']}, this run timed {symbol}"
    try:
        _, h = codeobj.kernel_sha1(lib_path, symbol)
    except Exception as e:  # (an unreadable library: not quoted)
        return None, f"kernel code not readable: {e}"
    if h != record["code_sha1"]:
        return None, f"kernel code changed since the record (sha1 {h} vs {record['code_sha1']})"
    return record, None


# ------------------------------------------------------------ CPU baseline ----
def host_topology():
    """(facts, {cpu: (socket, core)}) from lscpu, for the CPUs of this machine."""
    facts = {"nproc": len(os.sched_getaffinity(0)), "machine_cpus": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=30).stdout
        keys = {"Model name": "model", "Socket(s)": "sockets", "Core(s) per socket": "cores_per_socket",
                "Thread(s) per core": "threads_per_core"}
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in keys:
                v = v.strip()
                facts[keys[k.strip()]] = int(v) if v.isdigit() else v
        topo = {}
        out = subprocess.run(["lscpu", "-p=CPU,CORE,SOCKET"], capture_output=True, text=True, timeout=30).stdout
        for line in out.splitlines():
            if line and not line.startswith("#"):
                cpu, core, sock = (int(x) if x else 0 for x in line.split(","))
                topo[cpu] = (sock, core)
    except Exception:
        topo = {}
    return facts, topo


def socket_cpus(topo, allowed):
    """The allowed CPUs of one socket (socket 0 when it has any, else the
    socket with the most), one per physical core first, then SMT siblings."""
    if not topo:
        return sorted(allowed)
    by_sock = {}
    for c in allowed:
        by_sock.setdefault(topo.get(c, (0, c))[0], []).append(c)
    sock = 0 if 0 in by_sock else max(by_sock, key=lambda s: len(by_sock[s]))
    first, rest, seen = [], [], set()
    for c in sorted(by_sock[sock]):
        core = topo.get(c, (0, c))[1]
        (rest if core in seen else first).append(c)
        seen.add(core)
    return first + rest


def pinned(cmd, cpus):
    tp = "/usr/bin/taskset"
    return ([tp, "-c", ",".join(str(c) for c in cpus)] + cmd) if os.path.exists(tp) else cmd


def run_ref_harness(binary, threads, spp, cpus):
    out = subprocess.run(pinned([binary, "bench", str(threads), str(W), str(H), str(spp), str(DEPTH)], cpus),
                         capture_output=True, text=True, timeout=300, check=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def cpu_restatement_child(argv):
    """--cpu-restatement child: the oracle's fast-mode C restatement (OpenMP)
    on evenly spaced rows of the config-2 image; prints Msamples/s."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_py as O

    rows, spp = int(argv[0]), int(argv[1])
    sc, _ = O.final_scene()
    cam = O.final_camera(W / H)
    t0 = time.perf_counter()
    O.fast_render(sc, cam, W, H, spp, DEPTH, SEED, row0=0, row_step=H // rows, nrows=rows)
    dt = time.perf_counter() - t0
    print(json.dumps({"seconds": dt, "msamples_per_s": rows * W * spp / dt / 1e6, "lib": O.LIB_PATH}), flush=True)


def cpu_baseline():
    """BASELINE.md §4 rows (i)-(iii) on the host of rank 0, pinned to one
    socket's allowed CPUs.  Reported value: row (ii)."""
    facts, topo = host_topology()
    # the CPU share this job may load: OMP_NUM_THREADS where the pool sets it
    # (16 per GPU on the MI355X boxes), else every allowed CPU
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    cpus = socket_cpus(topo, os.sched_getaffinity(0))[:share]
    threads = len(cpus)
    facts["cpu_share"] = share
    facts["pinned_cpus"] = ",".join(str(c) for c in cpus)
    facts["pinned_physical_cores"] = len({topo.get(c, (0, c)) for c in cpus}) if topo else None
    facts["note"] = ("threads = this job's CPU share (OMP_NUM_THREADS), one per physical core of one socket, "
                     "pinned with taskset; cores_per_socket is the machine's")
    rows = {}
    ref = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    ref0 = os.path.join(REPO, "oracle", "_ref", "ref_harness_O0")
    try:  # (ii) the reference source at -O2, threads = the pinned CPUs
        spp = 2
        r = run_ref_harness(ref, threads, spp, cpus)
        rows["ii_reference_O2"] = {"value": round(r["msamples_per_s"], 5), "threads": threads,
                                   "sample": f"{W}x{H}x{spp}spp depth {DEPTH}", "seconds": round(r["seconds"], 2)}
    except Exception as e:
        rows["ii_reference_O2"] = {"error": str(e)[:200]}
    try:  # (i) as shipped: g++ -O0 (Makefile:7), the reference's 16 threads (main.cpp:318)
        spp = 1
        r = run_ref_harness(ref0, 16, spp, cpus)
        rows["i_as_shipped_O0"] = {"value": round(r["msamples_per_s"], 5), "threads": 16,
                                   "sample": f"{W}x{H}x{spp}spp depth {DEPTH}", "seconds": round(r["seconds"], 2)}
    except Exception as e:
        rows["i_as_shipped_O0"] = {"error": str(e)[:200]}
    try:  # (iii) this build's CPU restatement, -O3 -march=native, built here
        import tempfile

        # built on the host it is timed on (never a copy built elsewhere)
        native = os.path.join(tempfile.mkdtemp(prefix="rtmi_oracle_"), "liboracle_native.so")
        subprocess.run(["make", "-B", "-C", os.path.join(REPO, "oracle"), "native", f"NATIVE_SO={native}"],
                       capture_output=True, timeout=120, check=True)
        env = dict(os.environ, ORACLE_LIBRARY=native, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="true")
        nrows, spp = 100, 96
        out = subprocess.run(pinned([sys.executable, os.path.abspath(__file__), "--cpu-restatement", str(nrows), str(spp)], cpus),
                             capture_output=True, text=True, timeout=300, env=env, check=True).stdout
        r = json.loads(out.strip().splitlines()[-1])
        rows["iii_restatement_O3_native"] = {"value": round(r["msamples_per_s"], 5), "threads": threads,
                                             "sample": f"{nrows} evenly spaced rows x {W} x {spp}spp depth {DEPTH}",
                                             "seconds": round(r["seconds"], 2)}
    except Exception as e:
        rows["iii_restatement_O3_native"] = {"error": str(e)[:200]}
    # the share of one socket these rows use (north_star: "single-socket CPU
    # reference"): row (ii) is bound by the reference's global rand() lock
    # (128 threads on a full socket measured 0.052 Msamples/s,
    # DESIGN.md §5), row (iii) scales with cores
    cps = facts.get("cores_per_socket")
    if isinstance(cps, int) and cps > 0:
        facts["socket_share"] = round(threads / cps, 4)
        r3 = rows.get("iii_restatement_O3_native", {})
        if "value" in r3 and threads < cps:
            r3["full_socket_linear_estimate"] = round(r3["value"] * cps / threads, 3)
            r3["note"] = (f"{threads} of {cps} cores of one socket: a full socket would give up to ~{cps / threads:.0f}x "
                          "this (linear estimate, not measured: the pool's CPU share per GPU job is "
                          f"{threads} threads)")
    main_row = rows["ii_reference_O2"]
    if "value" not in main_row:
        return {"value": None, "unit": "Msamples/s", "cores": threads, "kind": "reference", "host": facts, "rows": rows}
    return {"value": main_row["value"], "unit": "Msamples/s", "cores": threads, "kind": "reference",
            "sample": f"reference worker() g++ -O2 (oracle/_ref/ref_harness), {threads} std::threads pinned to "
                      f"{threads} physical cores of one socket (of {cps if cps else '?'}; the job's CPU share), final "
                      f"scene {main_row['sample']} ({main_row['seconds']} s wall); bound by the reference's global "
                      "rand() lock, so more cores do not raise it",
            "host": facts, "rows": rows}


# -------------------------------------------------------------------- main ----
def nw_executed_counts_child(argv):
    """--nw-exec-counts child (RTMI_LIBRARY = the RTMI_STATS build): render the
    given Next-Week rows once and print the executed-work counters."""
    import ctypes as C

    import torch

    import a_dive_into_ray_tracing_amd as rt
    import a_dive_into_ray_tracing_amd.nextweek as nw

    which, Wn, Hn, spp, row0, row_step, nrows = (int(x) for x in argv[:7])
    accel = argv[7]
    earth = nw.load_image(os.path.join(REPO, "tests", "golden", "earthmap.jpeg")) if which != 1 else None
    scene, cam = nw.preset(which, image=earth, aspect=Wn / Hn)
    r = nw.NwRenderer(scene, 0)
    r.set_accel(accel)
    L = rt.load()
    v = (C.c_uint64 * 4)()
    rt.check(L.rt_nw_debug_counters(v), "rt_nw_debug_counters")  # zero them
    strip = torch.empty((nrows, Wn, 3), dtype=torch.float32, device="cuda:0")
    r.render_rows(cam, Wn, Hn, spp, DEPTH, SEED, row0, row_step, nrows, strip.data_ptr(), 0)
    segs = r.last_segments()
    rt.check(L.rt_nw_debug_counters(v), "rt_nw_debug_counters")
    print(json.dumps({"segments": segs, "flop": v[0], "node_visits": v[1], "object_tests": v[2], "cell_steps": v[3]}),
          flush=True)
    r.close()


def nw_executed_counts(which, Wn, Hn, spp, row0, row_step, nrows, accel):
    if not os.path.exists(STATS_LIB):
        return None, f"{STATS_LIB} not built"
    env = dict(os.environ, RTMI_LIBRARY=STATS_LIB)
    try:
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--nw-exec-counts", str(which), str(Wn), str(Hn),
                              str(spp), str(row0), str(row_step), str(nrows), accel],
                             capture_output=True, text=True, timeout=600, env=env, check=True).stdout
        return json.loads(out.strip().splitlines()[-1]), None
    except Exception as e:  # reported, never replaced by another figure
        return None, f"stats child failed: {e}"


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--exec-counts":
        return executed_counts_child(sys.argv[2:])
    if len(sys.argv) > 1 and sys.argv[1] == "--nw-exec-counts":
        return nw_executed_counts_child(sys.argv[2:])
    if len(sys.argv) > 1 and sys.argv[1] == "--cpu-restatement":
        return cpu_restatement_child(sys.argv[2:])
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tile-w", type=int, default=0, help="0 = automatic (the library default)")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--tail-spp", type=int, default=-1)
    ap.add_argument("--tail-chunk", type=int, default=0)
    ap.add_argument("--kernel", choices=["auto", "persistent", "grid", "queue", "resident"], default="auto")
    ap.add_argument("--accel", choices=["none", "bvh", "grid"], default="grid",
                    help="closest-hit search: grid (default: uniform grid + DDA), bvh or brute force; same image bit for bit")
    ap.add_argument("--ordering", choices=["cost", "none"], default="cost")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exec-counts", action="store_true", help="skip the RTMI_STATS work count (roofline.frac null)")
    ap.add_argument("--timed-only", action="store_true",
                    help="no untimed side launches (one-shot, brute force, gather check): for profiler runs whose "
                         "kernel averages must cover only the warmup + timed launches")
    ap.add_argument("--workload", choices=list(RTIOW_WORKLOADS) + ["nw_motion_blur", "nw_final"], default="config2")
    ap.add_argument("--nw-spp", type=int, default=0, help="spp of the nw_* workloads (default: 500 / 1024)")
    ap.add_argument("--nw-preset", type=int, default=0,
                    help="analysis only: render create_world case 1..8 at the nw_* workload's size instead")
    ap.add_argument("--nw-accel", choices=["auto", "bvh", "grid"], default="auto",
                    help="closest-hit structure of the nw_* workloads (rt_nw_ctx_set_accel; same image)")
    ap.add_argument("--pipeline", type=int, choices=[1, 2, 3], default=0,
                    help="render contexts the steps alternate over, each on its own hardware queue (2: consecutive "
                         "steps' renders may overlap; 1: one context, one stream).  Default: 2, or 3 when the steps "
                         "gather (N > 1): a context's gather then sits between its renders, and a third context "
                         "keeps two renders in flight meanwhile (one-rank RCCL run, 1/8 strip 2.60 -> 2.57 ms; "
                         "profiles/r06/rccl_one_rank/ab_pipeline3.txt)")
    ap.add_argument("--strip-of", type=int, default=0,
                    help="analysis only: time ONE rank's interleaved strip of an N-GPU run on this GPU")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args, sys.argv[1:]))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws != args.gpus:
        sys.exit(f"bench: --gpus {args.gpus} but the launcher started {ws} ranks")
    if args.workload.startswith("nw_"):
        return bench_nw(args)
    W, H, SPP = RTIOW_WORKLOADS[args.workload]

    import torch
    import torch.distributed as dist

    import a_dive_into_ray_tracing_amd as rt
    from a_dive_into_ray_tracing_amd import dist as rdist

    world_size, rank, local_rank, dev, coll = dist_setup(torch, dist)
    from datetime import timedelta
    N = world_size
    DIST = N > 1 or FORCE_DIST  # the N > 1 path: process group, gathers, barriers, max over ranks
    if not args.pipeline:
        args.pipeline = 3 if DIST else 2
    # inline gathers: one process group (communicator) per context, created
    # in the same order on every rank
    ctx_groups = [None] * args.pipeline
    if DIST and GATHER_INLINE:
        with stdout_to_stderr():
            ctx_groups = [collective(f"new_group for context {c}", dist.new_group, list(range(N)),
                                     timeout=timedelta(seconds=DIST_TIMEOUT_S)) for c in range(args.pipeline)]

    world = rt.random_scene()
    cam = rt.final_camera(W / H)
    npipe = args.pipeline  # (the stub rehearses the same alternation over two stand-in contexts)

    def make_renderer():
        x = StubRenderer() if STUB else rt.Renderer(world, local_rank, tile_w=args.tile_w, chunk=args.chunk)
        x.set_schedule(args.chunk, args.tail_spp, args.tail_chunk)
        x.set_kernel(args.kernel)
        x.set_accel(args.accel)
        x.set_ordering(args.ordering)
        # the launches of the two contexts overlap: fewer, longer items
        # (rt_ctx_set_overlap) — from 8 timed steps up; in shorter runs the
        # last launch's longer drain is shared by too few steps (1/8 strip at
        # K = 5: 2.81 vs 2.74 ms; K = 10: 2.65 vs 2.70; profiles/r05/pipeline/ab_items_short.txt)
        if npipe > 1 and args.steps >= 8:
            x.set_overlap(True)
        return x

    rs = [make_renderer() for _ in range(npipe)]  # the steps' render contexts (step k: rs[k % npipe])
    r = rs[0]  # the context of the side launches below
    row0, row_step, nrows = rdist.strip_rows(H, rank, N)  # interleaved rows, row j -> rank j % N
    if args.strip_of > 1 and N == 1:  # analysis mode: one rank's share of an N-GPU render
        row0, row_step, nrows = rdist.strip_rows(H, 0, args.strip_of)
    nrows_valid = len(range(row0, H, row_step))  # rows of this strip inside the image
    strip = torch.empty((nrows, W, 3), dtype=torch.float32, device=dev)
    # Strip buffers: one per context, two per context with gathers (N > 1).
    # Buffer b is always rendered by context b % npipe on its stream, and
    # rendered into again only after its previous gather is done; with two
    # per context a render waits for the gather of the step npipe * 2 back,
    # not of the step before on its stream, so a gather that waits for
    # CU slots (or for a slower rank) does not hold up the next render of
    # its context (one-rank RCCL rehearsal: frame 19.26 -> 19.09 ms per step,
    # the 1/8 strip unchanged at 2.66; RTMI_BENCH_STRIP_BUFS overrides the
    # count for that A/B).
    nbuf = int(os.environ.get("RTMI_BENCH_STRIP_BUFS", "0")) or (2 * npipe if DIST else npipe)
    if nbuf % npipe:
        sys.exit(f"bench: RTMI_BENCH_STRIP_BUFS={nbuf} is not a multiple of --pipeline {npipe}")
    strips = [strip] + [torch.empty_like(strip) for _ in range(nbuf - 1)]
    tw = args.tile_w or rt.auto_tile_w(W, -(-(H - row0) // row_step) if row0 < H else 0)  # reported tile shape
    gathered = None
    destroy_streams = None
    if STUB:
        streams, Event = [None] * npipe, StubEvent

        def sync():
            pass

        def render_into(rows, buf, c=0):
            rs[c].render_rows(cam, W, H, SPP, DEPTH, SEED, *rows, buf)
    else:
        # non-default streams, one per context: each context's kernels, the
        # HIP events around them and the RCCL gather of its strip are ordered
        # on its stream (the null stream would bypass the events)
        streams, destroy_streams = hw_queue_streams(torch, dev, npipe)
        Event = torch.cuda.Event
        torch.cuda.set_stream(streams[0])

        def sync():
            torch.cuda.synchronize(dev)

        def render_into(rows, buf, c=0):
            rs[c].render_rows(cam, W, H, SPP, DEPTH, SEED, *rows, buf.data_ptr(), streams[c].cuda_stream)

    stream = streams[0]  # the side launches' stream (context 0)
    ev, gev = [], []

    def timed_render(rows=(row0, row_step, nrows), buf=strip, c=0):
        e0, e1 = Event(enable_timing=True), Event(enable_timing=True)
        e0.record(streams[c])
        render_into(rows, buf, c)
        e1.record(streams[c])
        return e0, e1

    pend = {}  # buffer -> (step, gathered strips, Work, source) of the gather in flight from it
    nstep = [0]

    def collect(b):
        nonlocal gathered
        k, bufs, work, _src = pend.pop(b)
        collective(f"gather of step {k}'s strips (wait)", work.wait)
        gathered = bufs

    def step(record):
        nonlocal gathered
        b = nstep[0] % len(strips)
        c = b % npipe  # this step's context and stream
        nstep[0] += 1
        if not STUB:
            torch.cuda.set_stream(streams[c])  # the gather below (and the wait on its buffer) on this stream
        if b in pend:  # this buffer's previous gather must be done before the render overwrites it
            collect(b)
        buf = strips[b]
        if record:
            ev.append(timed_render(buf=buf, c=c))
        else:
            render_into((row0, row_step, nrows), buf, c)
        if STALL_RANK == rank:  # test only: this rank stalls before its gather
            time.sleep(STALL_S)
        if DIST:  # the single exchange step: strips -> rank 0 over RCCL/xGMI, overlapping the next render
            src = buf if coll.type == dev.type else buf.cpu()  # (gloo rehearsal: host copy)
            if GATHER_INLINE:
                gathered = collective(f"gather of step {nstep[0]}'s strips", rdist.gather_strips, src, rank, N, dst=0,
                                      group=ctx_groups[c])
            else:
                bufs, work = collective(f"gather of step {nstep[0]}'s strips", rdist.gather_strips, src, rank, N,
                                        dst=0, async_op=True)
                pend[b] = (nstep[0], bufs, work, src)  # the source stays referenced until the gather is done

    def drain():  # every gather in flight, in the order issued (the last one's strips are `gathered`)
        for b in sorted(pend, key=lambda k: pend[k][0]):
            collect(b)

    for _ in range(args.warmup):
        step(False)
    drain()
    for c in range(min(args.warmup, npipe), npipe):
        # a context the warmup steps did not reach renders its rows once,
        # untimed, so that every timed step reuses its own context's cost map
        render_into((row0, row_step, nrows), strips[c], c)
    sync()
    if not STUB:
        torch.cuda.set_stream(streams[0])
    if DIST:
        collective("barrier before the timed region", dist.barrier)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    drain()
    sync()
    if DIST:
        collective("barrier after the timed region", dist.barrier)
    sync()
    elapsed = my_elapsed = time.perf_counter() - t0
    if not STUB:
        torch.cuda.set_stream(streams[0])
    if DIST:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll)
        collective("all_reduce(max) of the timed region", dist.all_reduce, t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # GPU time per launch: the union of the launches' intervals / K (launches on
    # two streams overlap at their ends); launch_ms = the mean of each launch's
    # own start-to-end time, which counts the overlap once per launch
    kernel_ms = busy_ms_per_launch(ev)
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    segs = r.last_segments()  # this rank's strip, last render
    timed_sched = None if STUB else r.last_schedule()  # the timed launches' kernel (roofline.pmc guard)
    # The side launches below run one at a time on context 0: the
    # single-launch schedule, not the overlap hint of the timed steps
    r.set_overlap(False)
    dist_info = None
    if DIST:
        # the gather's own time (outside the timed region, where it overlaps
        # the next render): one more step with a blocking gather between HIP
        # events on the render's stream (from the end of this rank's render to
        # the end of the collective: includes waiting for the slowest rank)
        render_into((row0, row_step, nrows), strip)
        g0, g1 = Event(enable_timing=True), Event(enable_timing=True)
        g0.record(stream)
        collective("blocking gather (gather_ms)", rdist.gather_strips,
                   strip if coll.type == dev.type else strip.cpu(), rank, N, dst=0)
        g1.record(stream)
        sync()
        gev.append((g0, g1))
        # per-rank attribution of the step time: each rank's kernel time, its
        # gather time (from the end of its own render to the end of the
        # collective: includes waiting for the slowest rank) and its work
        gather_ms = float(np.mean([a.elapsed_time(b) for a, b in gev]))
        mine = torch.tensor([kernel_ms, gather_ms, float(segs), my_elapsed], dtype=torch.float64, device=coll)
        every = [torch.zeros_like(mine) for _ in range(N)]
        collective("all_gather of per-rank timings", dist.all_gather, every, mine)
        every = np.array([e.cpu().numpy() for e in every])
        total_segs = float(every[:, 2].sum())
        kernel_ms_max = float(every[:, 0].max())
        if not GATHER_INLINE:
            gather_note = "timed steps overlap step k's gather with step k+1's render (strip buffers per context)"
        elif npipe > 1:
            gather_note = ("timed steps: step k's gather runs on its context's stream right after its render, over "
                           "that context's process group, while step k+1 renders on the other context")
        else:
            gather_note = "timed steps: step k's gather runs on the render stream between renders k and k+1"
        dist_info = {"backend": str(dist.get_backend()), "world_size": dist.get_world_size(),
                     "kernel_ms_per_rank": [round(float(x), 3) for x in every[:, 0]],
                     "gather_ms_per_rank": [round(float(x), 3) for x in every[:, 1]],
                     "gather_note": gather_note + "; gather_ms is one blocking gather measured after the timed region",
                     "segments_per_rank": [int(x) for x in every[:, 2]],
                     "wall_s_per_rank": [round(float(x), 4) for x in every[:, 3]],
                     "kernel_imbalance": round(float(every[:, 0].max() / every[:, 0].mean()), 4)}
    else:
        total_segs, kernel_ms_max = float(segs), kernel_ms

    # --- everything below is outside the timed region ---------------------
    # config-3 parity: the gathered N-GPU image == rank 0's own render of the
    # whole frame, bit for bit (every pixel's stream is keyed by its
    # coordinates, so the partition must not change a single value)
    gather_check = None
    if DIST and not args.timed_only:
        if rank == 0:
            full = torch.empty((H, W, 3), dtype=torch.float32, device=dev)
            e0, e1 = timed_render((0, 1, H), full)
            sync()
            img = rdist.unpermute([g.cpu().numpy() for g in gathered], H)
            ref = full.cpu().numpy()
            equal = bool(np.array_equal(img, ref))
            gather_check = {"rows": H, "bit_exact_vs_1gpu_frame": equal, "max_abs_diff": float(np.abs(img - ref).max()),
                            "one_gpu_frame_ms": round(e0.elapsed_time(e1), 3)}
            if not equal:
                print(f"bench: gathered {N}-GPU image differs from the 1-GPU frame: {gather_check}", file=sys.stderr)
        collective("barrier after the gather check", dist.barrier)

    # one-shot render (the reference's use case renders once, main.cpp:292-360):
    # no cost map from a previous identical render, so the library runs its
    # probe pass first (included); and the same render in plain image order
    one_shot = None
    if args.ordering == "cost" and not args.timed_only:
        r.set_ordering("cost")  # forgets the previous render's cost map
        if DIST:
            # One render as the reference's use case does it, on every rank: from
            # a common start (barrier) to the end of the blocking gather of the
            # strips at rank 0, max over ranks
            collective("barrier before the one-shot render", dist.barrier)
            sync()
            t1 = time.perf_counter()
            e0, e1 = timed_render()
            collective("one-shot gather", rdist.gather_strips, strip if coll.type == dev.type else strip.cpu(), rank, N,
                       dst=0)
            sync()
            os_wall = time.perf_counter() - t1
            t = torch.tensor([os_wall], dtype=torch.float64, device=coll)
            collective("all_reduce(max) of the one-shot render", dist.all_reduce, t, op=dist.ReduceOp.MAX)
            os_wall = float(t.item())
        else:
            e0, e1 = timed_render()
        r.set_ordering("none")
        e2, e3 = timed_render()
        sync()
        one_shot = {"probe_ordered_ms": round(e0.elapsed_time(e1), 3), "image_order_ms": round(e2.elapsed_time(e3), 3)}
        if not DIST:  # this rank's rows are the whole workload (or the --strip-of strip)
            one_shot["msamples_per_s"] = round(nrows_valid * W * SPP / (one_shot["probe_ordered_ms"] * 1e-3) / 1e6, 3)
        else:  # the whole frame over N GPUs: render with its probe + gather, wall clock, max over ranks
            one_shot["wall_ms_max_rank"] = round(os_wall * 1e3, 3)
            one_shot["msamples_per_s"] = round(W * H * SPP / os_wall / 1e6, 3)
            one_shot["note"] = ("one render of the frame from a common barrier to the end of the blocking gather at "
                                "rank 0 (cost probe included), host wall clock, max over ranks; probe_ordered_ms is "
                                "rank 0's render alone (HIP events)")
        r.set_ordering(args.ordering)

    # The brute-force kernel's own VALU roofline: one more launch of the same
    # rows, untimed.
    bf = None
    if args.accel != "none" and rank == 0 and not args.timed_only:
        r.set_accel("none")
        e0, e1 = timed_render()
        sync()
        bf_ms = e0.elapsed_time(e1)
        bf_segs = r.last_segments()
        r.set_accel(args.accel)
        bf_ach = bf_segs * FLOP_PER_SPHERE_TEST * len(world) / (bf_ms * 1e-3) / 1e12
        bf = {"kernel_ms": round(bf_ms, 3), "achieved": round(bf_ach, 3), "frac": round(bf_ach / PEAK_FP32_TFLOPS, 4)}

    if rank == 0:
        samples = W * H * SPP if not args.strip_of else nrows * W * SPP
        value = samples * args.steps / elapsed / 1e6
        flop_eq = segs * FLOP_PER_SPHERE_TEST * len(world)  # brute-force-equivalent work of this rank's launch
        counts, why = None, None
        if args.accel == "none":
            flop_exec = flop_eq  # brute force executes every miss test
        elif args.no_exec_counts or STUB:
            flop_exec, why = None, "skipped (stub renderer)" if STUB else "skipped (--no-exec-counts)"
        else:
            counts, why = executed_counts(W, H, SPP, row0, row_step, nrows, args.accel, args.kernel)
            flop_exec = executed_flop(counts, args.accel) if counts else None
            if counts and counts["segments"] != segs:
                why = f"stats build segments {counts['segments']} != product {segs}"
                flop_exec = None
        achieved = flop_exec / (kernel_ms * 1e-3) / 1e12 if flop_exec else None
        eq_ach = flop_eq / (kernel_ms * 1e-3) / 1e12
        traffic, pmc_notes = None, {}
        lib_path = None if STUB else rt._abi.LIB_PATH
        ksym = None if STUB else timed_kernel_symbol(timed_sched, r.grid_info()[0][1] == 1)
        pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc) and args.workload == "config2" and not args.strip_of and N == 1 and not STUB:  # measured on config 2
            try:
                rec, pmc_notes["traffic"] = pmc_guard(json.load(open(pmc)).get(args.accel), lib_path, ksym)
                traffic = rec["hbm_bytes_per_launch"] if rec else None
            except Exception as e:
                traffic, pmc_notes["traffic"] = None, f"unreadable: {e}"
        roof = {
            "bound": "valu",
            "achieved": round(achieved, 3) if achieved else None,
            "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP32_TFLOPS, 4) if achieved else None,
            # SURVEY 8(d) also asks for the fraction of a 78.6 TFLOP/s "non-packed" peak;
            # on gfx950 a wave64 v_fma_f32 issues every 2 cycles (MI355X_MICROARCH.md), so
            # plain FMAs already reach 157.3 and this is context only
            "frac_vs_78_6": round(achieved / (PEAK_FP32_TFLOPS / 2), 4) if achieved else None,
            "traffic": traffic,
            "work": {"bvh": "executed: node slab tests x 25 + sphere miss tests x 18 FLOP, counted per lane by the "
                            "RTMI_STATS build on the same rows",
                     "grid": "executed: one grid-box slab test x 25 per segment + DDA cell steps x 5 + sphere miss "
                             "tests x 18 FLOP, counted per lane by the RTMI_STATS build on the same rows",
                     "none": "executed: segments x spheres x 18 FLOP (brute force)"}[args.accel],
            "flop_per_launch": flop_exec,
            "kernel_ms": round(kernel_ms, 3),
            "kernel_ms_note": ("GPU time per launch: union of the timed launches' HIP-event intervals / steps (launches "
                               "of consecutive steps overlap at their ends on two streams; launch_ms_mean counts the "
                               "overlap in both)") if npipe > 1 else "mean HIP-event duration of the timed launches",
            "launch_ms_mean": round(launch_ms, 3),
            "kernel_ms_max_rank": round(kernel_ms_max, 3),
            "segments_per_launch": segs,
            "segments_per_sample": round(total_segs / samples, 4),
            "work_equivalent_achieved": round(eq_ach, 3),
            "work_equivalent_frac": round(eq_ach / PEAK_FP32_TFLOPS, 4),
            "brute_force_frac": bf["frac"] if bf else (round(eq_ach / PEAK_FP32_TFLOPS, 4) if args.accel == "none" else None),
            "brute_force": bf,
        }
        if counts:
            ls = counts["segments"]
            ws_ = ls / 64.0
            roof["counts"] = {
                "node_visits_per_segment": round(counts["node_visits"] / ls, 3),
                "leaf_sphere_tests_per_segment": round(counts["leaf_sphere_tests"] / ls, 3),
                "big_spheres": counts["big_spheres"],
                "node_iterations_per_wave_segment": round(counts["node_iterations_wave"] / ws_, 3),
                "leaf_sphere_iterations_per_wave_segment": round(counts["leaf_sphere_iterations_wave"] / ws_, 3),
                "walk_lane_utilisation": round(counts["node_visits"] / max(1, 64 * counts["node_iterations_wave"]), 4),
                "leaf_lane_utilisation": round(counts["leaf_sphere_tests"] / max(1, 64 * counts["leaf_sphere_iterations_wave"]), 4),
            }
            if counts.get("wave_passes"):  # (a stats build that counts wave passes)
                roof["counts"]["live_lanes_per_pass"] = round(counts["segments"] / counts["wave_passes"], 2)
        # Context beside the algorithmic fraction, from the committed PMC passes
        # of the same kernel on the same workload (tools/profile.sh,
        # profiles/pmc_valu.json) over this run's kernel time: every FP32 FLOP
        # the kernel executes (shading, regeneration and idle-lane slots
        # included) and how busy the VALU issue is — the bound of this
        # divergent kernel
        pmcv = os.path.join(REPO, "profiles", "pmc_valu.json")
        if (os.path.exists(pmcv) and args.workload == "config2" and args.accel == "grid" and not args.strip_of and N == 1
                and not STUB):
            try:
                pv, pmc_notes["pmc"] = pmc_guard(json.load(open(pmcv)), lib_path, ksym)
                roof["pmc"] = None
            except Exception as e:
                pv, pmc_notes["pmc"] = None, f"unreadable: {e}"
            try:
                ks = kernel_ms * 1e-3
                roof["pmc"] = None if pv is None else {
                    "source": "profiles/pmc_valu.json",
                    "executed_fp32_flop_per_launch": pv["executed_fp32_flop_per_launch"],
                    "executed_fp32_frac": round(pv["executed_fp32_flop_per_launch"] / ks / 1e12 / PEAK_FP32_TFLOPS, 4),
                    "valu_issue_busy": round(pv["per_launch"]["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9 * ks), 4),
                    "lane_utilisation": round(pv["lane_utilisation"], 4),
                    "wait_fraction": round(pv["wait_fraction"], 4),
                }
            except Exception:
                pass
        pmc_notes = {k: v for k, v in pmc_notes.items() if v}
        if pmc_notes:  # why roofline.traffic / roofline.pmc are null
            roof["pmc_guard"] = {"timed_kernel": ksym, **pmc_notes}
        if why:
            roof["note"] = why
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            # the reference's use case renders once (main.cpp:292-360): a render
            # with no cost map of its layout runs a 1-spp, depth-8 probe pass first
            # (kernel time of that one render, HIP events); the timed steps
            # above reuse the previous identical render's map (config.timed_steps)
            "one_shot_msamples_per_s": (one_shot or {}).get("msamples_per_s"),
            "unit": "Msamples/s",
            "n_gpus": N,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / PUBLISHED_CPU_MSPS, 1),
            "dtype": "f32",
            "data": ("STUB renderer: CPU rehearsal of the launch / rank / gather / line path, not a measurement"
                     if STUB else "synthetic: RTIOW final scene regenerated from glibc rand() seed 1 (487 spheres, = reference)"),
            "config": {
                "workload": f"rtiow_final_{W}x{H}_{SPP}spp_depth{DEPTH}",
                "width": W, "height": H, "spp": SPP, "max_depth": DEPTH, "seed": SEED, "spheres": len(world),
                "partition": "interleaved rows, one RCCL gather" if DIST else "single GPU",
                "tile": f"{tw}x{64 // tw}" + ("" if args.tile_w else " (auto)"),
                "kernel": args.kernel,
                "accel": args.accel,
                "ordering": args.ordering,
                "pipeline": npipe,
                **({"gather": ("inline: on each context's stream, one process group per context" if GATHER_INLINE
                               else "side: async on the default group's NCCL stream")} if DIST else {}),
                "overlap_schedule": bool(npipe > 1 and args.steps >= 8 and not STUB),
                "timed_steps": ("each step re-renders the same workload; with ordering 'cost' it dispatches tiles by the "
                                "previous identical render's per-tile cost map (RT_ORDER_COST): the first render of a "
                                "layout (warmup) pays a 1-spp probe pass instead, see one_shot_msamples_per_s"
                                if args.ordering == "cost" else "image-order dispatch, no cost map"),
            },
            "roofline": roof,
            "one_shot": one_shot,
            "vs_baseline_ref": "published CPU rt_in_one_weekend 0.1189 Msamples/s (README.md:16-19)",
        }
        if STUB:
            line["stub"] = True
        if FORCE_DIST and N == 1:
            line["config"]["dist_rehearsal"] = DIST_REHEARSAL
        if dist_info is not None:
            line["dist"] = dist_info
        if gather_check is not None:
            line["gather_check"] = gather_check
        if not DIST and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), flush=True)
        if gather_check is not None and not gather_check["bit_exact_vs_1gpu_frame"]:
            dist.destroy_process_group()
            close_all(rs, destroy_streams)
            sys.exit(3)
    if DIST:  # (before the streams its collectives ran on are destroyed)
        dist.destroy_process_group()
    close_all(rs, destroy_streams)


def close_all(rs, destroy_streams):
    for x in rs:
        x.close()
    if destroy_streams:
        destroy_streams()


NW_PUBLISHED_MSPS = 1200 * 800 * 500 / 37.8792 / 1e6  # rt_next_week/cuda/README.md:167-174 (RTX 2060 Max-Q)
# Algorithmic FLOP of one miss test per Next-Week object kind (the reference's
# hit functions): sphere.h 18 (as the RTIOW count, |d|^2
# hoisted); moving_sphere.h center(t) 12 + 18; aarect.h t, two coordinates 6;
# box.h = its six rects 36; constant_medium.h its boundary twice + 4; and per
# instance (translate + rotate_y of the ray) 15.
NW_FLOP = {0: 18, 1: 30, 2: 6, 3: 6, 4: 6, 5: 36}
NW_FLOP_INSTANCE = 15


def nw_flop_per_segment(flat):
    """Brute-force-equivalent FLOP of one world.hit over the flattened scene."""
    obj = flat["obj"].view(np.int32).reshape(-1, 16)
    kind, aux = obj[:, 12], obj[:, 15]
    total = 0
    for k, a in zip(kind, aux):
        total += NW_FLOP[int(k)] if k != 6 else 2 * NW_FLOP[int(a) & 255] + 4
    return total + NW_FLOP_INSTANCE * (flat["inst"].size // 8)


def nw_cpu_baseline(flat, cam, which, W, H):
    """The oracle's Next-Week restatement (C, OpenMP, brute force over the
    objects: the CPU port, the reference being CUDA only) on a bounded
    sample of the same scene: 40 evenly spaced rows."""
    try:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_py as O

        spp = 20 if which == 8 else 160  # ~10-15 s on the GPU box's 16 host threads
        rows = 40
        t0 = time.perf_counter()
        O.nw_render(flat, cam, W, H, spp, DEPTH, SEED, row0=0, row_step=H // rows, nrows=rows)
        dt = time.perf_counter() - t0
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        return {"value": round(rows * W * spp / dt / 1e6, 5), "unit": "Msamples/s", "cores": threads, "kind": "port",
                "sample": f"oracle Next-Week C restatement (brute force over objects), {rows} rows x {W} x {spp} spp "
                          f"({dt:.1f} s wall, OpenMP)"}
    except Exception as e:
        print(f"bench: nw cpu baseline unavailable: {e}", file=sys.stderr)
        return None


def bench_nw(args):
    """Secondary line: a Next-Week scene (include/rtmi_nw.h) with the headline's
    timing contract (barrier + sync around K steps, max over ranks)."""
    import torch
    import torch.distributed as dist

    import a_dive_into_ray_tracing_amd.nextweek as nw
    from a_dive_into_ray_tracing_amd import dist as rdist

    N, rank, local_rank, dev, coll = dist_setup(torch, dist)
    DIST = N > 1 or FORCE_DIST  # (as in main)
    if args.workload == "nw_motion_blur":
        which, Wn, Hn, spp = 1, 1200, 800, args.nw_spp or 500
        earth = None
    else:
        which, Wn, Hn, spp = 8, 800, 800, args.nw_spp or 1024
        earth = nw.load_image(os.path.join(REPO, "tests", "golden", "earthmap.jpeg"))
    if args.nw_preset:
        which = args.nw_preset
        earth = nw.load_image(os.path.join(REPO, "tests", "golden", "earthmap.jpeg"))
    scene, cam = nw.preset(which, image=earth, aspect=Wn / Hn)
    r = nw.NwRenderer(scene, local_rank)
    r.set_accel(args.nw_accel)
    accel = r.accel_info()
    row0, row_step, nrows = rdist.strip_rows(Hn, rank, N)
    strip = torch.empty((nrows, Wn, 3), dtype=torch.float32, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ev = []

    def step(record):
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        r.render_rows(cam, Wn, Hn, spp, DEPTH, SEED, row0, row_step, nrows, strip.data_ptr(), stream.cuda_stream)
        if record:
            e1.record(stream)
            ev.append((e0, e1))
        if DIST:
            collective("gather of the strips", rdist.gather_strips, strip if coll.type == "cuda" else strip.cpu(), rank, N,
                       dst=0)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if DIST:
        collective("barrier before the timed region", dist.barrier)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    if DIST:
        collective("barrier after the timed region", dist.barrier)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if DIST:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll)
        collective("all_reduce(max) of the timed region", dist.all_reduce, t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # GPU time per launch: the union of the launches' intervals / K (launches on
    # two streams overlap at their ends); launch_ms = the mean of each launch's
    # own start-to-end time, which counts the overlap once per launch
    kernel_ms = busy_ms_per_launch(ev)
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    segs = r.last_segments()
    flop_seg = nw_flop_per_segment(scene.flat())
    flop_rank = segs * flop_seg  # this rank's launch, brute-force equivalent
    eq_achieved = flop_rank / (kernel_ms * 1e-3) / 1e12
    counts, why = None, None
    if rank == 0 and not args.no_exec_counts:
        counts, why = nw_executed_counts(which, Wn, Hn, spp, row0, row_step, nrows, args.nw_accel)
        if counts and counts["segments"] != segs:
            why, counts = f"stats build segments {counts['segments']} != product {segs}", None
    elif args.no_exec_counts:
        why = "skipped (--no-exec-counts)"
    achieved = counts["flop"] / (kernel_ms * 1e-3) / 1e12 if counts else None
    if rank == 0:
        samples = Wn * Hn * spp
        value = samples * args.steps / elapsed / 1e6
        line = {
            "metric": f"Msamples/sec (pixels x spp) on the Next-Week {args.workload[3:]} scene",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": N, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": round(value / NW_PUBLISHED_MSPS, 1) if args.workload == "nw_motion_blur" and spp == 500 else None,
            "dtype": "f32",
            "data": "synthetic: the reference's scene regenerated from a restated curand XORWOW (curand_init(1984,0,0))",
            "config": {"workload": f"{args.workload}_{Wn}x{Hn}_{spp}spp_depth{DEPTH}", "scene": which, "width": Wn,
                       "height": Hn, "spp": spp, "max_depth": DEPTH, "seed": SEED,
                       "partition": "interleaved rows, one RCCL gather" if DIST else "single GPU",
                       "accel": accel["accel"], "grid_dims": list(accel["dims"]), "grid_max_cell": accel["max_cell"],
                       "brute_force_objects": accel["n_big"]},
            "roofline": {
                "bound": "valu", "achieved": round(achieved, 3) if achieved else None, "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4) if achieved else None,
                "traffic": None,
                "work": "executed: the miss tests the BVH / grid walk performs (bench.NW_FLOP per kind, +15 per "
                        "instance transform, media 2 x boundary + 4) + 25 per node slab test or grid clip + 5 per "
                        "cell step, counted per lane by the RTMI_STATS build on the same rows",
                "flop_per_launch": counts["flop"] if counts else None,
                "counts": {k: counts[k] for k in ("node_visits", "object_tests", "cell_steps")} if counts else None,
                "kernel_ms": round(kernel_ms, 3), "segments_per_launch": segs,
                "work_equivalent_achieved": round(eq_achieved, 3),
                "work_equivalent_frac": round(eq_achieved / PEAK_FP32_TFLOPS, 4),
                "work_equivalent_flop_per_segment": flop_seg,
                "work_equivalent_note": "brute-force-equivalent FLOP (every object's miss test per world.hit) over "
                                        "the kernel's time, as SURVEY 8(d) prescribes for culling: can exceed 1",
            },
            "kernel_ms": round(kernel_ms, 3),
            "segments_per_sample_rank0": round(segs / (nrows * Wn * spp), 4),
            "objects_bvh_nodes": list(r.info()),
            "vs_baseline_ref": "reference rt_next_week CUDA, random_scene with moving spheres 1200x800x500 in 37.88 s "
                               "(RTX 2060 Max-Q): 12.67 Msamples/s",
        }
        if why:
            line["roofline"]["note"] = why
        if FORCE_DIST and N == 1:
            line["config"]["dist_rehearsal"] = DIST_REHEARSAL
        if not DIST and not args.no_cpu_baseline:
            line["cpu_baseline"] = nw_cpu_baseline(scene.flat(), cam, which, Wn, Hn)
        print(json.dumps(line), flush=True)
    r.close()
    if DIST:
        dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    except CollectiveError as e:
        # a stalled or failed collective: non-zero at once, rank and collective
        # on stderr, stdout untouched (the JSON line is printed only at the
        # end); os._exit, since tearing down a group whose peer is stuck can
        # block (the reference's check_cuda exits the process too, final.cu:13-24)
        print(f"bench: rank {os.environ.get('RANK', '0')} of {os.environ.get('WORLD_SIZE', '1')}: collective failed "
              f"(timeout {DIST_TIMEOUT_S:g} s): {e}", file=sys.stderr, flush=True)
        os._exit(5)
