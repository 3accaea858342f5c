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

Closest hits go through the BVH by default (--accel bvh): the same closest
hit as the brute-force loop, bit for bit (tests/test_gpu_parity.py), so the
same image.  --accel none times the brute-force kernel.

roofline: FP32 VALU.  achieved = segments * 18 * 487 FLOP per launch
(18 flops per ray-sphere test, brute force over 487 spheres;
segments = world.hit calls, counted exactly on the GPU) / mean launch time
from HIP events on the launch stream; peak = 157.3 TFLOP/s FP32 vector.
With the BVH this is the brute-force-equivalent ("work_equivalent", as
SURVEY §8(d) prescribes for culling), so frac can exceed 1; roofline.
brute_force gives the brute-force kernel's own figure from one extra,
untimed launch of the same rows.
cpu_baseline: the reference itself (oracle/_ref/ref_harness: worker() at -O2,
16 std::threads as the reference's concurrency) on a bounded sample, rank 0,
N = 1 only.

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
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

W, H, SPP, DEPTH, SEED = 1200, 800, 500, 50, 1984
FLOP_PER_SPHERE_TEST = 18
PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 vector (MI355X_MICROARCH.md)
PUBLISHED_CPU_MSPS = 0.1189  # README.md:16-19: rt_in_one_weekend, 1200x800x500, 16 threads, 4036.1 s
METRIC = "Msamples/sec (pixels x spp) on RTIOW final scene"
# BASELINE.json configs on the final scene: config2 = the headline (1 GPU,
# 1200x800x500); config4 = the same at 5000 spp; config5 = 3840x2160 (16:9
# camera) at 2000 spp (quoted for 8 GPUs; the final scene has the
# reference's defocus blur, aperture 0.1).
RTIOW_WORKLOADS = {"config2": (1200, 800, 500), "config4": (1200, 800, 5000), "config5": (3840, 2160, 2000)}


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
    device = local_rank % max(1, torch.cuda.device_count()) if backend == "gloo" else local_rank
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    if world_size > 1:
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    coll = dev if backend == "nccl" else torch.device("cpu")
    return world_size, rank, device, dev, coll


def cpu_baseline(threads=16):
    """The reference's own worker() (oracle/_ref/ref_harness bench) on a
    bounded sample: full 1200x800 image at 4 spp (~3.8 M samples)."""
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    spp = 4
    if os.path.exists(harness):
        try:
            out = subprocess.run([harness, "bench", str(threads), str(W), str(H), str(spp), str(DEPTH)],
                                 capture_output=True, text=True, timeout=300, check=True).stdout
            r = json.loads(out.strip().splitlines()[-1])
            return {"value": round(r["msamples_per_s"], 5), "unit": "Msamples/s", "cores": threads, "kind": "reference",
                    "sample": f"reference worker() g++ -O2, {threads} std::threads, final scene {W}x{H}x{spp}spp depth {DEPTH} "
                              f"({r['seconds']:.1f} s wall)"}
        except Exception as e:  # fall through to the port
            print(f"bench: reference harness failed: {e}", file=sys.stderr)
    try:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_py as O
        import ctypes

        sc, _ = O.final_scene()
        cam = O.final_camera(1.5)
        rows = 40
        os.environ.setdefault("OMP_NUM_THREADS", str(threads))
        t0 = time.perf_counter()
        O.fast_render(sc, cam, W, H, spp, DEPTH, SEED, row0=0, row_step=H // rows, nrows=rows)
        dt = time.perf_counter() - t0
        return {"value": round(rows * W * spp / dt / 1e6, 5), "unit": "Msamples/s", "cores": int(os.environ["OMP_NUM_THREADS"]),
                "kind": "port", "sample": f"oracle fast-mode C restatement, {rows} rows x {W} x {spp} spp"}
    except Exception as e:
        print(f"bench: cpu baseline unavailable: {e}", file=sys.stderr)
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tile-w", type=int, default=0, help="0 = automatic (the library default)")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--tail-spp", type=int, default=-1)
    ap.add_argument("--tail-chunk", type=int, default=0)
    ap.add_argument("--kernel", choices=["auto", "persistent", "grid"], default="auto")
    ap.add_argument("--accel", choices=["none", "bvh"], default="bvh",
                    help="closest-hit search: bvh (default; same image bit for bit) or brute force")
    ap.add_argument("--ordering", choices=["cost", "none"], default="cost")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=list(RTIOW_WORKLOADS) + ["nw_motion_blur", "nw_final"], default="config2")
    ap.add_argument("--nw-spp", type=int, default=0, help="spp of the nw_* workloads (default: 500 / 1024)")
    ap.add_argument("--strip-of", type=int, default=0,
                    help="analysis only: time ONE rank's interleaved strip of an N-GPU run on this GPU")
    args = ap.parse_args()
    if args.workload.startswith("nw_"):
        return bench_nw(args)
    W, H, SPP = RTIOW_WORKLOADS[args.workload]

    import torch
    import torch.distributed as dist

    import a_dive_into_ray_tracing_amd as rt
    from a_dive_into_ray_tracing_amd import dist as rdist

    world_size, rank, local_rank, dev, coll = dist_setup(torch, dist)
    if world_size != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE {world_size}", file=sys.stderr)
    N = world_size

    world = rt.random_scene()
    cam = rt.final_camera(W / H)
    r = rt.Renderer(world, local_rank, tile_w=args.tile_w, chunk=args.chunk)
    r.set_schedule(args.chunk, args.tail_spp, args.tail_chunk)
    r.set_kernel(args.kernel)
    r.set_accel(args.accel)
    r.set_ordering(args.ordering)
    row0, row_step, nrows = rdist.strip_rows(H, rank, N)  # interleaved rows, row j -> rank j % N
    if args.strip_of > 1 and N == 1:  # analysis mode: one rank's share of an N-GPU render
        row0, row_step, nrows = rdist.strip_rows(H, 0, args.strip_of)
    strip = torch.empty((nrows, W, 3), dtype=torch.float32, device=dev)
    tw = args.tile_w or rt.auto_tile_w(W, -(-(H - row0) // row_step) if row0 < H else 0)  # reported tile shape
    gathered = None
    # a non-default stream: the kernel, its HIP events and the RCCL gather
    # are all ordered on it (the null stream would bypass the events)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    ev = []

    def step(record):
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        nonlocal gathered
        r.render_rows(cam, W, H, SPP, DEPTH, SEED, row0, row_step, nrows, strip.data_ptr(), stream.cuda_stream)
        if record:
            e1.record(stream)
            ev.append((e0, e1))
        if N > 1:  # the single exchange step: strips -> rank 0 over RCCL/xGMI
            gathered = rdist.gather_strips(strip if coll.type == "cuda" else strip.cpu(), rank, N, dst=0)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if N > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    if N > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if N > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    segs = r.last_segments()  # this rank's strip, last render
    if N > 1:
        t = torch.tensor([segs], dtype=torch.float64, device=coll)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        total_segs = float(t.item())
        km = torch.tensor([kernel_ms], dtype=torch.float64, device=coll)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kernel_ms_max = float(km.item())
    else:
        total_segs, kernel_ms_max = float(segs), kernel_ms

    # The brute-force kernel's own VALU roofline, beside the BVH's
    # work-equivalent one: one more launch of the same rows, untimed.
    bf = None
    if args.accel != "none":
        r.set_accel("none")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r.render_rows(cam, W, H, SPP, DEPTH, SEED, row0, row_step, nrows, strip.data_ptr(), stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        bf_ms = e0.elapsed_time(e1)
        bf_segs = r.last_segments()
        r.set_accel(args.accel)
        bf_ach = bf_segs * FLOP_PER_SPHERE_TEST * len(world) / (bf_ms * 1e-3) / 1e12
        bf = {"kernel_ms": round(bf_ms, 3), "achieved": round(bf_ach, 3), "frac": round(bf_ach / PEAK_FP32_TFLOPS, 4),
              "note": "brute-force kernel (RT_ACCEL_NONE) on the same rows: the FP32 VALU roofline proper"}

    if rank == 0 and N > 1:  # the gathered image is whole: every row rendered, none twice
        img = rdist.unpermute([g.cpu().numpy() for g in gathered], H)
        assert np.isfinite(img).all() and (img.reshape(H, -1).max(axis=1) > 0).all(), "incomplete gathered image"
    if rank == 0:
        samples = W * H * SPP if not args.strip_of else nrows * W * SPP
        value = samples * args.steps / elapsed / 1e6
        flop_rank = segs * FLOP_PER_SPHERE_TEST * len(world)  # this rank's launch
        achieved = flop_rank / (kernel_ms * 1e-3) / 1e12
        traffic = None
        pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc) and args.workload == "config2" and not args.strip_of:  # measured on config 2
            try:
                traffic = (json.load(open(pmc)).get(args.accel) or {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": N,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / PUBLISHED_CPU_MSPS, 1),
            "dtype": "f32",
            "data": "synthetic: RTIOW final scene regenerated from glibc rand() seed 1 (487 spheres, = reference)",
            "config": {
                "workload": f"rtiow_final_{W}x{H}_{SPP}spp_depth{DEPTH}",
                "width": W, "height": H, "spp": SPP, "max_depth": DEPTH, "seed": SEED, "spheres": len(world),
                "partition": "interleaved rows, one RCCL gather" if N > 1 else "single GPU",
                "tile": f"{tw}x{64 // tw}" + ("" if args.tile_w else " (auto)"),
                "kernel": args.kernel,
                "accel": args.accel,
                "ordering": args.ordering,
            },
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved, 3),
                "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                "traffic": traffic,
                "flop_per_launch": flop_rank,
                "segments_per_launch": segs,
                "segments_per_sample": round(total_segs / samples, 4),
                "kernel_ms": round(kernel_ms, 3),
                "kernel_ms_max_rank": round(kernel_ms_max, 3),
                # with the BVH the FLOP count stays the brute-force figure
                # ("work-equivalent"), so frac can pass 1
                "work_equivalent": args.accel != "none",
                "brute_force": bf,
            },
            "vs_baseline_ref": "published CPU rt_in_one_weekend 0.1189 Msamples/s (README.md:16-19)",
        }
        if N == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), flush=True)
    r.close()
    if N > 1:
        dist.destroy_process_group()


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
    if args.workload == "nw_motion_blur":
        which, Wn, Hn, spp = 1, 1200, 800, args.nw_spp or 500
        earth = None
    else:
        which, Wn, Hn, spp = 8, 800, 800, args.nw_spp or 1024
        earth = nw.load_image(os.path.join(REPO, "tests", "golden", "earthmap.jpeg"))
    scene, cam = nw.preset(which, image=earth, aspect=Wn / Hn)
    r = nw.NwRenderer(scene, local_rank)
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
        if N > 1:
            rdist.gather_strips(strip if coll.type == "cuda" else strip.cpu(), rank, N, dst=0)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if N > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    if N > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if N > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    segs = r.last_segments()
    flop_seg = nw_flop_per_segment(scene.flat())
    flop_rank = segs * flop_seg  # this rank's launch
    achieved = flop_rank / (kernel_ms * 1e-3) / 1e12
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
                       "partition": "interleaved rows, one RCCL gather" if N > 1 else "single GPU"},
            "roofline": {
                "bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": None,
                "flop_per_launch": flop_rank, "flop_per_segment": flop_seg, "segments_per_launch": segs,
                "kernel_ms": round(kernel_ms, 3), "work_equivalent": True,
                "note": "brute-force-equivalent FLOP (every object's miss test per world.hit, bench.NW_FLOP) over the "
                        "BVH kernel's time, as SURVEY 8(d) prescribes for culling: frac can exceed 1",
            },
            "kernel_ms": round(kernel_ms, 3),
            "segments_per_sample_rank0": round(segs / (nrows * Wn * spp), 4),
            "objects_bvh_nodes": list(r.info()),
            "vs_baseline_ref": "reference rt_next_week CUDA, random_scene with moving spheres 1200x800x500 in 37.88 s "
                               "(RTX 2060 Max-Q): 12.67 Msamples/s",
        }
        if N == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = nw_cpu_baseline(scene.flat(), cam, which, Wn, Hn)
        print(json.dumps(line), flush=True)
    r.close()
    if N > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
