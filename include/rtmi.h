/* include/rtmi.h — C ABI of librtmi.so, the MI355X-native path tracer.
 *
 * Drop-in boundary for the reference's per-pixel sample loop
 * (xyloid/a_dive_into_ray_tracing, rt_in_one_weekend/).  The reference has no
 * FFI; its de-facto interface is the C++ call
 *     worker(start, end, std::ref(img), W, H, world, cam, spp, max_depth)
 *                                               rt_in_one_weekend/main.cpp:267-290
 * fed by hittable_list::objects (hittable_list.h:16-17) and the public camera
 * fields (camera.h:64-70), and followed by the P3 writer (color.h:14-28 via
 * main.cpp:344-355).  Every entry point below names the reference code it
 * replaces.  Plain pointers and sizes only; no C++ or torch types.
 *
 * Conventions
 *  - Every int-returning call returns RT_OK (0) or a negative RT_E* code and
 *    never exits the process (the CUDA reference exit(99)s: final.cu:13-24).
 *    rt_last_error() describes the last failure of the calling thread.
 *  - Inputs are copied; the caller keeps ownership.  Host outputs are caller
 *    allocated.  Image buffers are W*H*3 floats, index (j*W + i)*3 + c, row
 *    j = 0 at the BOTTOM (main.cpp:274-275), holding per-pixel SUMS over the
 *    samples (main.cpp:276-285) — not means.
 *  - Scene and camera are given in double (the reference's type) and rounded
 *    to float on entry; the render computes in float.
 *  - The image is a pure function of (scene, camera, W, H, spp, max_depth,
 *    seed): independent of tiling, scheduling, row partition and GPU count.
 *  - There is no CPU fallback: without a usable gfx950 device every render
 *    call fails with RT_ENODEVICE.
 */
#ifndef RTMI_H
#define RTMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTMI_VERSION_MAJOR 0
#define RTMI_VERSION_MINOR 1

enum {
  RT_OK = 0,
  RT_EINVAL = -1,       /* bad argument                                   */
  RT_EHIP = -2,         /* HIP runtime failure                            */
  RT_ENODEVICE = -3,    /* no HIP device / device index out of range      */
  RT_EUNSUPPORTED = -4, /* object/material type the path cannot render    */
  RT_ENOMEM = -5,       /* host or device allocation failed               */
  RT_ERCCL = -6,        /* RCCL failure (multi-GPU render)                */
  RT_EIO = -7,          /* file output failed                             */
  RT_ESTREAM = -8       /* replay stream exhausted                        */
};

/* material kinds, material.h:15-97 */
enum { RT_MAT_LAMBERTIAN = 0, RT_MAT_METAL = 1, RT_MAT_DIELECTRIC = 2 };

/* hittable_list of spheres (hittable_list.h:16-17, sphere.h:15-19). */
typedef struct rt_scene {
  int32_t n;                   /* number of spheres                               */
  const double *center_radius; /* 4n: cx cy cz radius (negative radius allowed)   */
  const int32_t *mat_kind;     /* n: RT_MAT_*                                     */
  const double *mat_params;    /* 4n: albedo r g b, then fuzz (metal) | ir (diel.) */
} rt_scene;

/* camera public fields, camera.h:64-70 */
typedef struct rt_camera {
  double origin[3];
  double lower_left_corner[3];
  double horizontal[3];
  double vertical[3];
  double u[3], v[3], w[3];
  double lens_radius;
} rt_camera;

typedef struct rt_ctx rt_ctx; /* one device, its stream, the resident scene */

/* ---------------- host helpers (no GPU needed) ------------------------- */
const char *rt_last_error(void);
int rt_version(void); /* (major << 16) | minor */

/* camera::camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist)
 * camera.h:8-45, evaluated in double exactly as the reference does. */
int rt_camera_init(rt_camera *cam, const double lookfrom[3], const double lookat[3],
                   const double vup[3], double vfov_deg, double aspect_ratio,
                   double aperture, double focus_dist);

/* random_scene() main.cpp:86-131 (final random-spheres scene), generated from
 * glibc's rand() stream seeded with `glibc_seed` (the reference never seeds:
 * 1) with GCC's draw order, so it equals the reference's 487 objects.
 * Writes up to `cap` spheres; *n_out = count.  RT_EINVAL if cap too small. */
int rt_scene_random(uint32_t glibc_seed, double *center_radius, int32_t *mat_kind,
                    double *mat_params, int32_t cap, int32_t *n_out);
/* learn() scene main.cpp:198-210 (config 1, five spheres incl. radius -0.4). */
int rt_scene_learn(double *center_radius, int32_t *mat_kind, double *mat_params, int32_t cap,
                   int32_t *n_out);

/* write_color(out, sum, spp) color.h:14-28 over the image, top row first
 * (main.cpp:344-355).  path "-" = stdout.  binary != 0 writes P6 instead of P3
 * with the same 8-bit values. */
int rt_write_ppm(const char *path, const float *sum, int32_t W, int32_t H, int32_t spp,
                 int32_t binary);
/* Same quantisation into rgb[W*H*3] bytes, top row first. */
int rt_quantize(const float *sum, int32_t W, int32_t H, int32_t spp, uint8_t *rgb);

/* PFM (colour "PF", little-endian): the pre-gamma mean sum/spp per channel,
 * bottom row first (PFM's own order, = row index order here). */
int rt_write_pfm(const char *path, const float *sum, int32_t W, int32_t H, int32_t spp);

/* Scene text files (the format of tests/golden/scene_final.txt): optional
 * count line, then "cx cy cz r kind a0 a1 a2 p" per sphere (%.17g, kind
 * RT_MAT_*, p = fuzz | ir), '#' comments.  rt_scene_read fills up to `cap`
 * spheres and sets *n_out to the file's count (RT_EINVAL if cap is too
 * small: call with cap 0 to size the arrays). */
int rt_scene_write(const char *path, const rt_scene *scene);
int rt_scene_read(const char *path, double *center_radius, int32_t *mat_kind, double *mat_params,
                  int32_t cap, int32_t *n_out);

/* ---------------- device ----------------------------------------------- */
int rt_device_count(int32_t *n);
/* Create a context on HIP device `device` (its own non-blocking stream). */
int rt_ctx_create(int32_t device, rt_ctx **out);
int rt_ctx_destroy(rt_ctx *ctx);
/* Upload the scene (replaces the per-thread copies of `world`,
 * main.cpp:331-333).  Synchronous; O(n). */
int rt_ctx_set_scene(rt_ctx *ctx, const rt_scene *scene);
/* Tuning: tile_w in {0, 8, 16, 32, 64} (tile = tile_w x 64/tile_w pixels per
 * wavefront; 0 = automatic, the default: 8 unless 16 leaves fewer idle lanes
 * in partial tiles); chunk = samples per work item (0 = automatic).  Neither
 * changes the image. */
int rt_ctx_set_tuning(rt_ctx *ctx, int32_t tile_w, int32_t chunk);
/* Work schedule: the first spp - tail_spp samples of every tile in items of
 * `chunk` samples, the last tail_spp in items of `tail_chunk`, dispatched
 * last (0 / -1 = automatic).  Does not change the image. */
int rt_ctx_set_schedule(rt_ctx *ctx, int32_t chunk, int32_t tail_spp, int32_t tail_chunk);
/* Launch-mode hint (MI355X extension, no reference counterpart): overlapped =
 * 1 when this context's renders run concurrently with another context's on
 * the same device (e.g. consecutive frames alternating over two contexts on
 * streams of their own hardware queues, bench.py --pipeline 2): the other
 * launch fills this one's dispatch tail, so the automatic schedule uses fewer,
 * longer work items.  0 (default) = launches run one at a time.  Does not
 * change the image. */
int rt_ctx_set_overlap(rt_ctx *ctx, int32_t overlapped);

/* Kernel shape.  RT_KERNEL_PERSISTENT: a resident grid of waves pulls work
 * items from a global counter and streams paths continuously (two items in
 * flight per wave) — brute force (RT_ACCEL_NONE) only: with the grid or the
 * BVH the grid kernel runs, which measured faster.
 * RT_KERNEL_GRID: one wave per work item.  RT_KERNEL_AUTO (default):
 * persistent for brute-force strips (fewer than 6e6 tile-samples), grid
 * otherwise.  RT_KERNEL_QUEUE (round 5's LDS ray-queue kernel, retired in
 * round 6: DESIGN.md §4.6) and RT_KERNEL_RESIDENT (CU-resident blocks over a
 * global work counter, DESIGN.md §4.7: built only into the experimental
 * library, lib/librtmi_experimental.so) run RT_KERNEL_AUTO in librtmi.so —
 * both measured slower than the grid kernel.  All give bit-identical images. */
enum { RT_KERNEL_GRID = 0, RT_KERNEL_PERSISTENT = 1, RT_KERNEL_AUTO = 2, RT_KERNEL_QUEUE = 3, RT_KERNEL_RESIDENT = 4 };
int rt_ctx_set_kernel(rt_ctx *ctx, int32_t kind);

/* Closest-hit search.  RT_ACCEL_NONE: brute force over all spheres, the
 * reference's hittable_list::hit (hittable_list.h:20-34).  RT_ACCEL_BVH: the
 * spheres much larger than the median (the ground) brute force, the rest
 * through a BVH with conservative boxes and an order-independent tie rule:
 * the same closest hit, bit for bit.  rt_ctx_accel_info
 * reports the split (big spheres, BVH nodes) of the current scene.
 * RT_ACCEL_GRID: the same split, the small spheres in a uniform grid walked
 * by a 3D DDA; same closest hit bit for bit.
 * rt_ctx_grid_info reports its cells per axis, references and image bytes
 * (RT_EUNSUPPORTED when the scene has no grid — over 65 535 spheres: the
 * render then uses the BVH).  Each structure is staged in LDS per block when
 * it fits; a larger one (scenes of thousands of spheres) is walked in global
 * memory — the same hits. */
enum { RT_ACCEL_NONE = 0, RT_ACCEL_BVH = 1, RT_ACCEL_GRID = 2 };
/* (a new context starts with RT_ACCEL_GRID: same image as brute force, and
 * the fastest on the reference's scenes — DESIGN.md §4.4) */

/* Dispatch order.  RT_ORDER_COST (default): every render counts world.hit
 * calls per tile and dispatches its tiles most-expensive-first (a GPU radix
 * sort of per-tile counts), so the end of the launch is cheap work.  The
 * counts come from the previous render with the same tile layout, or — when
 * there is none (a one-shot render) — from a probe pass of 1 sample per
 * pixel with paths cut at depth 8, run first on the same stream (under 1/500
 * of the work).  RT_ORDER_NONE:
 * tiles in image order.  Never changes the image. */
enum { RT_ORDER_NONE = 0, RT_ORDER_COST = 1 };
int rt_ctx_set_ordering(rt_ctx *ctx, int32_t ordering);
int rt_ctx_set_accel(rt_ctx *ctx, int32_t accel);
int rt_ctx_accel_info(rt_ctx *ctx, int32_t *n_big, int32_t *n_nodes);
int rt_ctx_grid_info(rt_ctx *ctx, int32_t *dims3, int32_t *n_refs, int32_t *lds_bytes);

/* The whole image: replaces the 16-thread worker() block main.cpp:313-338.
 * Synchronous; `sum` is a HOST buffer of W*H*3 floats.  max_depth is in
 * [0, 2^24) (RT_EINVAL otherwise; the reference's recursion would exhaust its
 * stack long before). */
int rt_render(rt_ctx *ctx, const rt_camera *cam, int32_t W, int32_t H, int32_t spp,
              int32_t max_depth, uint64_t seed, float *sum);

/* Rows row0, row0+row_step, ..., (nrows of them) into a DEVICE strip buffer
 * dev_strip[nrows*W*3] (strip row r = image row row0 + r*row_step; rows past
 * H are zero-filled).  Asynchronous on `stream` (hipStream_t; NULL = the
 * context's stream).  This is the per-GPU unit of the multi-GPU row
 * partition.  dev_strip must stay valid until the stream
 * reaches the end of this call's work. */
int rt_render_rows(rt_ctx *ctx, const rt_camera *cam, int32_t W, int32_t H, int32_t spp,
                   int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step,
                   int32_t nrows, float *dev_strip, void *stream);
/* Number of world.hit calls (path segments) of the context's
 * last render, counted on the GPU; waits for that render to finish.  The
 * algorithmic work of a render is segments * 18 * n_spheres FLOP. */
int rt_ctx_last_segments(rt_ctx *ctx, uint64_t *segments);
/* Diagnostic: the schedule of the context's last launch (not its probe):
 * {tile width, samples per item, items per tile, tail items per tile,
 *  block flush (2: the block owns its tile and writes the floats), block
 *  pool, persistent kernel, accelerator (0 none, 1 BVH, 2 grid)}. */
int rt_ctx_last_schedule(rt_ctx *ctx, int32_t *out8);
/* Block until the context's stream is idle. */
int rt_ctx_synchronize(rt_ctx *ctx);

/* Progressive accumulation (resumable).  The context
 * keeps a fixed-point accumulator for a W x nrows strip (the rows of
 * rt_render_rows' row set; nrows = H, row0 0, row_step 1 for a whole image).
 * rt_render_pass adds samples [s_begin, s_begin + s_count) of every pixel;
 * any split of [0, S) into passes, in any order, gives bit for bit the sums
 * of one rt_render(..., spp = S, ...).  rt_accum_resolve converts the sums
 * to floats into a DEVICE strip and/or a HOST buffer (W*nrows*3).
 * rt_accum_export / rt_accum_import copy the raw int64 accumulator and its
 * sample count out / in (checkpoint and resume, across processes). */
int rt_accum_reset(rt_ctx *ctx, int32_t W, int32_t nrows);
int rt_render_pass(rt_ctx *ctx, const rt_camera *cam, int32_t W, int32_t H, int32_t s_begin,
                   int32_t s_count, int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step,
                   int32_t nrows, void *stream);
int rt_accum_resolve(rt_ctx *ctx, float *dev_sum, float *host_sum, void *stream);
int rt_accum_export(rt_ctx *ctx, int64_t *host, size_t n, int32_t *spp_done);
int rt_accum_import(rt_ctx *ctx, const int64_t *host, size_t n, int32_t spp_done);
/* Checkpoint files: the accumulator plus what it was rendered from (size,
 * row set, depth, seed, hashes of the scene and camera).  rt_accum_save
 * writes atomically (tmp + rename); rt_accum_load resets the accumulator to
 * W x nrows, refuses (RT_EINVAL) a file made for another render, and sets
 * *spp_done to the samples already in it. */
int rt_accum_save(rt_ctx *ctx, const char *path, const rt_scene *scene, const rt_camera *cam,
                  int32_t H, int32_t row0, int32_t row_step, int32_t max_depth, uint64_t seed);
int rt_accum_load(rt_ctx *ctx, const char *path, const rt_scene *scene, const rt_camera *cam,
                  int32_t W, int32_t H, int32_t row0, int32_t row_step, int32_t nrows,
                  int32_t max_depth, uint64_t seed, int32_t *spp_done);

/* Exact replay (validation): runs n_jobs reference worker(start, end, ...)
 * calls (main.cpp:267-290) on the GPU in DOUBLE with the reference's op
 * order, consuming for job k the supplied glibc rand() values
 * streams[stream_offsets[k] .. stream_offsets[k+1]) in place of rand().
 * job_ranges = {start0, end0, start1, end1, ...}; host_sums receives
 * Σ(end-start)*3 doubles in job order; draws_used[k] = values consumed.
 * max_depth <= 64.  RT_ESTREAM if a job runs out of stream values. */
int rt_replay_worker(rt_ctx *ctx, const rt_camera *cam, int32_t W, int32_t H, int32_t spp,
                     int32_t max_depth, int32_t n_jobs, const int32_t *job_ranges,
                     const int32_t *streams, const int64_t *stream_offsets, double *host_sums,
                     int64_t *draws_used);

/* Multi-GPU render in one process (the C++ drop-in path): rows interleaved
 * over n_gpus devices (row j -> device j % n_gpus), one RCCL gather of the
 * per-device strips to device 0 over xGMI, un-permuted into `sum` (HOST,
 * W*H*3).  n_gpus = 0 means all visible devices.  Same image as rt_render. */
int rt_render_multi(const rt_scene *scene, const rt_camera *cam, int32_t W, int32_t H,
                    int32_t spp, int32_t max_depth, uint64_t seed, int32_t n_gpus, float *sum);

/* The same with everything kept across renders: rt_multi_create makes one
 * context per device 0..n_gpus-1 (0 = all visible; RT_ENODEVICE if more are
 * asked than visible) with the scene resident, and the RCCL communicator
 * (ncclCommInitAll) once; rt_multi_render reuses them (strips and the gather
 * buffer grow as needed).  rt_multi_last_timing reports the last render's
 * per-device strip time (HIP events around each device's rt_render_rows,
 * strip_ms[n_gpus]) and the gather alone (device 0 waits for every strip
 * before the gather's start event), in ms.  Progressive passes on N GPUs:
 * rt_multi_accum_reset(W, H), any number of rt_multi_render_pass over
 * sample ranges (each device adds its rows' samples to its own fixed-point
 * accumulator), then rt_multi_accum_resolve gathers the sums (same bits as
 * one rt_render of the covered samples).  rt_multi_context exposes device
 * g's context (tuning, accelerator, counters).
 * Errors: a call that fails after enqueuing work on some devices waits for
 * every device's stream before it returns; a failed rt_multi_render_pass (or
 * rt_multi_accum_reset) leaves the device set without a valid accumulator
 * (the devices' sums would cover different samples): rt_multi_render_pass and
 * rt_multi_accum_resolve return RT_EINVAL until the next successful
 * rt_multi_accum_reset. */
typedef struct rt_multi rt_multi;
int rt_multi_create(const rt_scene *scene, int32_t n_gpus, rt_multi **out);
int rt_multi_destroy(rt_multi *m);
int rt_multi_device_count(rt_multi *m, int32_t *n);
int rt_multi_context(rt_multi *m, int32_t g, rt_ctx **ctx);
int rt_multi_render(rt_multi *m, const rt_camera *cam, int32_t W, int32_t H, int32_t spp,
                    int32_t max_depth, uint64_t seed, float *sum);
int rt_multi_last_timing(rt_multi *m, float *strip_ms, float *gather_ms);
int rt_multi_accum_reset(rt_multi *m, int32_t W, int32_t H);
int rt_multi_render_pass(rt_multi *m, const rt_camera *cam, int32_t s_begin, int32_t s_count,
                         int32_t max_depth, uint64_t seed);
int rt_multi_accum_resolve(rt_multi *m, float *sum);

/* Host helper (no GPU): the row partition's inverse.  strips holds n_strips
 * strips of nrows x W x 3 floats; strip g holds image rows g, g + n_strips,
 * g + 2*n_strips, ... (rt_render_rows with row0 = g, row_step = n_strips),
 * rows >= H being padding.  Writes the H x W x 3 image.  RT_EINVAL when
 * n_strips * nrows < H. */
int rt_unpermute_rows(const float *strips, int32_t n_strips, int32_t nrows, int32_t W, int32_t H,
                      float *image);

#ifdef __cplusplus
}
#endif
#endif /* RTMI_H */
