/* include/rtmi_nw.h — C ABI of librtmi's Next-Week renderer (SURVEY §8(f)
 * rank 4): the scene vocabulary of the reference's rt_next_week/cuda/ —
 * textures (texture.h, perlin.h), materials incl. emission and isotropic
 * phase (material.h), spheres and moving spheres (sphere.h, moving_sphere.h),
 * axis-aligned rectangles and boxes (aarect.h, box.h), instances
 * (translate / rotate_y, hittable.h:49-191), participating media
 * (constant_medium.h), a background colour and emission-aware path
 * integration (get_color, main.cu:47-101) — rendered by gfx950 kernels in
 * the same wave-queue / fixed-point design as the RTIOW path.
 *
 * The reference builds its scenes with `new` on the device and renders them
 * through virtual hit()/scatter() calls.  Here the caller builds a host-side
 * scene with the calls below (one per reference constructor); the library
 * flattens it — every leaf primitive carrying its composed rotate_y +
 * translate instance — builds a BVH and uploads it.
 *
 * Conventions are those of rtmi.h: RT_OK / negative RT_E* returns (builders
 * return the new handle, >= 0, or a negative RT_E*), rt_last_error(), no
 * CPU fallback, per-pixel colour SUMS with row 0 at the bottom.  Differences
 * from the reference's semantics are listed in DESIGN.md §9.
 */
#ifndef RTMI_NW_H
#define RTMI_NW_H

#include "rtmi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_nw_scene rt_nw_scene; /* host-side scene under construction */
typedef struct rt_nw_ctx rt_nw_ctx;     /* one device, its stream, the resident scene */

/* camera.h:24-83 (Next-Week camera: shutter interval [time0, time1]) */
typedef struct rt_nw_camera {
  rt_camera cam;
  double time0, time1;
} rt_nw_camera;

/* camera::camera(lookfrom, lookat, vup, vfov, aspect, aperture, focal_dist,
 * time0, time1) camera.h:24-62, evaluated in double, rounded to float on use. */
int rt_nw_camera_init(rt_nw_camera *cam, const double lookfrom[3], const double lookat[3],
                      const double vup[3], double vfov_deg, double aspect_ratio, double aperture,
                      double focus_dist, double time0, double time1);

int rt_nw_scene_create(rt_nw_scene **out);
int rt_nw_scene_destroy(rt_nw_scene *s);

/* ---- textures (texture.h) ---------------------------------------------- */
int rt_nw_tex_solid(rt_nw_scene *s, double r, double g, double b);        /* solid_color      */
int rt_nw_tex_checker(rt_nw_scene *s, int32_t even, int32_t odd);          /* checker_texture  */
/* noise_texture(scale) over a perlin table: ranvec[256*3] (xyz per entry)
 * and perm[3*256] (perm_x, perm_y, perm_z), perlin.h:8-21. */
int rt_nw_tex_noise(rt_nw_scene *s, double scale, const float *ranvec, const int32_t *perm);
/* image_texture(data, w, h) texture.h:84-124: rgb bytes, w*h*3, row 0 at the
 * top (stb_image order); copied.  data == NULL renders cyan (texture.h:96). */
int rt_nw_tex_image(rt_nw_scene *s, const uint8_t *rgb, int32_t w, int32_t h);

/* ---- materials (material.h) -------------------------------------------- */
enum { RT_NW_LAMBERTIAN = 0, RT_NW_METAL = 1, RT_NW_DIELECTRIC = 2, RT_NW_DIFFUSE_LIGHT = 3, RT_NW_ISOTROPIC = 4 };
int rt_nw_mat_lambertian(rt_nw_scene *s, int32_t tex);
int rt_nw_mat_metal(rt_nw_scene *s, int32_t tex, double fuzz); /* fuzz clamped to <= 1 (material.h:58-62) */
int rt_nw_mat_dielectric(rt_nw_scene *s, double ir);
int rt_nw_mat_diffuse_light(rt_nw_scene *s, int32_t tex);
int rt_nw_mat_isotropic(rt_nw_scene *s, int32_t tex);

/* ---- objects (handles; an object is rendered once added to the world) --- */
enum { RT_NW_XY = 0, RT_NW_XZ = 1, RT_NW_YZ = 2 };
int rt_nw_sphere(rt_nw_scene *s, const double center[3], double radius, int32_t mat);
int rt_nw_moving_sphere(rt_nw_scene *s, const double center0[3], const double center1[3], double time0,
                        double time1, double radius, int32_t mat);
/* xy_rect(a0,a1,b0,b1,k) etc. aarect.h: (a, b) are the in-plane axes in
 * order (xy: x,y; xz: x,z; yz: y,z), k the plane coordinate. */
int rt_nw_rect(rt_nw_scene *s, int32_t plane, double a0, double a1, double b0, double b1, double k, int32_t mat);
int rt_nw_box(rt_nw_scene *s, const double p0[3], const double p1[3], int32_t mat);
/* constant_medium(boundary, density, tex) constant_medium.h: boundary is a
 * sphere, moving sphere or box object, optionally under translate/rotate_y. */
int rt_nw_constant_medium(rt_nw_scene *s, int32_t boundary, double density, int32_t tex);
/* Scattering-distance samples of a medium per ray segment (1..8, default 1):
 * each draws -log(u)/density anew and the last one that lands inside the
 * boundary wins — what the reference's bvh_node does to a medium alone in a
 * span-1 leaf, which it evaluates twice (bvh.h:90-97, 147-151).
 * Media are resolved before the other objects of a segment, and a medium's
 * hit hides its own boundary object when that is in the world too (the
 * reference visits constant_medium after its boundary, main.cu:386-391, and
 * constant_medium::hit ignores t_max).  DESIGN.md §9. */
int rt_nw_medium_samples(rt_nw_scene *s, int32_t medium, int32_t samples);
/* hittable_list / bvh_node of objects (one handle for the set). */
int rt_nw_group(rt_nw_scene *s, const int32_t *objects, int32_t n);
int rt_nw_translate(rt_nw_scene *s, int32_t object, const double offset[3]); /* hittable.h:49-88  */
int rt_nw_rotate_y(rt_nw_scene *s, int32_t object, double angle_deg);       /* hittable.h:90-189 */
int rt_nw_world_add(rt_nw_scene *s, int32_t object);
int rt_nw_set_background(rt_nw_scene *s, double r, double g, double b);

/* The reference's scenes, create_world main.cu:415-490 (`which` = its switch
 * case: 1 random_scene, 2 two_spheres, 3 two_perlin_spheres, 4 earth,
 * 5 simple_light, 6 cornell_box, 7 cornell_smoke, 8 rt_next_week_final_scene).
 * Random draws come from a restatement of curand XORWOW seeded as the
 * reference seeds it (curand_init(1984, 0, 0), main.cu:103-107).  `image`
 * (w*h*3 bytes, may be NULL) is the earth texture.  Writes the camera the
 * reference uses for that scene at `aspect` (main.cu:486-489).  flags bit 0:
 * evaluate the three draws of vec3(rnd, rnd, rnd) right to left (argument
 * evaluation order is unspecified in C++; default left to right). */
enum { RT_NW_ARGS_RTL = 1 };
int rt_nw_scene_preset(rt_nw_scene *s, int32_t which, const uint8_t *image, int32_t w, int32_t h,
                       double aspect, uint32_t flags, rt_nw_camera *cam);

/* curand XORWOW restated (curand_init(seed, 0, 0) then curand_uniform):
 * n uniforms in (0, 1].  Validation of the scene generator. */
int rt_nw_xorwow_uniforms(uint64_t seed, int32_t n, float *out);

/* Flattened view of a scene (what the device renders), for tests and the
 * oracle.  Pointers stay valid until the scene is modified or destroyed.
 *   obj  : n_obj * 16 floats: g0[4] g1[4] g2[4] then kind, mat, inst, aux as
 *          int32 bit patterns (layout: DESIGN.md §9; aux: medium -> boundary
 *          kind | samples << 8, other -> insertion index of the medium whose
 *          boundary it is + 1, or 0)
 *   inst : n_inst * 8 floats: cos, sin, off.x, off.y, off.z, flags(int bits), 0, 0
 *   mat  : n_mat * 4: kind(int bits), tex(int bits), fuzz, ir
 *   tex  : n_tex * 8: kind, a, b, 0 (int bits), r, g, b, scale
 *   perlin_vec : n_perlin * 256 * 4 floats; perlin_perm : n_perlin * 768 int32
 *   image_px : all image bytes; image_desc : n_image * 4 int32 (offset, w, h, 0) */
typedef struct rt_nw_flat {
  int32_t n_obj, n_inst, n_mat, n_tex, n_perlin, n_image;
  const float *obj, *inst, *mat, *tex, *perlin_vec;
  const int32_t *perlin_perm, *image_desc;
  const uint8_t *image_px;
  int64_t image_bytes;
  float background[3];
} rt_nw_flat;
int rt_nw_scene_flat(rt_nw_scene *s, rt_nw_flat *out);
/* Host only (no device needed): the uniform grid rt_nw_ctx_set_scene would
 * build for this scene — cells per axis (zeros: no grid),
 * the fullest cell's object count, the brute-force list's length and the
 * total cell references.  Any output may be null. */
int rt_nw_scene_grid_stats(rt_nw_scene *s, int32_t *dims3, int32_t *max_cell, int32_t *n_big, int32_t *n_refs);

/* ---- device ------------------------------------------------------------ */
int rt_nw_ctx_create(int32_t device, rt_nw_ctx **out);
int rt_nw_ctx_destroy(rt_nw_ctx *ctx);
/* Flatten, build the BVH, upload.  Synchronous. */
int rt_nw_ctx_set_scene(rt_nw_ctx *ctx, rt_nw_scene *s);
/* n_prims, n_nodes of the resident BVH */
int rt_nw_ctx_info(rt_nw_ctx *ctx, int32_t *n_prims, int32_t *n_nodes);
/* Closest-hit structure over the non-media objects (media are always tested
 * first).  RT_NW_ACCEL_BVH: the SAH BVH (skip-link walk).
 * RT_NW_ACCEL_GRID: a uniform grid walked by a 3D DDA, objects much larger
 * than the median in a brute-force list beside it; offered
 * when the scene has one (rt_nw_ctx_accel_info).  RT_NW_ACCEL_AUTO (a new
 * context's setting): the grid when it is balanced (at most 24 objects in
 * any cell), else the BVH.  All give the same closest hit, so the same image
 * bit for bit.  Replaces the choice of hittable in main.cu:420-490 (the
 * reference always wraps the world in its bvh_node). */
enum { RT_NW_ACCEL_AUTO = 0, RT_NW_ACCEL_BVH = 1, RT_NW_ACCEL_GRID = 2 };
int rt_nw_ctx_set_accel(rt_nw_ctx *ctx, int32_t accel);
/* The structure renders use now (RT_NW_ACCEL_BVH or _GRID, after AUTO is
 * resolved); the grid's cells per axis (dims3, 0 when the scene has no grid),
 * its largest cell's object count and the brute-force list's length.  Any
 * output may be null. */
int rt_nw_ctx_accel_info(rt_nw_ctx *ctx, int32_t *accel_used, int32_t *dims3, int32_t *max_cell, int32_t *n_big);
/* The whole image (main.cu:125-145 + the caller's output loop), host sums,
 * synchronous.  Pixel (i, j) samples u = (i + r)/W, v = (j + r)/H
 * (main.cu:139-140). */
int rt_nw_render(rt_nw_ctx *ctx, const rt_nw_camera *cam, int32_t W, int32_t H, int32_t spp, int32_t max_depth,
                 uint64_t seed, float *sum);
/* Rows row0 + r*row_step, r < nrows, into a DEVICE strip (as rt_render_rows). */
int rt_nw_render_rows(rt_nw_ctx *ctx, const rt_nw_camera *cam, int32_t W, int32_t H, int32_t spp,
                      int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step, int32_t nrows,
                      float *dev_strip, void *stream);
/* Debug (parity investigations): the path segments of ONE camera sample
 * (pixel i, j, sample s), up to cap: per segment 12 floats o.xyz, d.xyz, t,
 * the winner's insertion index (int32 bits, -1: miss), its hit-record normal
 * xyz and the box face (int32 bits, -1: none).  *n = segments. */
int rt_nw_debug_trace(rt_nw_ctx *ctx, const rt_nw_camera *cam, int32_t W, int32_t H, int32_t max_depth,
                      uint64_t seed, int32_t i, int32_t j, int32_t s, float *rec, int32_t cap, int32_t *n);
/* Validation: the closest hit of n given rays through the walk a render of
 * this context uses (the uniform grid or the BVH: rt_nw_ctx_accel_info) —
 * rays {o.xyz, d.xyz, time, unused} per ray (8 floats), keys the segments'
 * medium keys (null: 0).  Out: the winner's insertion index (-1: miss), t
 * and the box face (-1: none), as one segment of rt_nw_debug_trace. */
int rt_nw_debug_hits(rt_nw_ctx *ctx, const float *rays, const uint64_t *keys, int32_t n, int32_t *out_id, float *out_t,
                     int32_t *out_face);
/* world.hit calls of the last render (waits for it). */
int rt_nw_ctx_last_segments(rt_nw_ctx *ctx, uint64_t *segments);
/* Diagnostic: the kernel of the last render, {persistent, uniform grid,
 * spheres-only instantiation (spheres and moving spheres, no instances or
 * media, solid / checker textures: the other kinds' code compiled out),
 * samples per work item}.  Same image for every choice. */
int rt_nw_ctx_last_kernel(rt_nw_ctx *ctx, int32_t *out4);
/* Analysis builds only (-DRTMI_NW_PHASES=1): wave-level cycles of the loop
 * passes since the last call — closest hit, hit record + texture + scatter,
 * accumulation + regeneration, whole items; RT_EUNSUPPORTED otherwise. */
int rt_nw_debug_phases(uint64_t *out4);
/* Analysis: the executed work of the launches since the last call, counted
 * per lane by the RTMI_STATS build (librtmi_stats.so): {algorithmic FLOP of
 * the miss tests performed (per-kind counts as bench.py NW_FLOP) + 25 per
 * node slab test / grid clip + 5 per cell step, node visits, object tests,
 * cell steps}; zeroed after reading.  RT_EUNSUPPORTED in the product build. */
int rt_nw_debug_counters(uint64_t *out4);

#ifdef __cplusplus
}
#endif
#endif /* RTMI_NW_H */
