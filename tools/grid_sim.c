/* tools/grid_sim.c — CPU model of the uniform-grid walk's SIMD efficiency on
 * the final scene, and of regrouping rays across a block's waves.
 *
 * Analysis only (not product, not oracle).  Traces an approximate path
 * distribution over the fixture scene (as tools/bvh_sim.c: camera rays, then
 * lambertian / metal / dielectric bounces, brute-force closest hit in double),
 * records every segment, and replays the segments through the grid walk of
 * hit_world_grid (big spheres first for t_max, clip to the grid box, 3D DDA,
 * stop at the first cell whose exit is >= t_max) in 64-lane lockstep groups.
 * A wave pays for its longest walk: per wave the cell iterations are the max
 * over lanes of the cells walked, the sphere iterations the sum over cell
 * steps of the max over lanes of that cell's list length.
 *
 * Groupings of a tile's (shuffled) segments into waves:
 *   shuffled  64 consecutive segments (path regeneration mixes depths: the kernel today)
 *   block/K   256 consecutive segments (a 4-wave block) sorted by key K, then cut into 4 waves
 *   ideal/K   all of the tile's segments sorted by key K (an upper bound on any regrouping)
 * keys: oct = direction octant; cell = entry cell; oct+cell; len = the walk's own cell count (oracle)
 *
 * Also (round 3): the walk split by primary (camera) and secondary segments;
 * per sphere iteration whether any lane has a candidate (disc >= 0) and
 * whether any lane accepts a root (what a sqrt-free reject filter could skip
 * at wave level); and a "flattened" schedule testing the round's (lane,
 * sphere) pairs over all 64 lanes.
 *
 *   gcc -O2 -o /tmp/grid_sim tools/grid_sim.c -lm && /tmp/grid_sim tests/golden/scene_final.txt [spp] [stride]
 *   (BEHIND_CULL=1: candidates without the spheres a ray leaves from outside, as RTMI_BEHIND_CULL)
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MAXS 1024
static int g_behind_cull;
static int N;
static double C[MAXS][4];
static int KIND[MAXS];
static double MAT[MAXS][4];

static unsigned long long rs = 88172645463325252ull;
static double rnd(void) {
  rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
  return (rs >> 11) * (1.0 / 9007199254740992.0);
}

typedef struct { double o[3], d[3]; int depth, path; } Ray;
static unsigned long long *g_cand, *g_use;
static Ray *segs; static int nseg, capseg, cur_depth, cur_path;
static int *tile_start; static int ntiles, captiles;

static int hit_bf(const double o[3], const double d[3], double *tt) {
  double tmax = INFINITY; int best = -1;
  double a = d[0]*d[0]+d[1]*d[1]+d[2]*d[2];
  for (int k = 0; k < N; k++) {
    double oc[3] = {o[0]-C[k][0], o[1]-C[k][1], o[2]-C[k][2]};
    double hb = oc[0]*d[0]+oc[1]*d[1]+oc[2]*d[2];
    double c = oc[0]*oc[0]+oc[1]*oc[1]+oc[2]*oc[2]-C[k][3]*C[k][3];
    double disc = hb*hb - a*c;
    if (disc < 0) continue;
    double sq = sqrt(disc), r = (-hb - sq)/a;
    if (r < 0.001 || r > tmax) { r = (-hb + sq)/a; if (r < 0.001 || r > tmax) continue; }
    tmax = r; best = k;
  }
  *tt = tmax; return best;
}

static void rand_unit(double v[3]) {
  double z = 1 - 2*rnd(), ph = 2*M_PI*rnd(), s = sqrt(1 - z*z);
  v[0] = s*cos(ph); v[1] = s*sin(ph); v[2] = z;
}

static void push(const double o[3], const double d[3]) {
  if (nseg == capseg) { capseg = capseg ? 2*capseg : 1<<20; segs = realloc(segs, capseg*sizeof(Ray)); }
  memcpy(segs[nseg].o, o, 24); memcpy(segs[nseg].d, d, 24); segs[nseg].depth = cur_depth; segs[nseg].path = cur_path; nseg++;
}

/* ---- grid (build_grid's shape: small spheres, margin-grown boxes, ~0.3 cells per sphere) ---- */
static int small_[MAXS], nsmall, big_[MAXS], nbig;
static double g0[3], h[3]; static int n[3];
static int *cell_start, *cell_refs;

static void build(double density) {
  double rad[MAXS]; int m = 0;
  for (int k = 0; k < N; k++) rad[m++] = fabs(C[k][3]);
  for (int i = 0; i < m; i++) for (int j = i + 1; j < m; j++) if (rad[j] < rad[i]) { double t = rad[i]; rad[i] = rad[j]; rad[j] = t; }
  double med = rad[m/2];
  nsmall = nbig = 0;
  for (int k = 0; k < N; k++) { if (fabs(C[k][3]) > 4*med) big_[nbig++] = k; else small_[nsmall++] = k; }
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = 0; i < nsmall; i++) { int k = small_[i]; double r = fabs(C[k][3]) * 1.001 + 1e-6;
    for (int a = 0; a < 3; a++) { if (C[k][a]-r < lo[a]) lo[a] = C[k][a]-r; if (C[k][a]+r > hi[a]) hi[a] = C[k][a]+r; } }
  double ext[3], vol = 1; for (int a = 0; a < 3; a++) { ext[a] = hi[a]-lo[a]; vol *= ext[a]; }
  double side = cbrt(vol / (density * nsmall));
  int tot = 1;
  for (int a = 0; a < 3; a++) { n[a] = (int)floor(ext[a]/side + 0.5); if (n[a] < 1) n[a] = 1; if (n[a] > 64) n[a] = 64; g0[a] = lo[a]; h[a] = ext[a]/n[a]; tot *= n[a]; }
  int *cnt = calloc(tot + 1, sizeof(int));
  for (int pass = 0; pass < 2; pass++) {
    for (int i = 0; i < nsmall; i++) { int k = small_[i]; double r = fabs(C[k][3]) * 1.001 + 1e-6; int c0[3], c1[3];
      for (int a = 0; a < 3; a++) { c0[a] = (int)floor((C[k][a]-r-g0[a])/h[a]); c1[a] = (int)floor((C[k][a]+r-g0[a])/h[a]);
        if (c0[a] < 0) c0[a] = 0; if (c1[a] >= n[a]) c1[a] = n[a]-1; }
      for (int z = c0[2]; z <= c1[2]; z++) for (int y = c0[1]; y <= c1[1]; y++) for (int x = c0[0]; x <= c1[0]; x++) {
        int c = x + n[0]*(y + n[1]*z);
        if (pass == 0) cnt[c+1]++; else cell_refs[cnt[c]++] = k; } }
    if (pass == 0) { for (int c = 0; c < tot; c++) cnt[c+1] += cnt[c]; cell_start = malloc((tot+1)*sizeof(int));
      memcpy(cell_start, cnt, (tot+1)*sizeof(int)); cell_refs = malloc((cnt[tot] + 1)*sizeof(int)); }
  }
  printf("grid %d x %d x %d, %d small spheres, %d refs (%.2f per sphere), %d big\n", n[0], n[1], n[2], nsmall,
         cell_start[tot], (double)cell_start[tot]/nsmall, nbig);
  free(cnt);
}

/* one segment's walk: the list lengths of the cells visited (returns their count) */
static int g_pred;  /* the walk's cell-count bound known before it: |dcx|+|dcy|+|dcz|+1 (0: no walk) */
static int g_pred_nobig;  /* the same bound from the grid box alone (before the big-sphere pass) */
static int bound_of(const Ray *r, const double inv[3], double tmax) {
  double tn = 0, tf = tmax;
  for (int k = 0; k < 3; k++) { double t0 = (g0[k]-r->o[k])*inv[k], t1 = (g0[k]+n[k]*h[k]-r->o[k])*inv[k];
    if (t0 > t1) { double x = t0; t0 = t1; t1 = x; } if (t0 > tn) tn = t0; if (t1 < tf) tf = t1; }
  if (tn > tf) return 0;
  int b = 1;
  for (int k = 0; k < 3; k++) { double p0 = r->o[k] + tn*r->d[k], p1 = r->o[k] + tf*r->d[k];
    int c0 = (int)floor((p0-g0[k])/h[k]), c1 = (int)floor((p1-g0[k])/h[k]);
    if (c0 < 0) c0 = 0; if (c0 >= n[k]) c0 = n[k]-1; if (c1 < 0) c1 = 0; if (c1 >= n[k]) c1 = n[k]-1; b += abs(c1 - c0); }
  return b;
}
static int walk(const Ray *r, int *lens, int *entry_cell) {
  double a = r->d[0]*r->d[0]+r->d[1]*r->d[1]+r->d[2]*r->d[2], tmax = INFINITY;
  for (int i = 0; i < nbig; i++) { int q = big_[i];
    double oc[3] = {r->o[0]-C[q][0], r->o[1]-C[q][1], r->o[2]-C[q][2]};
    double hb = oc[0]*r->d[0]+oc[1]*r->d[1]+oc[2]*r->d[2];
    double c = oc[0]*oc[0]+oc[1]*oc[1]+oc[2]*oc[2]-C[q][3]*C[q][3];
    double disc = hb*hb - a*c; if (disc < 0) continue;
    double sq = sqrt(disc), rt = (-hb-sq)/a;
    if (rt < 0.001 || rt > tmax) { rt = (-hb+sq)/a; if (rt < 0.001 || rt > tmax) continue; }
    tmax = rt; }
  double inv[3], tn = 0, tf = tmax;
  for (int k = 0; k < 3; k++) inv[k] = 1.0 / (fabs(r->d[k]) < 1e-20 ? copysign(1e-20, r->d[k]) : r->d[k]);
  g_pred_nobig = bound_of(r, inv, INFINITY);
  for (int k = 0; k < 3; k++) {
    double t0 = (g0[k]-r->o[k])*inv[k], t1 = (g0[k]+n[k]*h[k]-r->o[k])*inv[k];
    if (t0 > t1) { double x = t0; t0 = t1; t1 = x; } if (t0 > tn) tn = t0; if (t1 < tf) tf = t1; }
  *entry_cell = -1; g_pred = 0;
  if (tn > tf) return 0;
  int c[3], step[3]; double tnext[3], dt[3];
  for (int k = 0; k < 3; k++) { double p = r->o[k] + tn*r->d[k]; c[k] = (int)floor((p-g0[k])/h[k]);
    if (c[k] < 0) c[k] = 0; if (c[k] >= n[k]) c[k] = n[k]-1;
    step[k] = r->d[k] >= 0 ? 1 : -1; dt[k] = fabs(h[k]*inv[k]);
    tnext[k] = (g0[k] + (c[k] + (step[k] > 0)) * h[k] - r->o[k]) * inv[k]; }
  *entry_cell = c[0] + n[0]*(c[1] + n[1]*c[2]);
  g_pred = 1;
  for (int k = 0; k < 3; k++) { double p = r->o[k] + tf*r->d[k]; int e = (int)floor((p-g0[k])/h[k]);
    if (e < 0) e = 0; if (e >= n[k]) e = n[k]-1; g_pred += abs(e - c[k]); }
  int nc = 0;
  for (;;) {
    int cell = c[0] + n[0]*(c[1] + n[1]*c[2]);
    lens[nc] = cell_start[cell+1] - cell_start[cell]; g_cand[nc] = 0; g_use[nc] = 0; nc++;
    /* the spheres tested here can only shrink tmax */
    for (int i = cell_start[cell]; i < cell_start[cell+1]; i++) { int q = cell_refs[i];
      double oc[3] = {r->o[0]-C[q][0], r->o[1]-C[q][1], r->o[2]-C[q][2]};
      double hb = oc[0]*r->d[0]+oc[1]*r->d[1]+oc[2]*r->d[2];
      double cc = oc[0]*oc[0]+oc[1]*oc[1]+oc[2]*oc[2]-C[q][3]*C[q][3];
      double disc = hb*hb - a*cc; if (disc < 0) continue;
      /* BEHIND_CULL=1: a sphere the ray leaves from outside (hb > 0, |oc|^2 >= r^2; the bounce origin sits on the
       * surface here, so |oc|^2 - r^2 >= -1e-9) is no candidate (the kernels' RTMI_BEHIND_CULL) */
      if (g_behind_cull && hb > 0 && cc >= -1e-9) continue;
      int pos = i - cell_start[cell]; if (pos < 64) g_cand[nc-1] |= 1ull << pos;
      double sq = sqrt(disc), rt = (-hb-sq)/a;
      if (rt < 0.001 || rt > tmax) { rt = (-hb+sq)/a; if (rt < 0.001 || rt > tmax) continue; }
      if (pos < 64) g_use[nc-1] |= 1ull << pos;
      tmax = rt; }
    int k = tnext[0] <= tnext[1] && tnext[0] <= tnext[2] ? 0 : (tnext[1] <= tnext[2] ? 1 : 2);
    if (!(tnext[k] < tmax)) break;
    c[k] += step[k];
    if (c[k] < 0 || c[k] >= n[k]) break;
    tnext[k] += dt[k];
  }
  return nc;
}

typedef struct { int nc, oct, cell, pred, pnb, lens[128]; unsigned long long cand[128], use[128]; } Walk;
static Walk *W;
static int key_mode;
static int key_of(const Walk *w) {
  switch (key_mode) {
    case 0: return w->oct;
    case 1: return w->cell;
    case 2: return w->oct * 100000 + w->cell + 1;
    case 3: return w->nc;
    case 4: return w->pred;
    case 5: return w->pred > 15 ? 15 : w->pred;
    default: return w->pnb;
  }
}
static int cmpk(const void *x, const void *y) {
  int a = key_of(&W[*(const int *)x]), b = key_of(&W[*(const int *)y]);
  return a < b ? -1 : a > b;
}

typedef struct { double lane_cells, lane_spheres, wave_cells, wave_spheres, waves; } Acc;
static void wave_cost(const int *ids, int nl, Acc *acc) {
  int maxc = 0;
  for (int l = 0; l < nl; l++) { const Walk *w = &W[ids[l]]; if (w->nc > maxc) maxc = w->nc;
    acc->lane_cells += w->nc; for (int i = 0; i < w->nc; i++) acc->lane_spheres += w->lens[i]; }
  acc->wave_cells += maxc;
  for (int s = 0; s < maxc; s++) { int m = 0; for (int l = 0; l < nl; l++) { const Walk *w = &W[ids[l]]; if (s < w->nc && w->lens[s] > m) m = w->lens[s]; } acc->wave_spheres += m; }
  acc->waves++;
}

/* the walk as ONE loop whose iteration is either a cell step or one sphere of
 * the current cell, per lane (the "if-if" form): iterations where some lane
 * tests a sphere (ns), where some lane steps a cell (nc), and in total (nt) */
static double u_ns, u_nc, u_nt;
static void unified_cost(const int *ids, int nl) {
  int pos[64] = {0}, cell[64] = {0}, left[64];
  for (int l = 0; l < nl; l++) left[l] = -1;  /* -1: the next event is a cell step */
  for (;;) {
    int any = 0, s = 0, c = 0;
    for (int l = 0; l < nl; l++) {
      const Walk *w = &W[ids[l]];
      if (left[l] > 0) { left[l]--; s = 1; any = 1; continue; }
      if (cell[l] < w->nc) { left[l] = w->lens[cell[l]]; cell[l]++; c = 1; any = 1; continue; }
    }
    (void)pos;
    if (!any) break;
    u_ns += s; u_nc += c; u_nt += 1;
  }
}


/* Early-exit walks: per pass, lanes without a walk start one (segment setup:
 * big spheres + clip), the walk loop runs while more than `thr` lanes are
 * still walking (a lane's walk state survives the pass), then the lanes whose
 * walk ended are shaded.  Cost per pass from the kernel's phase split
 * (per wave-segment, round 3): setup 0.17, shading + regeneration 0.49 when
 * any lane needs it, a cell iteration 0.0265 and a sphere iteration 0.0204
 * (3.76 x 0.0265 + 10.78 x 0.0204 = the walk's 0.32).  Lanes draw segments
 * from the shuffled stream; returns cost per segment relative to thr = 0. */
static double early_exit(int thr) {
  const double S = getenv("SIM_S") ? atof(getenv("SIM_S")) : 0.17, R = getenv("SIM_R") ? atof(getenv("SIM_R")) : 0.49;
  const double wk = getenv("SIM_W") ? atof(getenv("SIM_W")) / 0.32 : 1.0, CC = 0.0265 * wk, CS = 0.0204 * wk;
  double cost = 0, segs_done = 0;
  for (int w0 = 0; w0 + 64 * 64 <= nseg; w0 += 64 * 64) {   /* one wave: 64 lanes, 64 segments each */
    int next[64], cell[64], left[64], walking[64], done_n[64];
    for (int l = 0; l < 64; l++) { next[l] = w0 + l * 64; done_n[l] = 0; walking[l] = 0; cell[l] = 0; left[l] = 0; }
    int live = 64;
    while (live) {
      /* setup for lanes without a walk */
      int any_setup = 0;
      for (int l = 0; l < 64; l++) if (!walking[l] && done_n[l] < 64) { walking[l] = 1; cell[l] = 0; left[l] = -1; any_setup = 1; }
      if (any_setup) cost += S;
      /* walk loop: lockstep cell steps (each a cell iteration, then that cell's spheres) */
      for (;;) {
        int nwalk = 0;
        for (int l = 0; l < 64; l++) if (walking[l] && done_n[l] < 64) {
          const Walk *w = &W[next[l]];
          if (cell[l] < w->nc) nwalk++; }
        if (nwalk == 0 || (nwalk <= thr && nwalk < live)) break;
        int maxlen = 0;
        for (int l = 0; l < 64; l++) if (walking[l] && done_n[l] < 64) {
          const Walk *w = &W[next[l]];
          if (cell[l] < w->nc) { if (w->lens[cell[l]] > maxlen) maxlen = w->lens[cell[l]]; cell[l]++; } }
        cost += CC + maxlen * CS;
      }
      /* shade the lanes whose walk ended */
      int any_ready = 0;
      for (int l = 0; l < 64; l++) if (walking[l] && done_n[l] < 64) {
        const Walk *w = &W[next[l]];
        if (cell[l] >= w->nc) { walking[l] = 0; next[l]++; done_n[l]++; segs_done++; any_ready = 1; if (done_n[l] == 64) live--; } }
      if (any_ready) cost += R;
    }
  }
  return cost * 64 / segs_done;   /* per wave-segment, as the phase split */
}

static void report(const char *name, const Acc *a) {
  printf("  %-14s lane cells %5.3f spheres %5.3f | wave cells %5.3f spheres %6.3f | util cells %.3f spheres %.3f\n", name,
         a->lane_cells / nseg, a->lane_spheres / nseg, a->wave_cells * 64 / nseg, a->wave_spheres * 64 / nseg,
         a->lane_cells / (64 * a->wave_cells), a->lane_spheres / (64 * a->wave_spheres));
}

/* Instruction-cost model of the walk (round 4), from the ISA of
 * render_kernel<8, true, 3> (make -C a_dive_into_ray_tracing_amd/csrc asm):
 * a cell iteration ~30 instructions (range read, the select step, loop
 * masks), a sphere iteration ~14 (reference + record reads, 8 FMAs, compare,
 * mask) and a root resolution ~33 more whenever any lane of the wave has a
 * candidate there.  A pass costs ~850 VALU wave-instructions in all (1.78e10
 * per config-2 launch over ~2.1e7 wave-passes), so ~400 outside the walk. */
static double CI_CELL = 30, CI_SPH = 14, CI_RES = 33, CI_REST = 400;
static double walk_instr(const int *ids, int nl, double *wave_time) {
  int maxc = 0;
  for (int l = 0; l < nl; l++) if (W[ids[l]].nc > maxc) maxc = W[ids[l]].nc;
  double c = 0;
  for (int s = 0; s < maxc; s++) {
    int m = 0;
    for (int l = 0; l < nl; l++) { const Walk *w = &W[ids[l]]; if (s < w->nc && w->lens[s] > m) m = w->lens[s]; }
    c += CI_CELL + m * CI_SPH;
    for (int k = 0; k < m; k++) {
      int any = 0;
      for (int l = 0; l < nl && !any; l++) { const Walk *w = &W[ids[l]]; if (s < w->nc && k < w->lens[s] && ((w->cand[s] >> k) & 1)) any = 1; }
      c += any ? CI_RES : 0;
    }
  }
  if (wave_time) *wave_time = c;
  return c;
}

/* Regrouping a block's rays by the walk-length bound before the walk
 * (VERDICT r03 item 1), charged honestly: per wave-pass the rest of the pass
 * (CI_REST), the walk of the rays the wave holds after the sort, and the
 * exchange E (key from the exit cell, per-bin ballots and the block prefix,
 * the ray state through LDS and back, three barriers).  Rays with bound 0
 * (no walk) are not exchanged.  Also the barrier idle time: in a block pass
 * every wave waits at the walk's closing barrier for the block's longest walk
 * (sum over waves of max - own), which only other blocks' waves can fill. */
static void regroup_cost(int block, double E) {
  double base = 0, regroup = 0, idle = 0, passes = 0, wbase = 0, wreg = 0;
  int *ids = malloc(block * sizeof(int)), *walkers = malloc(block * sizeof(int));
  for (int t = 0; t < ntiles; t++)
    for (int i = tile_start[t]; i + block <= tile_start[t + 1]; i += block) {
      for (int w = 0; w < block; w += 64) {  /* today: each wave its own 64 rays */
        for (int l = 0; l < 64; l++) ids[l] = i + w + l;
        const double c = walk_instr(ids, 64, NULL);
        base += CI_REST + c; wbase += c; passes += 1;
      }
      int nw = 0;
      for (int l = 0; l < block; l++) if (W[i + l].pred > 0) walkers[nw++] = i + l;
      key_mode = 4;
      qsort(walkers, nw, sizeof(int), cmpk);
      double mx = 0, sum = 0;
      for (int w = 0; w < block; w += 64) {
        double c = 0;
        if (w < nw) walk_instr(walkers + w, nw - w < 64 ? nw - w : 64, &c);
        regroup += CI_REST + E + c; wreg += c; sum += c; if (c > mx) mx = c;
      }
      idle += (block / 64) * mx - sum;
    }
  printf("  regroup %4d rays, exchange %3.0f instr/wave-pass: walk %.1f -> %.1f instr/wave-pass (%.3f), pass %.1f -> %.1f "
         "(net %+.1f%%), barrier idle %.1f per wave-pass (%.1f%% of the new pass)\n", block, E, wbase / passes, wreg / passes,
         wreg / wbase, base / passes, regroup / passes, 100 * (regroup / base - 1), idle / passes, 100 * idle / regroup);
  free(ids); free(walkers);
}

/* The barrier-free LDS ray queue, modelled.  A
 * CU-resident block keeps a pool of P waiting rays in LDS, binned by the
 * pre-walk bound (min(bound, NB-1); bound 0 = no walk).  A wave pops 64 rays
 * from the fullest bin (topped up from the next fullest when it has fewer),
 * runs one segment of each (big spheres are done at push time, so the walk
 * and shading follow at once), and pushes the survivors back by the bound of
 * their next segment; an ended path is replaced by the next camera ray of
 * the block's work, pushed by its first segment's bound.  No wave waits for
 * another: the pool is the only coupling.  Paths are replayed in generation
 * order (tile by tile, sample-major), each path's segments in depth order.
 * Cost per wave-pass: CI_REST + the walk of the popped rays + E (push: key,
 * per-bin ranking, 16 dwords of ray state written; pop: the bin claim and 16
 * dwords read).  Baseline: today's 64 consecutive segments of the shuffled
 * stream per wave-pass. */
static int *pfirst, *plen, npaths;  /* per path: its segments' indices in depth order */
static int cmp_pd(const void *x, const void *y) {
  const Ray *a = &segs[*(const int *)x], *b = &segs[*(const int *)y];
  if (a->path != b->path) return a->path < b->path ? -1 : 1;
  return a->depth < b->depth ? -1 : a->depth > b->depth;
}
static int *pd_order;
static void build_paths(void) {
  pd_order = malloc(nseg * sizeof(int));
  for (int i = 0; i < nseg; i++) pd_order[i] = i;
  qsort(pd_order, nseg, sizeof(int), cmp_pd);
  int maxp = 0; for (int i = 0; i < nseg; i++) if (segs[i].path > maxp) maxp = segs[i].path;
  npaths = maxp + 1;
  pfirst = calloc(npaths, sizeof(int)); plen = calloc(npaths, sizeof(int));
  for (int i = 0; i < nseg; i++) { int p = segs[pd_order[i]].path; if (plen[p]++ == 0) pfirst[p] = i; }
}
static int qbox;  /* 1: key on the grid-box bound alone (no big-sphere pass before the key) */
static int qkey(int seg, int NB) { int b = qbox ? W[seg].pnb : W[seg].pred; return b >= NB ? NB - 1 : b; }
static void queue_model(int P, int NB, const double *Es, int nE) {
  /* bins hold (path, segment cursor) pairs */
  int cap = P + 64, **bin = malloc(NB * sizeof(int *)), **cur = malloc(NB * sizeof(int *)), *cnt = calloc(NB, sizeof(int));
  for (int b = 0; b < NB; b++) { bin[b] = malloc(cap * sizeof(int)); cur[b] = malloc(cap * sizeof(int)); }
  int next_path = 0, pool = 0;
  Acc acc = {0}; double walk = 0, passes = 0, part = 0;
  #define QPUSH(p, c) do { int s_ = pd_order[pfirst[p] + (c)], k_ = qkey(s_, NB); bin[k_][cnt[k_]] = (p); cur[k_][cnt[k_]++] = (c); pool++; } while (0)
  while (pool < P && next_path < npaths) { QPUSH(next_path, 0); next_path++; }
  int ids[64], pp[64], pc[64];
  while (pool > 0) {
    int n = 0;
    while (n < 64 && pool > 0) {  /* the fullest bin first */
      int bb = 0; for (int b = 1; b < NB; b++) if (cnt[b] > cnt[bb]) bb = b;
      while (n < 64 && cnt[bb] > 0) { cnt[bb]--; pool--; pp[n] = bin[bb][cnt[bb]]; pc[n] = cur[bb][cnt[bb]]; n++; }
      if (pool < 64 - n && next_path >= npaths) { /* the drain: take what is there */ }
    }
    if (n < 64) part++;
    for (int l = 0; l < n; l++) ids[l] = pd_order[pfirst[pp[l]] + pc[l]];
    wave_cost(ids, n, &acc);
    walk += walk_instr(ids, n, NULL); passes++;
    for (int l = 0; l < n; l++) {
      if (pc[l] + 1 < plen[pp[l]]) QPUSH(pp[l], pc[l] + 1);
      else if (next_path < npaths) { QPUSH(next_path, 0); next_path++; }
    }
  }
  /* baseline: the shuffled stream, 64 consecutive segments per wave-pass */
  double bwalk = 0, bpass = 0;
  for (int i = 0; i < nseg; i += 64) { int nl = nseg - i < 64 ? nseg - i : 64; for (int l = 0; l < nl; l++) ids[l] = i + l; bwalk += walk_instr(ids, nl, NULL); bpass++; }
  printf("  queue P %4d bins %d: wave cells %.3f spheres %.3f per wave-seg (util %.3f / %.3f), walk %.1f -> %.1f instr/wave-pass (%.3f), part-filled pops %.4f;",
         P, NB, acc.wave_cells * 64 / nseg, acc.wave_spheres * 64 / nseg, acc.lane_cells / (64 * acc.wave_cells),
         acc.lane_spheres / (64 * acc.wave_spheres), bwalk / bpass, walk / passes, (walk / passes) / (bwalk / bpass), part / passes);
  for (int e = 0; e < nE; e++) {
    const double base = CI_REST * bpass + bwalk, q = (CI_REST + Es[e]) * passes + walk;
    printf(" E %3.0f: net %+.1f%%", Es[e], 100 * (q / base - 1));
  }
  printf("\n");
  for (int b = 0; b < NB; b++) { free(bin[b]); free(cur[b]); }
  free(bin); free(cur); free(cnt);
  #undef QPUSH
}

int main(int argc, char **argv) {
  if (getenv("BEHIND_CULL")) g_behind_cull = atoi(getenv("BEHIND_CULL"));
  FILE *f = fopen(argc > 1 ? argv[1] : "tests/golden/scene_final.txt", "r");
  if (!f || fscanf(f, "%d", &N) != 1) return 1;
  for (int k = 0; k < N; k++)
    if (fscanf(f, "%lf %lf %lf %lf %d %lf %lf %lf %lf", &C[k][0], &C[k][1], &C[k][2], &C[k][3], &KIND[k],
               &MAT[k][0], &MAT[k][1], &MAT[k][2], &MAT[k][3]) != 9) return 1;
  double org[3] = {13, 2, 3}, llc[3] = {3.0237371659391918, -1.2262841980681716, 3.4122032022021487},
         hor[3] = {1.189463936993608, 0, -5.1543437269723009}, ver[3] = {-0.50942050206062017, 3.4875711294919385, -0.11755857739860466},
         cu[3] = {0.22485950669875845, 0, -0.97439119569461996}, cv[3] = {-0.14445336159384606, 0.98894993706556156, -0.033335391137041398};
  double lens = 0.05;
  int Wd = 1200, Ht = 800, spp = argc > 2 ? atoi(argv[2]) : 16, stride = argc > 3 ? atoi(argv[3]) : 7;
  for (int ty = 0; ty < Ht/8; ty += stride) for (int tx = 0; tx < Wd/8; tx += stride) {
    if (ntiles + 1 >= captiles) { captiles = captiles ? 2*captiles : 1024; tile_start = realloc(tile_start, captiles*sizeof(int)); }
    int start = tile_start[ntiles++] = nseg;
    for (int s = 0; s < spp; s++) for (int p = 0; p < 64; p++) {
      int i = tx*8 + p%8, j = ty*8 + p/8;
      double u = (i + rnd())/(Wd-1), v = (j + rnd())/(Ht-1);
      double rr = sqrt(rnd())*lens, ph = 2*M_PI*rnd(), dx = rr*cos(ph), dy = rr*sin(ph);
      double o[3], d[3];
      for (int a = 0; a < 3; a++) { o[a] = org[a] + cu[a]*dx + cv[a]*dy; d[a] = llc[a] + u*hor[a] + v*ver[a] - o[a]; }
      for (int depth = 0; depth < 50; depth++) {
        cur_depth = depth; push(o, d);
        if (depth == 0) cur_path++;
        double t; int k = hit_bf(o, d, &t);
        if (k < 0) break;
        double pp[3], nn[3], r = C[k][3];
        for (int a = 0; a < 3; a++) { pp[a] = o[a] + t*d[a]; nn[a] = (pp[a]-C[k][a])/r; }
        double dn = d[0]*nn[0]+d[1]*nn[1]+d[2]*nn[2];
        int front = dn < 0; if (!front) for (int a = 0; a < 3; a++) nn[a] = -nn[a];
        double nd[3], ru[3]; rand_unit(ru);
        if (KIND[k] == 0) { for (int a = 0; a < 3; a++) nd[a] = nn[a] + ru[a]; }
        else if (KIND[k] == 1) {
          double dl = sqrt(d[0]*d[0]+d[1]*d[1]+d[2]*d[2]), ud[3]; for (int a = 0; a < 3; a++) ud[a] = d[a]/dl;
          double c = ud[0]*nn[0]+ud[1]*nn[1]+ud[2]*nn[2];
          for (int a = 0; a < 3; a++) nd[a] = ud[a] - 2*c*nn[a] + MAT[k][3]*ru[a]*rnd();
          if (nd[0]*nn[0]+nd[1]*nn[1]+nd[2]*nn[2] <= 0) break;
        } else {
          double dl = sqrt(d[0]*d[0]+d[1]*d[1]+d[2]*d[2]), ud[3]; for (int a = 0; a < 3; a++) ud[a] = d[a]/dl;
          double eta = front ? 1/1.5 : 1.5, c = -(ud[0]*nn[0]+ud[1]*nn[1]+ud[2]*nn[2]); if (c > 1) c = 1;
          double s2 = eta*eta*(1-c*c);
          if (s2 > 1 || rnd() < 0.05) for (int a = 0; a < 3; a++) nd[a] = ud[a] + 2*c*nn[a];
          else { double k2 = sqrt(1-s2); for (int a = 0; a < 3; a++) nd[a] = eta*ud[a] + (eta*c - k2)*nn[a]; }
        }
        double side = nd[0]*nn[0]+nd[1]*nn[1]+nd[2]*nn[2] < 0 ? -1 : 1;
        for (int a = 0; a < 3; a++) { o[a] = pp[a] + side*7e-4*nn[a]; d[a] = nd[a]; }
      }
    }
    for (int i = nseg - 1; i > start; i--) {  /* path regeneration mixes depths in a wave */
      int jx = start + (int)(rnd() * (i - start + 1));
      Ray t = segs[i]; segs[i] = segs[jx]; segs[jx] = t;
    }
  }
  tile_start[ntiles] = nseg;
  printf("segments %d in %d tiles (%d spp)\n", nseg, ntiles, spp);
  build(getenv("DENSITY") ? atof(getenv("DENSITY")) : 0.3);
  W = malloc(nseg * sizeof(Walk));
  for (int i = 0; i < nseg; i++) {
    g_cand = W[i].cand; g_use = W[i].use;
    W[i].nc = walk(&segs[i], W[i].lens, &W[i].cell);
    W[i].pred = g_pred; W[i].pnb = g_pred_nobig;
    W[i].oct = (segs[i].d[0] < 0) | ((segs[i].d[1] < 0) << 1) | ((segs[i].d[2] < 0) << 2);
  }
  int *ids = malloc(nseg * sizeof(int));
  Acc a = {0};
  for (int i = 0; i < nseg; i += 64) { int nl = nseg - i < 64 ? nseg - i : 64; for (int l = 0; l < nl; l++) ids[l] = i + l; wave_cost(ids, nl, &a); }
  report("shuffled", &a);

  { double flat = 0, mx = 0, rounds = 0;
    for (int i = 0; i < nseg; i += 64) { int nl = nseg - i < 64 ? nseg - i : 64; int maxc = 0;
      for (int l = 0; l < nl; l++) if (W[i+l].nc > maxc) maxc = W[i+l].nc;
      for (int c = 0; c < maxc; c++) { int m = 0, sum = 0; for (int l = 0; l < nl; l++) if (c < W[i+l].nc) { sum += W[i+l].lens[c]; if (W[i+l].lens[c] > m) m = W[i+l].lens[c]; }
        mx += m; flat += (sum + 63) / 64; rounds++; } }
    printf("  flattened rounds: per wave-seg rounds %.3f, sphere iterations lockstep %.3f vs flattened %.3f\n", rounds*64/nseg, mx*64/nseg, flat*64/nseg);
  }

  { double it = 0, anyc = 0, anyu = 0, lc = 0, lu = 0;
    for (int i = 0; i < nseg; i += 64) { int nl = nseg - i < 64 ? nseg - i : 64; int maxc = 0;
      for (int l = 0; l < nl; l++) if (W[i+l].nc > maxc) maxc = W[i+l].nc;
      for (int c = 0; c < maxc; c++) { int m = 0; for (int l = 0; l < nl; l++) if (c < W[i+l].nc && W[i+l].lens[c] > m) m = W[i+l].lens[c];
        for (int k = 0; k < m; k++) { int ac = 0, au = 0; it++;
          for (int l = 0; l < nl; l++) { const Walk *w = &W[i+l]; if (c < w->nc && k < w->lens[c]) {
            if ((w->cand[c] >> k) & 1) { ac = 1; lc++; } if ((w->use[c] >> k) & 1) { au = 1; lu++; } } }
          anyc += ac; anyu += au; } } }
    printf("  sphere iterations per wave-seg %.3f: any lane candidate %.3f, any lane accepted %.3f; per lane-seg candidates %.3f accepted %.3f\n",
      it*64/nseg, anyc*64/nseg, anyu*64/nseg, lc/nseg, lu/nseg);
  }

  /* Deferred root resolution (round 4): a lane keeps its first candidate of
   * a cell (hb, disc, index) and resolves it after the cell's sphere loop; a
   * second candidate in the same cell resolves the kept one in the loop
   * first.  Wave-level resolution blocks per wave-segment: today one per
   * sphere position where some lane has a candidate; deferred, one per
   * position where some lane has its 2nd+ candidate of the cell, plus one
   * per cell step where some lane kept one. */
  { double now = 0, in_loop = 0, at_end = 0;
    for (int i = 0; i < nseg; i += 64) { int nl = nseg - i < 64 ? nseg - i : 64; int maxc = 0;
      for (int l = 0; l < nl; l++) if (W[i+l].nc > maxc) maxc = W[i+l].nc;
      for (int c = 0; c < maxc; c++) {
        int m = 0; for (int l = 0; l < nl; l++) if (c < W[i+l].nc && W[i+l].lens[c] > m) m = W[i+l].lens[c];
        int seen[64] = {0}, kept = 0;
        for (int k = 0; k < m; k++) { int any = 0, second = 0;
          for (int l = 0; l < nl; l++) { const Walk *w = &W[i+l]; if (c < w->nc && k < w->lens[c] && ((w->cand[c] >> k) & 1)) {
            any = 1; if (seen[l]) second = 1; seen[l] = 1; kept = 1; } }
          now += any; in_loop += second; }
        at_end += kept; } }
    printf("  root resolutions per wave-seg: today %.3f, deferred %.3f (in the loop %.3f + after the cell %.3f)\n",
           now * 64 / nseg, (in_loop + at_end) * 64 / nseg, in_loop * 64 / nseg, at_end * 64 / nseg);
  }

  { Acc p = {0}, q = {0}, r = {0}; int np = 0;
    for (int i = 0; i < nseg; i += 64) { int nl = nseg - i < 64 ? nseg - i : 64; int ip[64], is[64], npp = 0, ns = 0;
      for (int l = 0; l < nl; l++) { if (segs[i+l].depth == 0) ip[npp++] = i + l; else is[ns++] = i + l; }
      np += npp;
      if (npp) wave_cost(ip, npp, &p);
      if (ns) wave_cost(is, ns, &q); }
    printf("  primary share %.3f\n", (double)np / nseg);
    report("primary-only", &p); report("second-only", &q);
    /* per-lane averages by kind */
    double pc=0, ps=0, sc=0, ss=0; int npr=0, nse=0;
    for (int i = 0; i < nseg; i++) { double cs = 0; for (int k = 0; k < W[i].nc; k++) cs += W[i].lens[k];
      if (segs[i].depth == 0) { pc += W[i].nc; ps += cs; npr++; } else { sc += W[i].nc; ss += cs; nse++; } }
    printf("  per-lane: primary cells %.3f spheres %.3f | secondary cells %.3f spheres %.3f\n", pc/npr, ps/npr, sc/nse, ss/nse);
    (void)r;
  }
  for (int i = 0; i < nseg; i += 64) { int nl = nseg - i < 64 ? nseg - i : 64; for (int l = 0; l < nl; l++) ids[l] = i + l; unified_cost(ids, nl); }
  printf("  one loop (if-if): iterations %.3f per wave-segment: with a sphere test %.3f, with a cell step %.3f\n",
         u_nt * 64 / nseg, u_ns * 64 / nseg, u_nc * 64 / nseg);
  {
    const double base = early_exit(0);
    printf("  early-exit walks (cost per wave-segment, thr 0 = the kernel today = %.3f):", base);
    for (int thr = 1; thr <= 32; thr *= 2) printf("  thr %d: %.3f", thr, early_exit(thr) / base);
    printf("\n");
  }
  { /* how well the bound predicts the walk's length */
    double sp = 0, sn = 0, spn = 0, spp = 0, snn = 0, ex = 0; long hist[17] = {0};
    for (int i = 0; i < nseg; i++) { double x = W[i].pred, y = W[i].nc; sp += x; sn += y; spn += x*y; spp += x*x; snn += y*y;
      ex += x == y; hist[W[i].pred > 16 ? 16 : W[i].pred]++; }
    const double mp = sp/nseg, mn = sn/nseg;
    printf("  bound vs walk: mean bound %.3f, mean cells %.3f, exact %.3f, corr %.3f; bound histogram:", mp, mn, ex/nseg,
           (spn/nseg - mp*mn) / sqrt((spp/nseg - mp*mp) * (snn/nseg - mn*mn)));
    for (int k = 0; k <= 16; k++) printf(" %.3f", (double)hist[k]/nseg);
    printf("\n");
  }
  if (getenv("CI_REST")) CI_REST = atof(getenv("CI_REST"));
  if (getenv("QUEUE_ONLY")) {
    build_paths();
    const double Es[4] = {0, 60, 100, 140};
    printf("  (%d paths)\n", npaths);
    for (qbox = 0; qbox <= 1; qbox++) {
      printf("  key: %s\n", qbox ? "grid-box bound (before the big spheres)" : "bound after the big spheres");
      for (int NB = 4; NB <= 16; NB *= 2)
        for (int P = 256; P <= 1024; P *= 2) queue_model(P, NB, Es, 4);
    }
    return 0;
  }
  for (int block = 256; block <= 512; block *= 2)
    for (double E = 0; E <= 120; E += 40) regroup_cost(block, E);
  const char *kn[7] = {"oct", "cell", "oct+cell", "len", "bound", "bound15", "boxbound"};
  for (int block = 256; block <= 1024; block *= 2)
    for (key_mode = 0; key_mode < 7; key_mode++) {
      Acc b = {0};
      for (int t = 0; t < ntiles; t++) for (int i = tile_start[t]; i < tile_start[t+1]; i += block) {
        int nb = tile_start[t+1] - i < block ? tile_start[t+1] - i : block;
        for (int l = 0; l < nb; l++) ids[l] = i + l;
        qsort(ids, nb, sizeof(int), cmpk);
        for (int w = 0; w < nb; w += 64) wave_cost(ids + w, nb - w < 64 ? nb - w : 64, &b);
      }
      char nm[32]; snprintf(nm, sizeof nm, "%d/%s", block, kn[key_mode]); report(nm, &b);
    }
  return 0;
}
