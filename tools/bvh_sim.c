/* tools/bvh_sim.c — CPU model of the BVH traversal cost on the final scene.
 *
 * Analysis only (not product, not oracle): traces an approximate path
 * distribution (camera rays, then lambertian / metal / dielectric bounces,
 * brute-force closest hit in double) over the fixture scene, records every
 * segment's ray, and replays the segments through BVH variants in 64-lane
 * lockstep groups (one 8x8 tile's segments, shuffled: path regeneration mixes
 * depths in a wave).  Reports per-lane node visits and leaf tests, and the
 * wave-level loop iterations (max over lanes) that set the kernel's cost.
 *
 *   gcc -O2 -o /tmp/bvh_sim tools/bvh_sim.c -lm && /tmp/bvh_sim tests/golden/scene_final.txt
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MAXS 1024
static int N;
static double C[MAXS][4];
static int KIND[MAXS];
static double MAT[MAXS][4];

static unsigned long long rs = 88172645463325252ull;
static double rnd(void) {
  rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
  return (rs >> 11) * (1.0 / 9007199254740992.0);
}

typedef struct { double o[3], d[3]; } Ray;
static Ray *segs; static int nseg, capseg;
static int *seg_tile;

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

static void push(const double o[3], const double d[3], int tile) {
  if (nseg == capseg) { capseg = capseg ? 2*capseg : 1<<20; segs = realloc(segs, capseg*sizeof(Ray)); seg_tile = realloc(seg_tile, capseg*sizeof(int)); }
  memcpy(segs[nseg].o, o, 24); memcpy(segs[nseg].d, d, 24); seg_tile[nseg] = tile; nseg++;
}

/* ---- BVH ---------------------------------------------------------------- */
typedef struct { float lo[3], hi[3]; int left, right, first, cnt, axis; } BNode;
static BNode nodes[4096]; static int nn;
static int leafidx[MAXS];
static int nleafidx;
static int g_leafmax = 4, g_sah = 0, g_spec = 0, g_f16 = 0;
static float f16_down(double v) { _Float16 h = (_Float16)v; while ((double)h > v) { unsigned short b; __builtin_memcpy(&b, &h, 2); b = (h > 0) ? b - 1 : (h < 0 ? b + 1 : 0x8001); __builtin_memcpy(&h, &b, 2); } return (float)h; }
static float f16_up(double v) { return -f16_down(-v); }
static double margin = 0.0125;

static void bounds(int *ids, int cnt, double lo[3], double hi[3]) {
  for (int a = 0; a < 3; a++) { lo[a] = INFINITY; hi[a] = -INFINITY; }
  for (int i = 0; i < cnt; i++) for (int a = 0; a < 3; a++) {
    double r = fabs(C[ids[i]][3]) + margin;
    if (C[ids[i]][a]-r < lo[a]) lo[a] = C[ids[i]][a]-r;
    if (C[ids[i]][a]+r > hi[a]) hi[a] = C[ids[i]][a]+r;
  }
}
static int g_ax;
static int cmpax(const void *x, const void *y) {
  double a = C[*(int*)x][g_ax], b = C[*(int*)y][g_ax];
  return a < b ? -1 : a > b ? 1 : (*(int*)x - *(int*)y);
}
static double area(double lo[3], double hi[3]) {
  double e0 = hi[0]-lo[0], e1 = hi[1]-lo[1], e2 = hi[2]-lo[2];
  return 2*(e0*e1+e1*e2+e0*e2);
}
static int build(int *ids, int cnt) {
  int me = nn++;
  double lo[3], hi[3]; bounds(ids, cnt, lo, hi);
  for (int a = 0; a < 3; a++) {
    nodes[me].lo[a] = lo[a]; nodes[me].hi[a] = hi[a];
    if (g_f16) {  /* round outward to half precision */
      _Float16 l = (_Float16)lo[a], h = (_Float16)hi[a];
      nodes[me].lo[a] = f16_down(lo[a]); nodes[me].hi[a] = f16_up(hi[a]);
      (void)l; (void)h;
    }
  }
  if (cnt <= g_leafmax) {
    nodes[me].left = nodes[me].right = -1; nodes[me].first = nleafidx; nodes[me].cnt = cnt;
    for (int i = 0; i < cnt; i++) leafidx[nleafidx++] = ids[i];
    return me;
  }
  int ax = 0, mid = cnt/2;
  if (!g_sah) {
    double clo[3]={1e30,1e30,1e30}, chi[3]={-1e30,-1e30,-1e30};
    for (int i = 0; i < cnt; i++) for (int a = 0; a < 3; a++) { double c = C[ids[i]][a]; if (c<clo[a]) clo[a]=c; if (c>chi[a]) chi[a]=c; }
    for (int a = 1; a < 3; a++) if (chi[a]-clo[a] > chi[ax]-clo[ax]) ax = a;
    g_ax = ax; qsort(ids, cnt, sizeof(int), cmpax);
  } else {
    double best = INFINITY; int bax = 0, bmid = cnt/2;
    static double lar[MAXS], rar[MAXS];
    for (int a = 0; a < 3; a++) {
      g_ax = a; qsort(ids, cnt, sizeof(int), cmpax);
      double l[3], h[3];
      for (int i = 1; i < cnt; i++) { bounds(ids, i, l, h); lar[i] = area(l, h) * i; }
      for (int i = 1; i < cnt; i++) { bounds(ids+i, cnt-i, l, h); rar[i] = area(l, h) * (cnt-i); }
      for (int i = 1; i < cnt; i++) {
        double c = lar[i] + rar[i];
        if (c < best) { best = c; bax = a; bmid = i; }
      }
    }
    ax = bax; mid = bmid; g_ax = ax; qsort(ids, cnt, sizeof(int), cmpax);
    if (cnt <= g_leafmax) mid = cnt/2;
  }
  nodes[me].axis = ax; nodes[me].cnt = 0;
  int l = build(ids, mid); int r = build(ids+mid, cnt-mid);
  nodes[me].left = l; nodes[me].right = r;
  return me;
}

/* flattened DFS order for a given octant: at each inner node, near child first
 * (ordered=1: by the ray sign on the split axis; 0: left first) */
typedef struct { float lo[3], hi[3]; int skip, first, cnt; } FNode;
static FNode flat[8][4096]; static int nflat;
static void flatten(int oct, int ordered, int n, int *pos) {
  int me = (*pos)++;
  FNode *f = &flat[oct][me];
  memcpy(f->lo, nodes[n].lo, 12); memcpy(f->hi, nodes[n].hi, 12);
  f->first = nodes[n].first; f->cnt = nodes[n].left < 0 ? nodes[n].cnt : -1;
  if (nodes[n].left >= 0) {
    int a = nodes[n].left, b = nodes[n].right;
    if (ordered && ((oct >> nodes[n].axis) & 1)) { int t = a; a = b; b = t; }
    flatten(oct, ordered, a, pos); flatten(oct, ordered, b, pos);
  }
  f->skip = *pos;
}

typedef struct { long visits, tests, wave_iters, wave_leaf_iters, waves, res_blocks, res_lanes, res_acc, res_blocks_pf, pair_iters; } Stat;

static void run(const char *name, int ordered) {
  /* small spheres only, as the kernel: big (r > 4 x median) stay brute force */
  int ids[MAXS], cnt = 0;
  for (int k = 0; k < N; k++) if (fabs(C[k][3]) <= 0.8) ids[cnt++] = k;
  nn = 0; nleafidx = 0; build(ids, cnt);
  for (int o = 0; o < 8; o++) { int pos = 0; flatten(o, ordered, 0, &pos); nflat = pos; }
  Stat st = {0};
  /* groups of 64 segments of one tile (segments are stored tile by tile, shuffled) */
  for (int s0 = 0; s0 < nseg; s0 += 64) {
    int nl = nseg - s0 < 64 ? nseg - s0 : 64;
    int node[64]; double tmax[64]; float ix[64][3]; int oct[64];
    for (int l = 0; l < nl; l++) {
      Ray *r = &segs[s0+l];
      node[l] = 0; double t; int k = -1;
      /* t_max after the big spheres */
      double a = r->d[0]*r->d[0]+r->d[1]*r->d[1]+r->d[2]*r->d[2];
      tmax[l] = INFINITY;
      for (int q = 0; q < N; q++) if (fabs(C[q][3]) > 0.8) {
        double oc[3] = {r->o[0]-C[q][0], r->o[1]-C[q][1], r->o[2]-C[q][2]};
        double hb = oc[0]*r->d[0]+oc[1]*r->d[1]+oc[2]*r->d[2];
        double c = oc[0]*oc[0]+oc[1]*oc[1]+oc[2]*oc[2]-C[q][3]*C[q][3];
        double disc = hb*hb - a*c; if (disc < 0) continue;
        double sq = sqrt(disc), rt = (-hb-sq)/a;
        if (rt < 0.001 || rt > tmax[l]) { rt = (-hb+sq)/a; if (rt < 0.001 || rt > tmax[l]) continue; }
        tmax[l] = rt;
      }
      (void)t; (void)k;
      oct[l] = (r->d[0] < 0) | ((r->d[1] < 0) << 1) | ((r->d[2] < 0) << 2);
      for (int q = 0; q < 3; q++) ix[l][q] = 1.0f / (float)r->d[q];
    }
    if (g_spec) {
      int pend[64]; int done[64];
      for (int l = 0; l < nl; l++) { pend[l] = -1; done[l] = 0; }
      for (;;) {
        int alldone = 1;
        for (int l = 0; l < nl; l++) if (!done[l]) alldone = 0;
        if (alldone) break;
        for (;;) {  /* traversal until each lane holds a leaf or is done */
          int any = 0;
          for (int l = 0; l < nl; l++) {
            if (done[l] || pend[l] >= 0) continue;
            if (node[l] >= nflat) { done[l] = 1; continue; }
            any = 1;
            Ray *r = &segs[s0+l];
            FNode *f = &flat[oct[l]][node[l]];
            double tn = 0, tf = tmax[l];
            for (int q = 0; q < 3; q++) {
              double t0 = (f->lo[q]-r->o[q])*ix[l][q], t1 = (f->hi[q]-r->o[q])*ix[l][q];
              if (t0 > t1) { double x = t0; t0 = t1; t1 = x; }
              if (t0 > tn) tn = t0; if (t1 < tf) tf = t1;
            }
            int enter = tn <= tf;
            st.visits++;
            if (enter && f->cnt >= 0) pend[l] = node[l];
            node[l] = enter ? node[l] + 1 : f->skip;
          }
          if (!any) break;
          st.wave_iters++;
        }
        int maxcnt = 0;
        for (int l = 0; l < nl; l++) {
          if (pend[l] < 0) continue;
          FNode *f = &flat[oct[l]][pend[l]];
          Ray *r = &segs[s0+l];
          if (f->cnt > maxcnt) maxcnt = f->cnt;
          double a = r->d[0]*r->d[0]+r->d[1]*r->d[1]+r->d[2]*r->d[2];
          for (int i = 0; i < f->cnt; i++) {
            int q = leafidx[f->first+i]; st.tests++;
            double oc[3] = {r->o[0]-C[q][0], r->o[1]-C[q][1], r->o[2]-C[q][2]};
            double hb = oc[0]*r->d[0]+oc[1]*r->d[1]+oc[2]*r->d[2];
            double c = oc[0]*oc[0]+oc[1]*oc[1]+oc[2]*oc[2]-C[q][3]*C[q][3];
            double disc = hb*hb - a*c; if (disc < 0) continue;
            double sq = sqrt(disc), rt = (-hb-sq)/a;
            if (rt < 0.001 || rt > tmax[l]) { rt = (-hb+sq)/a; if (rt < 0.001 || rt > tmax[l]) continue; }
            tmax[l] = rt;
          }
          pend[l] = -1;
        }
        st.wave_leaf_iters += maxcnt;
      }
      st.waves++;
      continue;
    }
    int active = nl;
    while (active) {
      int anyleaf = 0, maxcnt = 0, cand[16] = {0}, candpf[16] = {0};
      active = 0;
      for (int l = 0; l < nl; l++) {
        if (node[l] >= nflat) continue;
        active++;
        Ray *r = &segs[s0+l];
        FNode *f = &flat[oct[l]][node[l]];
        double tn = 0, tf = tmax[l];
        for (int q = 0; q < 3; q++) {
          double t0 = (f->lo[q]-r->o[q])*ix[l][q], t1 = (f->hi[q]-r->o[q])*ix[l][q];
          if (t0 > t1) { double x = t0; t0 = t1; t1 = x; }
          if (t0 > tn) tn = t0; if (t1 < tf) tf = t1;
        }
        int enter = tn <= tf;
        st.visits++;
        if (enter && f->cnt >= 0) {
          anyleaf = 1; if (f->cnt > maxcnt) maxcnt = f->cnt;
          double a = r->d[0]*r->d[0]+r->d[1]*r->d[1]+r->d[2]*r->d[2];
          for (int i = 0; i < f->cnt; i++) {
            int q = leafidx[f->first+i]; st.tests++;
            double oc[3] = {r->o[0]-C[q][0], r->o[1]-C[q][1], r->o[2]-C[q][2]};
            double hb = oc[0]*r->d[0]+oc[1]*r->d[1]+oc[2]*r->d[2];
            double c = oc[0]*oc[0]+oc[1]*oc[1]+oc[2]*oc[2]-C[q][3]*C[q][3];
            double disc = hb*hb - a*c; if (disc < 0) continue;
            cand[i] = 1; st.res_lanes++;
            double sq = sqrt(disc), rt = (-hb-sq)/a;
            if (!(rt > tmax[l] || (-hb+sq)/a < 0.001)) candpf[i] = 1;
            if (rt < 0.001 || rt > tmax[l]) { rt = (-hb+sq)/a; if (rt < 0.001 || rt > tmax[l]) continue; }
            tmax[l] = rt; st.res_acc++;
          }
        }
        node[l] = enter ? node[l] + 1 : f->skip;
      }
      if (active) { st.wave_iters++; if (anyleaf) { st.wave_leaf_iters += maxcnt; st.pair_iters += (maxcnt + 1) / 2; } }
      for (int i = 0; i < 16; i++) { st.res_blocks += cand[i]; st.res_blocks_pf += candpf[i]; }
    }
    st.waves++;
  }
  if (!g_spec) printf("   pair-iters/wave-seg %.2f  cost(node 24, sphere 13, pair 16, resolve 45): scalar %.0f  packed %.0f\n",
         (double)st.pair_iters*64/nseg,
         ((double)st.wave_iters*24 + st.wave_leaf_iters*13 + st.res_blocks*45)*64/nseg,
         ((double)st.wave_iters*24 + st.pair_iters*16 + st.res_blocks*45)*64/nseg);
  if (!g_spec) printf("   resolve blocks/wave-seg %.2f (after a t_max prefilter %.2f); lane candidates/seg %.2f accepted %.2f\n",
         (double)st.res_blocks*64/nseg, (double)st.res_blocks_pf*64/nseg, (double)st.res_lanes/nseg, (double)st.res_acc/nseg);
  printf("%s%-26s nodes %4d  lane visits %6.2f  leaf tests %5.2f  wave iters %6.2f  wave leaf-iters %6.2f  (per segment)\n",
         g_spec ? "S " : "  ", name, nflat, (double)st.visits/nseg, (double)st.tests/nseg, (double)st.wave_iters*64/nseg,
         (double)st.wave_leaf_iters*64/nseg);
}

int main(int argc, char **argv) {
  FILE *f = fopen(argc > 1 ? argv[1] : "tests/golden/scene_final.txt", "r");
  if (!f || fscanf(f, "%d", &N) != 1) return 1;
  for (int k = 0; k < N; k++)
    if (fscanf(f, "%lf %lf %lf %lf %d %lf %lf %lf %lf", &C[k][0], &C[k][1], &C[k][2], &C[k][3], &KIND[k],
               &MAT[k][0], &MAT[k][1], &MAT[k][2], &MAT[k][3]) != 9) return 1;
  /* camera fixture (camera_final.txt) */
  double org[3] = {13, 2, 3}, llc[3] = {3.0237371659391918, -1.2262841980681716, 3.4122032022021487},
         hor[3] = {1.189463936993608, 0, -5.1543437269723009}, ver[3] = {-0.50942050206062017, 3.4875711294919385, -0.11755857739860466},
         cu[3] = {0.22485950669875845, 0, -0.97439119569461996}, cv[3] = {-0.14445336159384606, 0.98894993706556156, -0.033335391137041398};
  double lens = 0.05;
  int W = 1200, H = 800, spp = argc > 2 ? atoi(argv[2]) : 2, stride = argc > 3 ? atoi(argv[3]) : 5;
  /* tiles of 8x8 on a sparse grid of tiles */
  for (int ty = 0; ty < H/8; ty += stride) for (int tx = 0; tx < W/8; tx += stride) {
    int start = nseg;
    for (int s = 0; s < spp; s++) for (int p = 0; p < 64; p++) {
      int i = tx*8 + p%8, j = ty*8 + p/8;
      double u = (i + rnd())/(W-1), v = (j + rnd())/(H-1);
      double rr = sqrt(rnd())*lens, ph = 2*M_PI*rnd(), dx = rr*cos(ph), dy = rr*sin(ph);
      double o[3], d[3];
      for (int a = 0; a < 3; a++) { o[a] = org[a] + cu[a]*dx + cv[a]*dy; d[a] = llc[a] + u*hor[a] + v*ver[a] - o[a]; }
      for (int depth = 0; depth < 50; depth++) {
        push(o, d, ty*1000+tx);
        double t; int k = hit_bf(o, d, &t);
        if (k < 0) break;
        double pp[3], n[3], r = C[k][3];
        for (int a = 0; a < 3; a++) { pp[a] = o[a] + t*d[a]; n[a] = (pp[a]-C[k][a])/r; }
        double dn = d[0]*n[0]+d[1]*n[1]+d[2]*n[2];
        int front = dn < 0; if (!front) for (int a = 0; a < 3; a++) n[a] = -n[a];
        double nd[3], ru[3]; rand_unit(ru);
        if (KIND[k] == 0) { for (int a = 0; a < 3; a++) nd[a] = n[a] + ru[a]; if (rnd() > 0.55) break; }
        else if (KIND[k] == 1) {
          double dl = sqrt(d[0]*d[0]+d[1]*d[1]+d[2]*d[2]), ud[3]; for (int a = 0; a < 3; a++) ud[a] = d[a]/dl;
          double c = ud[0]*n[0]+ud[1]*n[1]+ud[2]*n[2];
          for (int a = 0; a < 3; a++) nd[a] = ud[a] - 2*c*n[a] + MAT[k][3]*ru[a]*rnd();
          if (nd[0]*n[0]+nd[1]*n[1]+nd[2]*n[2] <= 0) break;
        } else {
          double dl = sqrt(d[0]*d[0]+d[1]*d[1]+d[2]*d[2]), ud[3]; for (int a = 0; a < 3; a++) ud[a] = d[a]/dl;
          double eta = front ? 1/1.5 : 1.5, c = -(ud[0]*n[0]+ud[1]*n[1]+ud[2]*n[2]); if (c > 1) c = 1;
          double s2 = eta*eta*(1-c*c);
          if (s2 > 1 || rnd() < 0.05) for (int a = 0; a < 3; a++) nd[a] = ud[a] + 2*c*n[a];
          else { double k2 = sqrt(1-s2); for (int a = 0; a < 3; a++) nd[a] = eta*ud[a] + (eta*c - k2)*n[a]; }
        }
        double side = nd[0]*n[0]+nd[1]*n[1]+nd[2]*n[2] < 0 ? -1 : 1;
        for (int a = 0; a < 3; a++) { o[a] = pp[a] + side*7e-4*n[a]; d[a] = nd[a]; }
      }
    }
    /* shuffle the tile's segments: path regeneration mixes depths in a wave */
    for (int i = nseg - 1; i > start; i--) {
      int jx = start + (int)(rnd() * (i - start + 1));
      Ray t = segs[i]; segs[i] = segs[jx]; segs[jx] = t;
    }
  }
  printf("segments %d\n", nseg);
  if (getenv("F16")) g_f16 = 1;
  for (g_spec = 0; g_spec < 2; g_spec++)
  for (int lm = 1; lm <= 12; lm += (lm < 2 ? 1 : 2)) {
    if (g_spec) printf("-- speculative (leaves postponed until every lane holds one)\n");
    char nm[64];
    g_leafmax = lm; g_sah = 0; sprintf(nm, "median leaf%d fixed", lm); run(nm, 0);
    sprintf(nm, "median leaf%d ordered", lm); run(nm, 1);
    g_sah = 1; sprintf(nm, "sah leaf%d fixed", lm); run(nm, 0);
    sprintf(nm, "sah leaf%d ordered", lm); run(nm, 1);
  }
  return 0;
}
