/*
 * phasec_sim.c — measurement tooling (not a test, not the product): how much of phase C's
 * SIMD time is lane divergence?  For every DEP entry that hits at its exact carry-in (from
 * the CPU oracle) it replays shade_dep_cont's control flow (rc_device.hpp: levels 2.., a
 * nearest-hit per level, shading with a shadow ray per lit light at hit levels) and counts
 * shape tests.  A wave's cost is modelled level by level as lockstep execution: a level's
 * nearest-hit costs n tests if any lane is still looping, a light's shadow loop costs the
 * most tests any lane at that level needs.  The entries are taken in k_dep_chunks' order
 * (1 024-entry chunks, hit entries compacted in order, 64 per wave) and, for comparison,
 * sorted by their per-level pattern within each chunk.  It also prints the split of a hit
 * entry's tests between the nearest-hit searches and the shadow rays.
 *
 *   gcc -O2 -ffp-contract=off -Iinclude -Ioracle -Iraytracing-programs_amd/csrc \
 *       scripts/phasec_sim.c raytracing-programs_amd/csrc/rc_scene.c -lm -o /tmp/phasec_sim
 *   /tmp/phasec_sim tests/golden/scenes/quadric.scene 4096 7
 */
#include "../oracle/rc_oracle.c"

#include <stdio.h>

#define MAXL 8
typedef struct {
  int levels;            /* loop iterations executed */
  int hit[MAXL];         /* level hit */
  int sh[MAXL][4];       /* shadow tests per light at that level (0: inert / not shaded) */
  long long key;
} ent_t;

static int refl(const octx *c, int obj) { return c->shapes[obj].reflectivity > 0.0f; }

/* shadow tests until the first hit (the GPU's shadowed() stops there) */
static int shadow_tests(octx *c, const float *P, const float *D, int skip, int *hit) {
  int n = 0;
  *hit = 0;
  for (int k = 0; k < c->n; k++) {
    if (k == skip) continue;
    ++n;
    float t = 0.0f;
    int h = 0;
    const shape_t *s = &c->shapes[k];
    if (s->type == SPHERE) h = o_sphere(P, D, s, &t);
    else if (s->type == PLANE) h = o_plane(P, D, s, &t);
    else if (s->type == QUADRIC) {
      h = o_quadric(P, D, s, &t);
      if (h && skip != -1 && (P[2] + t * D[2]) < P[2]) h = 0;
    }
    if (h && t > 0.0f && t < INFINITY) {
      *hit = 1;
      return n;
    }
  }
  return n;
}

static void replay(octx *c, const float *A, const float *N0, int obj0, int maxrec,
                   const float *cin, ent_t *e) {
  memset(e, 0, sizeof *e);
  float O[3] = {cin[0], cin[1], cin[2]}, C[3] = {cin[0], cin[1], cin[2]};
  float D[3] = {A[0], A[1], A[2]}, N[3] = {N0[0], N0[1], N0[2]};
  int obj = obj0, S = -1, li = 0;
  for (int lvl = 2; lvl < maxrec && li < MAXL; ++lvl, ++li) {
    if (!refl(c, obj)) break;
    if (lvl > 2) {
      float t[3];
      o_reflect(t, D, N);
      o_normalize(c, D, t);
    }
    e->levels++;
    float P[3], Nn[3];
    const int i = o_nearest(c, O, D, P, Nn, S, 0);
    if (i >= 0) {
      memcpy(C, P, sizeof C);
      memcpy(N, Nn, sizeof N);
      obj = i;
      e->hit[li] = 1;
      const shape_t *o = &c->shapes[i];
      const float opacity = (float)((1.0 - (double)o->reflectivity) - (double)o->refractivity);
      if (opacity > 0.0f) {
        for (int l = 0; l < c->m && l < 4; l++) {
          const light_t *L = &c->lights[l];
          float ld[3] = {L->position[0] - C[0], L->position[1] - C[1], L->position[2] - C[2]};
          o_normalize(c, ld, ld);
          const float th = o_dot(N, ld);
          if (th <= 0.0f) continue;   /* inert: no shadow ray */
          int hh;
          e->sh[li][l] = shadow_tests(c, C, ld, i, &hh);
        }
      }
    }
    memcpy(O, C, sizeof O);
    S = i;
  }
  long long k = e->levels;
  for (int l = 0; l < e->levels && l < 5; ++l) k = k * 4 + e->hit[l] * 2 + (e->sh[l][0] > 0);
  e->key = k;
}

/* lockstep cost of a wave of up to 64 entries, in shape tests */
static long long wave_cost(ent_t **w, int nw, int nshapes, int m) {
  long long cost = 0;
  for (int l = 0; l < MAXL; ++l) {
    int any = 0, anyhit = 0;
    for (int q = 0; q < nw; ++q) {
      any |= w[q]->levels > l;
      anyhit |= w[q]->levels > l && w[q]->hit[l];
    }
    if (!any) break;
    cost += nshapes;   /* nearest-hit */
    if (!anyhit) continue;
    for (int li = 0; li < m && li < 4; ++li) {
      int mx = 0;
      for (int q = 0; q < nw; ++q)
        if (w[q]->levels > l && w[q]->sh[l][li] > mx) mx = w[q]->sh[l][li];
      cost += mx + 2;   /* shadow loop + the light's evaluation */
    }
  }
  return cost;
}

static int cmp_key(const void *a, const void *b) {
  const ent_t *x = *(ent_t *const *)a, *y = *(ent_t *const *)b;
  return (x->key > y->key) - (x->key < y->key);
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  json_data_t js;
  if (rco_load_scene(argv[1], &js)) return 1;
  const int W = atoi(argv[2]), H = W, maxrec = atoi(argv[3]);
  const size_t P = (size_t)W * H;
  uint8_t *img = malloc(P * 3), *cls = malloc(P);
  float *cin = malloc(P * 3 * sizeof(float));
  rco_stats st;
  if (rco_render_cls(&js, W, H, maxrec, RCO_MODE_PARITY, img, &st, cin, cls)) return 1;
  octx c;
  memset(&c, 0, sizeof c);
  rco_stats st2;
  memset(&st2, 0, sizeof st2);
  c.st = &st2;
  c.n = js.num_shapes;
  c.m = js.num_lights;
  shape_t *sh = calloc(c.n, sizeof(shape_t));
  light_t *li = calloc(c.m > 0 ? c.m : 1, sizeof(light_t));
  const shape_t *s = js.shapes_list;
  for (int k = 0; k < c.n; k++, s = s->next) sh[k] = *s;
  const light_t *l = js.lights_list;
  for (int k = 0; k < c.m; k++, l = l->next) li[k] = *l;
  c.shapes = sh;
  c.lights = li;
  o_build_phantom(&c);
  const float ph = js.camera_height / (float)H, pw = js.camera_width / (float)W;
  long long ndep = 0;
  for (size_t p = 0; p < P; ++p) ndep += cls[p] >= 2;
  ent_t *all = calloc((size_t)ndep, sizeof(ent_t));
  char *hitm = calloc((size_t)ndep, 1);
  long long j = 0, nhit = 0;
  for (size_t p = 0; p < P; ++p) {
    if (cls[p] < 2) continue;
    const int x = (int)(p % W), y = (int)(p / W);
    float d[3];
    d[0] = (float)((0.0 - (double)js.camera_width / 2.0) + (double)pw * ((double)x + 0.5));
    d[1] = (float)((0.0 + (double)js.camera_height / 2.0) - (double)ph * ((double)y + 0.5));
    d[2] = -1.0f;
    o_normalize(&c, d, d);
    float P0[3], N0[3], t[3], D1[3], A[3];
    const float O0[3] = {0, 0, 0};
    const int i0 = o_nearest(&c, O0, d, P0, N0, -1, 0);
    o_reflect(t, d, N0);
    o_normalize(&c, D1, t);
    memcpy(A, D1, 12);
    o_reflect(t, D1, N0);
    o_normalize(&c, A, t);
    replay(&c, A, N0, i0, maxrec, &cin[3 * p], &all[j]);
    int any = 0;
    for (int q = 0; q < all[j].levels; ++q) any |= all[j].hit[q];
    hitm[j] = (char)any;
    nhit += any;
    ++j;
  }
  /* k_dep_chunks' order: per 1024-entry chunk, the hit entries in order, 64 per wave */
  ent_t **lst = malloc(sizeof(ent_t *) * 1024);
  long long c_order = 0, c_sorted = 0, c_ideal = 0, waves = 0;
  for (long long ch = 0; ch < ndep; ch += 1024) {
    int n = 0;
    for (long long q = ch; q < ch + 1024 && q < ndep; ++q)
      if (hitm[q]) lst[n++] = &all[q];
    for (int w0 = 0; w0 < n; w0 += 64) {
      const int nw = n - w0 < 64 ? n - w0 : 64;
      c_order += wave_cost(lst + w0, nw, c.n, c.m);
      ++waves;
      for (int q = 0; q < nw; ++q) c_ideal += wave_cost(lst + w0 + q, 1, c.n, c.m);
    }
    qsort(lst, (size_t)n, sizeof(ent_t *), cmp_key);
    for (int w0 = 0; w0 < n; w0 += 64) {
      const int nw = n - w0 < 64 ? n - w0 : 64;
      c_sorted += wave_cost(lst + w0, nw, c.n, c.m);
    }
  }
  long long nn = 0, ns = 0, nl = 0;
  for (long long q = 0; q < ndep; ++q) {
    if (!hitm[q]) continue;
    nn += (long long)all[q].levels * c.n;
    for (int l = 0; l < all[q].levels; ++l)
      for (int li = 0; li < c.m && li < 4; ++li)
        if (all[q].sh[l][li] > 0) ns += all[q].sh[l][li], ++nl;
  }
  printf("per hit entry: nearest-hit tests %.2f, shadow tests %.2f (%.2f lit lights)\n",
         (double)nn / nhit, (double)ns / nhit, (double)nl / nhit);
  printf("DEP entries %lld, hit entries %lld, waves %lld\n", ndep, nhit, waves);
  printf("lockstep cost (shape tests per wave, mean): chunk order %.1f, sorted within chunks %.1f "
         "(%.1f %%), per-lane mean %.1f\n",
         (double)c_order / waves, (double)c_sorted / waves,
         100.0 * (double)c_sorted / (double)c_order, (double)c_ideal / (double)nhit);
  return 0;
}
