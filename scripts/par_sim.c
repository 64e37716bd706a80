/*
 * par_sim.c — measurement tooling (not a test, not the product): how many dependent steps the
 * team segment's changers would take if every level that follows the last hit were tested at
 * once.  After a hit (or at the carry-in) the remaining levels' directions depend only on the
 * current normal — D' = normalize(reflect(D, N)) from the same origin while rays miss — so
 * all of them can be tested in parallel and the first hit taken.  The sequential form (the
 * resolver's carry_path_spec: one level, or two after a miss, per step) and this "all
 * remaining levels per step" form are both run from the oracle's exact carry-ins and their
 * carry-outs compared bit for bit.
 *
 *   gcc -O2 -ffp-contract=off -Iinclude -Ioracle -Iraytracing-programs_amd/csrc \
 *       scripts/par_sim.c raytracing-programs_amd/csrc/rc_scene.c -lm -o /tmp/par_sim
 *   /tmp/par_sim tests/golden/scenes/quadric.scene 4096 7
 */
#include "../oracle/rc_oracle.c"

#include <stdio.h>

static int refl(const octx *c, int obj) { return c->shapes[obj].reflectivity > 0.0f; }

/* the resolver's step structure (rc_device.hpp carry_path_spec) */
static int seq_steps(octx *c, const float *A, const float *B, const float *N0, int obj0,
                     int maxrec, const float *cin, float *cout) {
  float C[3] = {cin[0], cin[1], cin[2]}, N[3] = {N0[0], N0[1], N0[2]};
  float D1[3] = {A[0], A[1], A[2]}, D2[3] = {B[0], B[1], B[2]};
  int obj = obj0, S = -1, lvl = 2, steps = 0;
  while (lvl < maxrec) {
    if (!refl(c, obj)) break;
    ++steps;
    float P[3], Nn[3], Dw[3];
    int w = o_nearest(c, C, D1, P, Nn, S, 0), two = 0;
    memcpy(Dw, D1, sizeof Dw);
    if (w < 0 && lvl + 1 < maxrec) {
      two = 1;
      w = o_nearest(c, C, D2, P, Nn, -1, 0);
      memcpy(Dw, D2, sizeof Dw);
    }
    if (w >= 0) {
      memcpy(C, P, sizeof C);
      memcpy(N, Nn, sizeof N);
      obj = w;
      S = w;
    } else {
      S = -1;
    }
    lvl += two ? 2 : 1;
    if (lvl >= maxrec || !refl(c, obj)) break;
    float t[3];
    o_reflect(t, Dw, N);
    o_normalize(c, D1, t);
    o_reflect(t, D1, N);
    o_normalize(c, D2, t);
  }
  memcpy(cout, C, sizeof C);
  return steps;
}

/* all remaining levels per step; *chain = serial reflections computed after the first step
 * (the first step's directions depend on the entry alone and could be precomputed) */
static int par_steps(octx *c, const float *A, const float *N0, int obj0, int maxrec,
                     const float *cin, float *cout, int *chain, int *hits) {
  float C[3] = {cin[0], cin[1], cin[2]}, N[3] = {N0[0], N0[1], N0[2]}, D[3] = {A[0], A[1], A[2]};
  int obj = obj0, S = -1, lvl = 2, steps = 0;
  *chain = 0;
  *hits = 0;
  while (lvl < maxrec && refl(c, obj)) {
    ++steps;
    float dirs[8][3];
    memcpy(dirs[0], D, sizeof D);
    const int nd = maxrec - lvl;
    for (int i = 1; i < nd; ++i) {
      float t[3];
      o_reflect(t, dirs[i - 1], N);
      memcpy(dirs[i], dirs[i - 1], sizeof D);   /* o_normalize leaves a zero vector's dst */
      memcpy(dirs[i], t, sizeof t);
      o_normalize(c, dirs[i], t);
      if (steps > 1) ++*chain;
    }
    int w = -1, i = 0;
    float P[3], Nn[3];
    for (; i < nd; ++i) {
      w = o_nearest(c, C, dirs[i], P, Nn, i == 0 ? S : -1, 0);
      if (w >= 0) break;
    }
    if (w < 0) break;
    ++*hits;
    memcpy(C, P, sizeof C);
    memcpy(N, Nn, sizeof N);
    obj = w;
    S = w;
    lvl += i + 1;
    if (lvl >= maxrec || !refl(c, obj)) break;
    float t[3];
    o_reflect(t, dirs[i], N);
    memcpy(D, t, sizeof t);
    o_normalize(c, D, t);
  }
  memcpy(cout, C, sizeof C);
  return steps;
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
  long long lo = 0, hi = 0, best = 0, cur = 0, cs = -1;
  for (size_t p = 0; p < P; ++p) {
    if (cls[p] == 1) cur = 0;
    else if (cls[p] >= 2) {
      if (cur == 0) cs = (long long)p;
      if (++cur > best) best = cur, lo = cs, hi = (long long)p + 1;
    }
  }
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
  long long n = 0, bad = 0, chg = 0, hs[8] = {0}, hp[8] = {0}, hh[8] = {0}, hc[16] = {0};
  long long seq_ch = 0, par_ch = 0, chain_ch = 0, last = -1, gh[12] = {0};
  for (long long p = lo; p < hi; ++p) {
    if (cls[p] < 2) continue;
    ++n;
    const int x = (int)(p % W), y = (int)(p / W);
    float d[3];
    d[0] = (float)((0.0 - (double)js.camera_width / 2.0) + (double)pw * ((double)x + 0.5));
    d[1] = (float)((0.0 + (double)js.camera_height / 2.0) - (double)ph * ((double)y + 0.5));
    d[2] = -1.0f;
    o_normalize(&c, d, d);
    float P0[3], N0[3], t[3], D1[3], A[3], B[3];
    const float O0[3] = {0, 0, 0};
    const int i0 = o_nearest(&c, O0, d, P0, N0, -1, 0);
    o_reflect(t, d, N0);
    o_normalize(&c, D1, t);
    memcpy(A, D1, 12);
    o_reflect(t, D1, N0);
    o_normalize(&c, A, t);
    memcpy(B, A, 12);
    o_reflect(t, A, N0);
    o_normalize(&c, B, t);
    float o1[3], o2[3];
    const int s1 = seq_steps(&c, A, B, N0, i0, maxrec, &cin[3 * p], o1);
    int ch, h;
    const int s2 = par_steps(&c, A, N0, i0, maxrec, &cin[3 * p], o2, &ch, &h);
    if (memcmp(o1, o2, 12)) ++bad;
    if (memcmp(o1, &cin[3 * p], 12)) {   /* a changer */
      ++chg;
      if (last >= 0) { long long g = n - 1 - last; int b = 0; while (b < 11 && (1LL << b) < g) ++b; gh[b]++; }
      last = n - 1;
      hs[s1 < 7 ? s1 : 7]++;
      hp[s2 < 7 ? s2 : 7]++;
      hh[h < 7 ? h : 7]++;
      hc[ch < 15 ? ch : 15]++;
      seq_ch += s1;
      par_ch += s2;
      chain_ch += ch;
    }
  }
  printf("team segment: %lld entries (pixels %lld..%lld), %lld changers, carry-out mismatches "
         "between the two forms %lld\n", n, lo, hi, chg, bad);
  printf("changers, sequential steps:");
  for (int q = 0; q < 8; ++q) printf(" %d:%lld", q, hs[q]);
  printf("  (sum %lld)\nchangers, all-levels steps:", seq_ch);
  for (int q = 0; q < 8; ++q) printf(" %d:%lld", q, hp[q]);
  printf("  (sum %lld)\nchangers, hits:", par_ch);
  for (int q = 0; q < 8; ++q) printf(" %d:%lld", q, hh[q]);
  printf("\nchangers, serial reflections after the first step:");
  for (int q = 0; q < 16; ++q) if (hc[q]) printf(" %d:%lld", q, hc[q]);
  printf("  (sum %lld)\n", chain_ch);
  printf("gaps between consecutive changers (entries, <= 2^b):");
  for (int q = 0; q < 12; ++q) printf(" %d:%lld", q, gh[q]);
  printf("\n");
  return 0;
}
