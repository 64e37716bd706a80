/*
 * step_sim.c — measurement tooling (not a test, not the product): how many cooperative
 * evaluation steps (k_resolve's carry_path_spec iterations: a level, or two when the first
 * misses) the entries of a carry segment take, and what a RESOLVE block step costs when it
 * waits for all of its 16 entries versus only for the entries up to its first changer.
 *
 * Builds on the CPU oracle's restatement (#included for its static helpers):
 *   gcc -O2 -ffp-contract=off -Iinclude -Ioracle scripts/step_sim.c -lm -o /tmp/step_sim
 *   /tmp/step_sim tests/golden/scenes/quadric.scene 4096 7 [window]
 */
#include "../oracle/rc_oracle.c"

#include <stdio.h>

typedef struct {
  float D1[3], D2[3], N0[3];
  int obj0;
} rec_t;

static int refl(const octx *c, int obj) { return c->shapes[obj].reflectivity > 0.0f; }

/* carry_path_spec's control flow on the CPU: returns the steps, writes the carry-out */
static int f_steps(octx *c, const rec_t *r, int maxrec, const float *cin, float *cout,
                   int *levels_hit) {
  float C[3] = {cin[0], cin[1], cin[2]}, N[3] = {r->N0[0], r->N0[1], r->N0[2]};
  float D1[3] = {r->D1[0], r->D1[1], r->D1[2]}, D2[3] = {r->D2[0], r->D2[1], r->D2[2]};
  int obj = r->obj0, S = -1, lvl = 2, steps = 0, hits = 0;
  while (lvl < maxrec) {
    if (!refl(c, obj)) break;
    ++steps;
    float P[3], Nn[3], Dw[3];
    int w = o_nearest(c, C, D1, P, Nn, S, 0);
    int two = 0;
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
      ++hits;
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
  if (levels_hit) *levels_hit = hits;
  return steps;
}

static int same(const float *a, const float *b) { return memcmp(a, b, 12) == 0; }

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: step_sim scene size maxrec [window]\n");
    return 2;
  }
  json_data_t js;
  if (rco_load_scene(argv[1], &js)) return 1;
  const int W = atoi(argv[2]), H = W, maxrec = atoi(argv[3]);
  const int win = argc > 4 ? atoi(argv[4]) : 16;
  const size_t P = (size_t)W * H;
  uint8_t *img = malloc(P * 3), *cls = malloc(P);
  float *cin = malloc(P * 3 * sizeof(float));
  rco_stats st;
  if (rco_render_cls(&js, W, H, maxrec, RCO_MODE_PARITY, img, &st, cin, cls)) return 1;
  /* the longest segment (segments split at first-reflection writers, class 1) */
  long long best_len = 0, best_start = -1, cur = 0, cur_start = -1;
  for (size_t p = 0; p < P; ++p) {
    if (cls[p] == 1) cur = 0;
    else if (cls[p] >= 2) {
      if (cur == 0) cur_start = (long long)p;
      if (++cur > best_len) best_len = cur, best_start = cur_start;
    }
  }
  /* its entries */
  long long n = 0;
  int64_t *pix = malloc(sizeof(int64_t) * best_len);
  for (size_t p = (size_t)best_start; p < P && n < best_len; ++p) {
    if (cls[p] == 1) break;
    if (cls[p] >= 2) pix[n++] = (int64_t)p;
  }
  printf("longest segment: %lld entries from pixel %lld (row %lld), %lld found\n", best_len,
         best_start, best_start / W, n);
  /* records: primary hit, level-1 (missed) and level-2/3 directions */
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
  rec_t *rec = malloc(sizeof(rec_t) * n);
  for (long long i = 0; i < n; ++i) {
    const int x = (int)(pix[i] % W), y = (int)(pix[i] / W);
    float d[3];
    d[0] = (float)((0.0 - (double)js.camera_width / 2.0) + (double)pw * ((double)x + 0.5));
    d[1] = (float)((0.0 + (double)js.camera_height / 2.0) - (double)ph * ((double)y + 0.5));
    d[2] = -1.0f;
    o_normalize(&c, d, d);
    float P0[3], N0[3], t[3], D1[3];
    const float O0[3] = {0, 0, 0};
    const int i0 = o_nearest(&c, O0, d, P0, N0, -1, 0);
    o_reflect(t, d, N0);
    o_normalize(&c, D1, t);   /* level 1: missed */
    rec[i].obj0 = i0;
    memcpy(rec[i].N0, N0, 12);
    o_reflect(t, D1, N0);
    o_normalize(&c, rec[i].D1, t);
    o_reflect(t, rec[i].D1, N0);
    o_normalize(&c, rec[i].D2, t);
  }
  /* check: each entry at its oracle carry-in gives the next entry's carry-in */
  long long bad = 0, changers = 0;
  long long hist[8] = {0}, hist_ch[8] = {0}, hist_cl[8] = {0};
  for (long long i = 0; i < n; ++i) {
    float out[3];
    int hits;
    const int k = f_steps(&c, &rec[i], maxrec, &cin[3 * pix[i]], out, &hits);
    const int ch = !same(out, &cin[3 * pix[i]]);
    if (i + 1 < n && !same(out, &cin[3 * pix[i + 1]])) ++bad;
    changers += ch;
    hist[k < 7 ? k : 7]++;
    (ch ? hist_ch : hist_cl)[k < 7 ? k : 7]++;
  }
  printf("chain check: %lld mismatches; changers %lld\n", bad, changers);
  printf("steps per entry (all / changers / clean):");
  for (int k = 0; k < 8; ++k) printf(" %d:%lld/%lld/%lld", k, hist[k], hist_ch[k], hist_cl[k]);
  printf("\n");
  /* RESOLVE simulation: windows of `win` entries at the current carry */
  long long pos = 0, nwin_ch = 0, nwin_clean_after = 0;
  long long cost_all = 0, cost_prefix = 0, cost_k = 0, cost_clean_after = 0;
  long long hist_all[8] = {0}, hist_pre[8] = {0};
  float C[3];
  memcpy(C, &cin[3 * pix[0]], 12);
  int after = 0;
  while (pos < n) {
    long long end = pos + win < n ? pos + win : n, k = -1;
    int mx = 0, mxp = 0;
    float outk[3];
    for (long long i = pos; i < end; ++i) {
      float out[3];
      const int st_ = f_steps(&c, &rec[i], maxrec, C, out, NULL);
      if (st_ > mx) mx = st_;
      if (k < 0) {
        if (st_ > mxp) mxp = st_;
        if (!same(out, C)) {
          k = i;
          memcpy(outk, out, 12);
          cost_k += st_;
        }
      }
    }
    if (k >= 0) {
      ++nwin_ch;
      cost_all += mx;
      cost_prefix += mxp;
      hist_all[mx]++;
      hist_pre[mxp]++;
      memcpy(C, outk, 12);
      pos = k + 1;
      after = 1;
    } else {
      if (after) {
        ++nwin_clean_after;
        cost_clean_after += mx;
      }
      after = 0;
      pos = end;
    }
  }
  printf("window %d: %lld changer windows: steps waited for all %lld (%.2f/window), up to the "
         "first changer %lld (%.2f), the changer alone %lld (%.2f); %lld clean windows after a "
         "change: %lld steps (%.2f)\n",
         win, nwin_ch, cost_all, (double)cost_all / nwin_ch, cost_prefix,
         (double)cost_prefix / nwin_ch, cost_k, (double)cost_k / nwin_ch, nwin_clean_after,
         cost_clean_after, nwin_clean_after ? (double)cost_clean_after / nwin_clean_after : 0.0);
  printf("max steps per changer window (all):");
  for (int k = 0; k < 8; ++k) printf(" %d:%lld", k, hist_all[k]);
  printf("\nmax steps per changer window (prefix):");
  for (int k = 0; k < 8; ++k) printf(" %d:%lld", k, hist_pre[k]);
  printf("\n");
  return 0;
}
