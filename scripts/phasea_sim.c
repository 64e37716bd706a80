/*
 * phasea_sim.c — measurement tooling (not a test, not the product): how much of phase A's
 * SIMD time is lane divergence?  Per pixel, the shape tests the reference's loop makes
 * (CPU oracle counters: nearest-hit and shadow tests) up to where phase A stops (a DEP pixel:
 * its primary level and first bounce only); a wave is an 8x8 pixel tile (k_phase_a) and runs
 * as long as its busiest lane, so its cost is modelled as 64 x the tile's maximum.  Lane
 * efficiency = sum of tests / sum of (64 x tile maximum).  Upper bound of the gain from
 * regrouping rays by bounce level (a wavefront scheme), before its own costs.
 *
 *   gcc -O2 -ffp-contract=off -Iinclude -Ioracle -Iraytracing-programs_amd/csrc \
 *       scripts/phasea_sim.c -lm -o /tmp/phasea_sim
 *   /tmp/phasea_sim tests/golden/scenes/quadric.scene 4096 7
 */
#include "../oracle/rc_oracle.c"

#include <stdio.h>

static int64_t tests(const rco_stats *s) {
  return s->sphere_tests + s->plane_tests + s->quadric_tests;
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  json_data_t js;
  if (rco_load_scene(argv[1], &js)) return 1;
  const int W = atoi(argv[2]), H = W, maxrec = atoi(argv[3]);
  rco_stats st, dep_st;
  octx c, cd;
  memset(&c, 0, sizeof c);
  memset(&st, 0, sizeof st);
  memset(&dep_st, 0, sizeof dep_st);
  c.st = &st;
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
  cd = c;               /* a second context for the DEP pixels' phase-A-only cost */
  cd.st = &dep_st;
  const float ph = js.camera_height / (float)H, pw = js.camera_width / (float)W;
  int *cost = calloc((size_t)W * H, sizeof(int));
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      float d[3];
      d[0] = (float)((0.0 - (double)js.camera_width / 2.0) + (double)pw * ((double)x + 0.5));
      d[1] = (float)((0.0 + (double)js.camera_height / 2.0) - (double)ph * ((double)y + 0.5));
      d[2] = -1.0f;
      o_normalize(&c, d, d);
      float col[3];
      pxinfo pi;
      const int64_t t0 = tests(&st);
      o_shoot(&c, d, maxrec, RCO_MODE_PARITY, col, &pi, NULL);
      int64_t n = tests(&st) - t0;
      if (pi.dep) {   /* phase A: primary level + first bounce (a miss), then deferred */
        memcpy(cd.carry, c.carry, sizeof cd.carry);
        const int64_t u0 = tests(&dep_st);
        o_shoot(&cd, d, 2, RCO_MODE_PARITY, col, &pi, NULL);
        n = tests(&dep_st) - u0;
      }
      cost[(size_t)y * W + x] = (int)n;
    }
  long long sum = 0, lock = 0;
  for (int ty = 0; ty < H; ty += 8)
    for (int tx = 0; tx < W; tx += 8) {
      int mx = 0, cnt = 0;
      for (int y = ty; y < ty + 8 && y < H; y++)
        for (int x = tx; x < tx + 8 && x < W; x++) {
          const int v = cost[(size_t)y * W + x];
          sum += v;
          mx = v > mx ? v : mx;
          ++cnt;
        }
      lock += (long long)mx * 64;
    }
  printf("%s %dx%d maxrec %d: %.2f shape tests per pixel in phase A, lane efficiency of 8x8 "
         "waves %.3f\n", argv[1], W, H, maxrec, (double)sum / ((double)W * H),
         (double)sum / (double)lock);
  return 0;
}
