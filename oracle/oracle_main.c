/*
 * oracle_main.c — TEST INFRASTRUCTURE ONLY.  CLI around the CPU restatement:
 *   oracle_raytrace WIDTH HEIGHT INPUT_SCENE OUTPUT_IMAGE [DEPTH] [parity|fast]
 * Writes the same P3 PPM the reference writes (C/ppm.c:168-184) and prints a JSON stats
 * line on stdout (per-pixel work counts used for SURVEY §8a / the roofline).
 */
#include "rc_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

int main(int argc, char **argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: oracle_raytrace W H SCENE OUT [DEPTH] [parity|fast]\n");
    return 2;
  }
  int W = atoi(argv[1]), H = atoi(argv[2]);
  int depth = argc > 5 ? atoi(argv[5]) : 6;
  int mode = (argc > 6 && !strcmp(argv[6], "fast")) ? RCO_MODE_FAST : RCO_MODE_PARITY;
  json_data_t js;
  if (rco_load_scene(argv[3], &js)) {
    fprintf(stderr, "cannot read %s\n", argv[3]);
    return 1;
  }
  uint8_t *px = (uint8_t *)malloc((size_t)W * H * 3);
  rco_stats st;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  rco_render(&js, W, H, depth + 1, mode, px, &st, NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  double sec = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  FILE *f = fopen(argv[4], "wb");
  if (!f) return 1;
  fprintf(f, "P3\n%d %d \n%u\n", W, H, 255u);
  for (size_t k = 0; k < (size_t)W * H * 3; k++) fprintf(f, "%d\n", px[k]);
  fclose(f);
  double np = (double)W * H;
  printf("{\"seconds\": %.6f, \"rays_per_s\": %.1f, \"sphere_tests_px\": %.4f, "
         "\"plane_tests_px\": %.4f, \"quadric_tests_px\": %.4f, \"nearest_px\": %.4f, "
         "\"shadow_px\": %.4f, \"bounce_px\": %.4f, \"shaded_px\": %.4f, \"light_evals_px\": %.4f, "
         "\"dep_pixels\": %lld, \"dep_writers\": %lld, \"indep_writers\": %lld, "
         "\"longest_segment\": %lld, \"zero_normalize\": %lld, \"phantom_shades\": %lld, "
         "\"parity_defined\": %d}\n",
         sec, np / sec, st.sphere_tests / np, st.plane_tests / np, st.quadric_tests / np,
         st.nearest_calls / np, st.shadow_rays / np, st.bounce_iters / np, st.shaded_hits / np,
         st.light_evals / np, (long long)st.dep_pixels, (long long)st.dep_writers,
         (long long)st.indep_writers, (long long)st.longest_segment,
         (long long)st.zero_normalize, (long long)st.phantom_shades, st.parity_defined);
  free(px);
  rco_free_scene(&js);
  return 0;
}
