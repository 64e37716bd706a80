/*
 * ref_timer.c — TEST INFRASTRUCTURE ONLY.  Timing driver for the reference render path.
 *
 * Linked (by oracle/Makefile) against the reference's own C/ sources compiled exactly as
 * C/Makefile:4 (gcc -O3) with the reference main renamed (-Dmain=ref_main).  Parses the
 * scene with the reference's parse_json (C/parse.c:13), then times ONLY raycast()
 * (C/raycast.c:79) with CLOCK_MONOTONIC, like SURVEY.md §8d.  Optionally writes the P3
 * with the reference's writer so the driver's output can be md5-checked against the stock
 * binary.
 *   ref_timer WIDTH HEIGHT SCENE [OUT.ppm]
 * Prints: {"seconds": s, "rays_per_s": r, "width": W, "height": H}
 */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <stdbool.h>
#include <time.h>

#include "raycast.h"   /* the reference's header (C/raycast.h), found via -I */

#undef main            /* -Dmain=ref_main renames only the reference's main */

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: ref_timer W H SCENE [OUT]\n");
    return 2;
  }
  int W = atoi(argv[1]), H = atoi(argv[2]);
  FILE *in = fopen(argv[3], "r");
  if (!in) { fprintf(stderr, "cannot open %s\n", argv[3]); return 1; }
  json_data_t *js = (json_data_t *)calloc(1, sizeof(json_data_t));
  parse_json(in, js);
  fclose(in);
  PPMFormat p;
  p.maxColor = 255;
  p.width = W;
  p.height = H;
  p.size = W * H * 3;
  p.depth = 0;
  p.tupleType = NULL;
  p.pixmap = (uint8_t *)malloc((size_t)p.size);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  raycast(js, p);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  double sec = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  if (argc > 4) {
    FILE *out = fopen(argv[4], "wb");
    if (!out) return 1;
    ppm_WriteOutP3(p, out);
    fclose(out);
  }
  printf("{\"seconds\": %.6f, \"rays_per_s\": %.1f, \"width\": %d, \"height\": %d}\n", sec,
         (double)W * H / sec, W, H);
  free(p.pixmap);
  return 0;
}
