/*
 * ppm.c — image output of the host front end.
 *
 * ppm_WriteOutP3 writes the byte stream of the reference's writer (C/ppm.c:168-184):
 *   "P3\n" "%d %d \n%u\n" (note the space before the newline), then one "%d\n" per
 * component, row-major.  Instead of 3*W*H fprintf calls it formats through a 256-entry
 * table of decimal strings into a large buffer (the reference's writer costs ~2 s at
 * 4096x4096 — SURVEY.md §8f row 2).
 */
#include <stdlib.h>
#include <string.h>

#include "raycast_hip.h"

float ppm_clamp(float value, float lower_bound, float upper_bound) {   /* C/ppm.c:350-359 */
  if (value > upper_bound) value = upper_bound;
  if (value < lower_bound) value = lower_bound;
  return value;
}

typedef struct {
  char txt[4];
  unsigned char len;
} dec_t;

void ppm_WriteOutP3(PPMFormat inData, FILE *outFile) {
  fprintf(outFile, "P3\n");
  fprintf(outFile, "%d %d \n%u\n", inData.width, inData.height, (unsigned)inData.maxColor);
  if (inData.width <= 0 || inData.height <= 0) return;
  static dec_t table[256];
  static int ready = 0;
  if (!ready) {
    for (int v = 0; v < 256; v++) {
      int n = snprintf(table[v].txt, sizeof table[v].txt, "%d", v);
      table[v].len = (unsigned char)n;
    }
    ready = 1;
  }
  const size_t total = (size_t)inData.width * (size_t)inData.height * 3;
  const size_t chunk = 1u << 20;   /* components per flush */
  char *buf = (char *)malloc(chunk * 4);
  if (!buf) {
    for (size_t k = 0; k < total; k++) fprintf(outFile, "%d\n", inData.pixmap[k]);
    return;
  }
  for (size_t base = 0; base < total; base += chunk) {
    const size_t end = base + chunk < total ? base + chunk : total;
    char *w = buf;
    for (size_t k = base; k < end; k++) {
      const dec_t *d = &table[inData.pixmap[k]];
      memcpy(w, d->txt, 4);   /* 4-byte copy, the tail is overwritten */
      w += d->len;
      *w++ = '\n';
    }
    fwrite(buf, 1, (size_t)(w - buf), outFile);
  }
  free(buf);
}
