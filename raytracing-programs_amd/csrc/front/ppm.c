/*
 * ppm.c — image output of the host front end.
 *
 * ppm_WriteOutP3 writes the byte stream of the reference's writer (C/ppm.c:168-184):
 *   "P3\n" "%d %d \n%u\n" (note the space before the newline), then one "%d\n" per
 * component, row-major.  Instead of 3*W*H fprintf calls it formats through a 256-entry
 * table of decimal strings, several threads at a time, into large buffers (the reference's
 * writer costs ~2 s at 4096x4096 — SURVEY.md §8f row 2; this one ~6 ms of formatting).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

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

static dec_t g_table[256];
static pthread_once_t g_table_once = PTHREAD_ONCE_INIT;
static void init_table(void) {
  for (int v = 0; v < 256; v++) {
    int n = snprintf(g_table[v].txt, sizeof g_table[v].txt, "%d", v);
    g_table[v].len = (unsigned char)n;
  }
}

/* Formats components [begin, end) as "%d\n" lines into out; returns the byte count. */
static size_t format_range(const uint8_t *px, size_t begin, size_t end, char *out) {
  char *w = out;
  for (size_t k = begin; k < end; k++) {
    const dec_t *d = &g_table[px[k]];
    memcpy(w, d->txt, 4);   /* 4-byte copy, the tail is overwritten */
    w += d->len;
    *w++ = '\n';
  }
  return (size_t)(w - out);
}

typedef struct {
  const uint8_t *px;
  size_t begin, end, bytes;
  char *buf;
} fmt_job;

static void *format_job(void *arg) {
  fmt_job *j = (fmt_job *)arg;
  j->bytes = format_range(j->px, j->begin, j->end, j->buf);
  return NULL;
}

/* Byte-identical to the reference's writer; large images are formatted by several threads
 * (slices of a 16M-component block each), then written in order. */
void ppm_WriteOutP3(PPMFormat inData, FILE *outFile) {
  fprintf(outFile, "P3\n");
  fprintf(outFile, "%d %d \n%u\n", inData.width, inData.height, (unsigned)inData.maxColor);
  if (inData.width <= 0 || inData.height <= 0) return;
  pthread_once(&g_table_once, init_table);
  const size_t total = (size_t)inData.width * (size_t)inData.height * 3;
  enum { kMaxThreads = 16 };
  long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
  int nt = total >= ((size_t)1 << 20) ? (int)(ncpu < kMaxThreads ? ncpu : kMaxThreads) : 1;
  if (nt < 1) nt = 1;
  const size_t block = (size_t)1 << 24;             /* components per written block */
  const size_t slice = (block + (size_t)nt - 1) / (size_t)nt;
  char *bufs[kMaxThreads];
  int ok = 1;
  for (int t = 0; t < nt; t++) {
    bufs[t] = (char *)malloc(slice * 4);
    if (!bufs[t]) ok = 0;
  }
  if (!ok) {
    for (int t = 0; t < nt; t++) free(bufs[t]);
    for (size_t k = 0; k < total; k++) fprintf(outFile, "%d\n", inData.pixmap[k]);
    return;
  }
  for (size_t base = 0; base < total; base += block) {
    const size_t end = base + block < total ? base + block : total;
    fmt_job jobs[kMaxThreads];
    pthread_t th[kMaxThreads];
    int started[kMaxThreads] = {0};
    for (int t = 0; t < nt; t++) {
      size_t b = base + (size_t)t * slice, e = b + slice;
      if (b > end) b = end;
      if (e > end) e = end;
      jobs[t] = (fmt_job){inData.pixmap, b, e, 0, bufs[t]};
      if (t > 0 && e > b) started[t] = pthread_create(&th[t], NULL, format_job, &jobs[t]) == 0;
      if (t > 0 && e > b && !started[t]) format_job(&jobs[t]);
    }
    format_job(&jobs[0]);
    for (int t = 1; t < nt; t++)
      if (started[t]) pthread_join(th[t], NULL);
    for (int t = 0; t < nt; t++)
      if (jobs[t].bytes) fwrite(bufs[t], 1, jobs[t].bytes, outFile);
  }
  for (int t = 0; t < nt; t++) free(bufs[t]);
}
