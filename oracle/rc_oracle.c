/*
 * rc_oracle.c — TEST INFRASTRUCTURE ONLY (see rc_oracle.h).
 *
 * A from-scratch CPU restatement of the reference's per-pixel render semantics
 * (SURVEY.md Appendix A).  Every C promotion that the reference performs implicitly is
 * written out as an explicit cast, so the result does not depend on optimisation level:
 * build with -O2/-O3 -ffp-contract=off, no -march (x86-64 SSE2: no FMA, FLT_EVAL_METHOD 0).
 *
 * The two undefined behaviours the reference's output depends on are modelled explicitly:
 *   - the scan-order carry: `next_intersecion` (C/raycast.c:340) is never initialised and,
 *     with iterative_shoot inlined by gcc -O3, keeps the last bounce-hit point of earlier
 *     pixels.  Modelled as one float3 per render call, initially (0,0,0), written on every
 *     accepted bounce hit and read as the next ray origin (C/raycast.c:365) even on a miss.
 *   - the phantom: on a bounce miss calc_color reads shapes_list[-1] (C/raycast.c:360,382),
 *     the 104 bytes below the object VLA, which overlap the light VLA (C/raycast.c:87-89).
 *     Modelled by rebuilding those bytes from the light records.
 * libm: pow/sqrt/cos are the host libm's, exactly the calls the reference makes.
 */
#include "rc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ render context -- */
typedef struct {
  const shape_t *shapes;   /* n records in file order (copied from the list)          */
  const light_t *lights;   /* m records                                               */
  int n, m;
  shape_t phantom;         /* shapes_list[-1]                                          */
  int phantom_defined;     /* every byte calc_color reads from the phantom is defined  */
  float carry[3];          /* next_intersecion, persistent across pixels              */
  rco_stats *st;
} octx;

/* ---------------------------------------------------------- v3 helpers (C/v3math.c) -- */
/* C/v3math.c:69-71 */
static float o_dot(const float *a, const float *b) {
  float s = a[0] * b[0];
  s = s + a[1] * b[1];
  return s + a[2] * b[2];
}
/* C/v3math.c:169-172: (float)sqrt(pow(a0,2)+pow(a1,2)+pow(a2,2)); pow(x,2) is an exact
 * double square (gcc folds it). */
static float o_length(const float *a) {
  double s = (double)a[0] * (double)a[0];
  s = s + (double)a[1] * (double)a[1];
  s = s + (double)a[2] * (double)a[2];
  return (float)sqrt(s);
}
/* C/v3math.c:180-192: a zero length leaves dst untouched (after a stderr message). */
static void o_normalize(octx *c, float *dst, const float *a) {
  float len = o_length(a);
  if (len == 0.0f) {
    c->st->zero_normalize++;
    return;
  }
  float t0 = a[0] / len, t1 = a[1] / len, t2 = a[2] / len;
  dst[0] = t0; dst[1] = t1; dst[2] = t2;
}
/* C/v3math.c:144-160: v - n*(2*dot(v,n)) */
static void o_reflect(float *dst, const float *v, const float *n) {
  float s = 2.0f * o_dot(v, n);
  float p0 = n[0] * s, p1 = n[1] * s, p2 = n[2] * s;
  dst[0] = v[0] - p0; dst[1] = v[1] - p1; dst[2] = v[2] - p2;
}

/* --------------------------------------------------- intersections (C/raycast.c) -- */
/* C/raycast.c:545-562 */
static int o_plane(const float *O, const float *D, const shape_t *s, float *t) {
  float sub[3] = {O[0] - s->position[0], O[1] - s->position[1], O[2] - s->position[2]};
  float num = o_dot(sub, s->normal);
  float den = o_dot(D, s->normal);
  if (den == 0.0f) return 0;
  float tt = (-num) / den;              /* -1 * num is exact negation */
  if (tt < 0.0f) return 0;
  *t = tt;
  return 1;
}

/* C/raycast.c:576-600 */
static int o_sphere(const float *O, const float *D, const shape_t *s, float *t) {
  float tv[3] = {O[0] - s->position[0], O[1] - s->position[1], O[2] - s->position[2]};
  double aa = (double)D[0] * (double)D[0];
  aa = aa + (double)D[1] * (double)D[1];
  aa = aa + (double)D[2] * (double)D[2];
  float a = (float)aa;
  float b = 2.0f * o_dot(D, tv);
  float c = (float)((double)o_dot(tv, tv) - (double)s->radius * (double)s->radius);
  float fac = (4.0f * a) * c;
  float disc = (float)((double)b * (double)b - (double)fac);
  if (disc < 0.0f) return 0;
  double den = 2.0 * (double)a;
  float tt = (float)(((double)(-b) - pow((double)disc, 0.5)) / den);
  if (tt < 0.0f) tt = (float)(((double)(-b) + pow((double)disc, 0.5)) / den);
  *t = tt;
  return 1;
}

/* Diagnostic for the tests (not part of the reference's algorithm): tests of a quadric without
 * cross terms (d = e = f = 0) in which a cross term is NaN — the case the HIP kernels handle by
 * rejecting the quadric (rc_device.hpp x0_reject).  Not thread-safe; read by the tests only. */
static long long g_cross_nan;
long long rco_cross_nan_events(int reset) {
  long long v = g_cross_nan;
  if (reset) g_cross_nan = 0;
  return v;
}

/* C/raycast.c:614-656 — the double accumulations follow the source's left-to-right order */
static int o_quadric(const float *O, const float *D, const shape_t *q, float *t) {
  if (q->d == 0.0f && q->e == 0.0f && q->f == 0.0f &&
      (isnan(q->d * D[0] * D[1]) || isnan(q->e * D[0] * D[2]) || isnan(q->f * D[1] * D[2]) ||
       isnan(q->d * (O[0] * D[1] + O[1] * D[0])) || isnan(q->e * (O[0] * D[2] + O[2] * D[0])) ||
       isnan(q->f * (O[1] * D[2] + O[2] * D[1])) || isnan(q->d * O[0] * O[1]) ||
       isnan(q->e * O[0] * O[2]) || isnan(q->f * O[1] * O[2])))
    g_cross_nan++;
  const double A = q->a, B = q->b, C = q->c;
  double acc;
  /* a_q (C/raycast.c:615-617) */
  acc = A * ((double)D[0] * (double)D[0]);
  acc = acc + B * ((double)D[1] * (double)D[1]);
  acc = acc + C * ((double)D[2] * (double)D[2]);
  acc = acc + (double)(q->d * D[0] * D[1]);
  acc = acc + (double)(q->e * D[0] * D[2]);
  acc = acc + (double)(q->f * D[1] * D[2]);
  float aq = (float)acc;
  /* b_q (C/raycast.c:619-627) */
  acc = 2.0 * A * (double)O[0] * (double)D[0];
  acc = acc + 2.0 * B * (double)O[1] * (double)D[1];
  acc = acc + 2.0 * C * (double)O[2] * (double)D[2];
  acc = acc + (double)(q->d * (O[0] * D[1] + O[1] * D[0]));
  acc = acc + (double)(q->e * (O[0] * D[2] + O[2] * D[0]));
  acc = acc + (double)(q->f * (O[1] * D[2] + O[2] * D[1]));
  acc = acc + (double)(q->g * D[0]);
  acc = acc + (double)(q->h * D[1]);
  acc = acc + (double)(q->i * D[2]);
  float bq = (float)acc;
  /* c_q (C/raycast.c:629-638) */
  acc = A * ((double)O[0] * (double)O[0]);
  acc = acc + B * ((double)O[1] * (double)O[1]);
  acc = acc + C * ((double)O[2] * (double)O[2]);
  acc = acc + (double)(q->d * O[0] * O[1]);
  acc = acc + (double)(q->e * O[0] * O[2]);
  acc = acc + (double)(q->f * O[1] * O[2]);
  acc = acc + (double)(q->g * O[0]);
  acc = acc + (double)(q->h * O[1]);
  acc = acc + (double)(q->i * O[2]);
  acc = acc + (double)q->j;
  float cq = (float)acc;

  if ((double)aq == 0.0) {                                   /* C/raycast.c:640-642 */
    *t = (float)((-1.0 * (double)cq) / (double)bq);
    return 1;
  }
  float disc = (float)((double)bq * (double)bq - 4.0 * (double)aq * (double)cq);
  if ((double)disc < 0.0) return 0;
  double den = 2.0 * (double)aq;
  float tt = (float)(((double)(-bq) - pow((double)disc, 0.5)) / den);
  if (tt <= 0.0f) tt = (float)(((double)(-bq) + pow((double)disc, 0.5)) / den);
  *t = tt;
  return 1;
}

/* -------------------------------------------- nearest hit (C/raycast.c:441-531) -- */
static int o_nearest(octx *c, const float *O, const float *D, float *P, float *N, int skip,
                     int shadow) {
  float best = INFINITY, t = 0.0f;
  int idx = -1;
  if (shadow) c->st->shadow_rays++; else c->st->nearest_calls++;
  for (int k = 0; k < c->n; k++) {
    if (k == skip) continue;
    const shape_t *s = &c->shapes[k];
    int hit;
    if (s->type == SPHERE) {
      c->st->sphere_tests++;
      hit = o_sphere(O, D, s, &t);
    } else if (s->type == PLANE) {
      c->st->plane_tests++;
      hit = o_plane(O, D, s, &t);
    } else if (s->type == QUADRIC) {
      c->st->quadric_tests++;
      hit = o_quadric(O, D, s, &t);
      /* C/raycast.c:492-494: hits "behind" the origin in z are ignored for bounce rays */
      if (hit && skip != -1 && (O[2] + t * D[2]) < O[2]) continue;
    } else {
      continue;
    }
    if (!hit) continue;
    if (!(best > t && t > 0.0f)) continue;
    best = t;
    idx = k;
    if (shadow) continue;
    float p0 = O[0] + D[0] * best, p1 = O[1] + D[1] * best, p2 = O[2] + D[2] * best;
    P[0] = p0; P[1] = p1; P[2] = p2;
    if (s->type == SPHERE) {                                   /* :465-469 */
      float inv = (float)(1.0 / (double)s->radius);
      N[0] = (p0 - s->position[0]) * inv;
      N[1] = (p1 - s->position[1]) * inv;
      N[2] = (p2 - s->position[2]) * inv;
      o_normalize(c, N, N);
    } else if (s->type == PLANE) {                             /* :484 */
      N[0] = s->normal[0]; N[1] = s->normal[1]; N[2] = s->normal[2];
    } else {                                                   /* :504-523 */
      double n0 = 2.0 * (double)s->a * (double)p0;
      n0 = n0 + (double)(s->d * p1);
      n0 = n0 + (double)(s->e * p2);
      n0 = n0 + (double)s->g;
      double n1 = 2.0 * (double)s->b * (double)p1;
      n1 = n1 + (double)(s->d * p0);
      n1 = n1 + (double)(s->f * p2);
      n1 = n1 + (double)s->h;
      double n2 = 2.0 * (double)s->c * (double)p2;
      n2 = n2 + (double)(s->e * p0);
      n2 = n2 + (double)(s->f * p1);
      n2 = n2 + (double)s->i;
      N[0] = (float)n0; N[1] = (float)n1; N[2] = (float)n2;
      o_normalize(c, N, N);
      if (o_dot(N, D) > 0.0f) {
        N[0] = N[0] * -1.0f; N[1] = N[1] * -1.0f; N[2] = N[2] * -1.0f;
      }
    }
  }
  return idx;
}

/* ------------------------------------------------ shading (C/raycast.c:381-421) -- */
static void o_shade(octx *c, float *out, int idx, const float *P, const float *N,
                    const float *D) {
  const shape_t *o = (idx >= 0) ? &c->shapes[idx] : &c->phantom;
  if (idx < 0) c->st->phantom_shades++;
  float opacity = (float)((1.0 - (double)o->reflectivity) - (double)o->refractivity);
  out[0] = out[1] = out[2] = 0.0f;
  if (!(opacity > 0.0f)) return;
  if (idx < 0 && !c->phantom_defined) c->st->parity_defined = 0;
  c->st->shaded_hits++;
  for (int l = 0; l < c->m; l++) {
    const light_t *L = &c->lights[l];
    float ld[3] = {L->position[0] - P[0], L->position[1] - P[1], L->position[2] - P[2]};
    float dist = o_length(ld);
    o_normalize(c, ld, ld);
    if (o_nearest(c, P, ld, NULL, NULL, idx, 1) != -1) continue;   /* in shadow */
    c->st->light_evals++;
    /* radial attenuation C/raycast.c:666-669 */
    float lin = L->radial_coef[0] + L->radial_coef[1] * dist;
    float rad = (float)(1.0 / ((double)lin + (double)L->radial_coef[2] *
                                                 ((double)dist * (double)dist)));
    /* angular attenuation C/raycast.c:679-696 */
    float ang = 1.0f;
    if (L->type == SPOTLIGHT) {
      float v[3] = {P[0] - L->position[0], P[1] - L->position[1], P[2] - L->position[2]};
      o_normalize(c, v, v);
      float alpha = o_dot(v, L->direction);
      if (alpha < L->cos_theta) ang = 0.0f;
      else ang = (float)pow((double)alpha, (double)L->a0);
    }
    /* diffuse C/raycast.c:708-720 and specular C/raycast.c:733-758 */
    float dif[3] = {0, 0, 0}, spe[3] = {0, 0, 0};
    float th = o_dot(N, ld);
    if (!(th <= 0.0)) {   /* C/raycast.c:713,740: a NaN theta is not <= 0 */
      for (int k = 0; k < 3; k++) dif[k] = (o->diffuse_color[k] * L->color[k]) * th;
      float view[3] = {D[0] * -1.0f, D[1] * -1.0f, D[2] * -1.0f};
      float r[3];
      o_reflect(r, ld, N);
      double angle = (double)o_dot(view, r);
      if (!(angle > 0.0)) {
        double p20 = pow(angle, 20.0);
        for (int k = 0; k < 3; k++)
          spe[k] = (float)((double)(o->specular_color[k] * L->color[k]) * p20);
      }
    }
    for (int k = 0; k < 3; k++) out[k] = out[k] + ((dif[k] + spe[k]) * rad) * ang;
  }
  out[0] = out[0] * opacity; out[1] = out[1] * opacity; out[2] = out[2] * opacity;
}

/* ------------------------------------- per-pixel shade (C/raycast.c:315-379) -- */
typedef struct { int dep, wrote; } pxinfo;

static void o_shoot(octx *c, const float *d, int maxrec, int mode, float *out, pxinfo *pi,
                    float *cin) {
  float P0[3], N0[3];
  out[0] = out[1] = out[2] = 0.0f;
  pi->dep = 0; pi->wrote = 0;
  int i0 = o_nearest(c, (const float[3]){0.0f, 0.0f, 0.0f}, d, P0, N0, -1, 0);
  if (i0 < 0) return;                                          /* :328-331 */

  int obj = i0, S = i0;
  float O[3] = {P0[0], P0[1], P0[2]};
  float D[3] = {d[0], d[1], d[2]};
  float N[3] = {N0[0], N0[1], N0[2]};
  float T = c->shapes[i0].reflectivity;
  float col[3];
  for (int lvl = 1; lvl < maxrec; lvl++) {                     /* :348-376 */
    if (!(c->shapes[obj].reflectivity > 0.0f)) break;
    c->st->bounce_iters++;
    float r[3];
    o_reflect(r, D, N);
    o_normalize(c, r, r);
    D[0] = r[0]; D[1] = r[1]; D[2] = r[2];
    int i = o_nearest(c, O, D, c->carry, N, S, 0);            /* writes the carry on hit */
    if (i < 0) {
      if (mode == RCO_MODE_FAST) break;                        /* CUDA/raycast.cu:224-237 */
      if (lvl == 1) {                                          /* reads another pixel's carry */
        pi->dep = 1;
        if (cin) { cin[0] = c->carry[0]; cin[1] = c->carry[1]; cin[2] = c->carry[2]; }
      }
    } else {
      obj = i;
      pi->wrote = 1;
    }
    o_shade(c, col, i, c->carry, N, D);
    col[0] = col[0] * T; col[1] = col[1] * T; col[2] = col[2] * T;
    T = T * c->shapes[obj].reflectivity;
    out[0] = out[0] + col[0]; out[1] = out[1] + col[1]; out[2] = out[2] + col[2];
    O[0] = c->carry[0]; O[1] = c->carry[1]; O[2] = c->carry[2];
    S = i;
  }
  o_shade(c, col, i0, P0, N0, d);                              /* :377-378 */
  out[0] = out[0] + col[0]; out[1] = out[1] + col[1]; out[2] = out[2] + col[2];
}

/* ppm_clamp (C/ppm.c:350-359) then the float -> uint8_t store (C/raycast.c:124-126).
 * x86-64 converts through cvttss2si: NaN -> 0x80000000, low byte 0. */
static uint8_t o_quant(float v) {
  v = v * 255.0f;
  if (v > 255.0f) v = 255.0f;
  if (v < 0.0f) v = 0.0f;
  if (v != v) return 0;
  return (uint8_t)(int32_t)v;
}

/* ------------------------------- phantom record (C/raycast.c:87-89,382) ---------- */
/* gcc allocates object_array then light_array below it, each VLA rounded to 16 bytes, so
 * shapes_list[-1] covers light-VLA bytes [R-104, R), R = (72m+15)&~15.  Bytes outside the
 * light records (stack garbage, padding), list pointers and the fields add_new_point_light
 * leaves uninitialised are "undefined": modelled as zero and tracked. */
static void o_build_phantom(octx *c) {
  unsigned char img[sizeof(shape_t)];
  unsigned char def[sizeof(shape_t)];
  const long m = c->m;
  const long R = (72 * m + 15) & ~15L;
  memset(img, 0, sizeof img);
  for (long o = 0; o < (long)sizeof(shape_t); o++) {
    long off = R - (long)sizeof(shape_t) + o;
    def[o] = 0;
    if (off < 0 || off >= 72 * m) continue;
    const light_t *L = &c->lights[off / 72];
    long lo = off % 72;
    light_t tmp;
    memcpy(&tmp, L, sizeof tmp);
    tmp.next = (off / 72 == m - 1) ? NULL : tmp.next;
    img[o] = ((const unsigned char *)&tmp)[lo];
    int defined = 1;
    if (lo >= 64) defined = (off / 72 == m - 1);                  /* next pointer          */
    if (L->type == POINT && lo >= 36 && lo < 60) defined = 0;     /* uninitialised fields */
    if (!defined) img[o] = 0;
    def[o] = (unsigned char)defined;
  }
  memcpy(&c->phantom, img, sizeof(shape_t));
  c->phantom.next = NULL;
  /* calc_color reads diffuse[0..12), specular[12..24), reflectivity[36..40),
   * refractivity[40..44) (C/raycast.c:382-383,408-412). */
  int all = 1;
  for (int o = 0; o < 24; o++) all &= def[o];
  for (int o = 36; o < 44; o++) all &= def[o];
  c->phantom_defined = all || m == 0;   /* no lights: the shade is black regardless */
}

int rco_render(const json_data_t *js, int width, int height, int max_recursion, int mode,
               uint8_t *pixmap, rco_stats *stats, float *carry_in) {
  return rco_render_cls(js, width, height, max_recursion, mode, pixmap, stats, carry_in, NULL);
}

int rco_render_cls(const json_data_t *js, int width, int height, int max_recursion, int mode,
                   uint8_t *pixmap, rco_stats *stats, float *carry_in, uint8_t *cls) {
  rco_stats local;
  octx c;
  memset(&c, 0, sizeof c);
  memset(&local, 0, sizeof local);
  c.st = stats ? stats : &local;
  memset(c.st, 0, sizeof *c.st);
  c.st->parity_defined = 1;
  c.n = js->num_shapes;
  c.m = js->num_lights;
  shape_t *sh = (shape_t *)calloc((size_t)(c.n > 0 ? c.n : 1), sizeof(shape_t));
  light_t *li = (light_t *)calloc((size_t)(c.m > 0 ? c.m : 1), sizeof(light_t));
  if (!sh || !li) { free(sh); free(li); return -1; }
  const shape_t *s = js->shapes_list;
  for (int k = 0; k < c.n; k++) { if (!s) { free(sh); free(li); return -2; } sh[k] = *s; s = s->next; }
  const light_t *l = js->lights_list;
  for (int k = 0; k < c.m; k++) { if (!l) { free(sh); free(li); return -2; } li[k] = *l; l = l->next; }
  c.shapes = sh;
  c.lights = li;
  o_build_phantom(&c);

  /* C/raycast.c:109-110 */
  const float ph = js->camera_height / (float)height;
  const float pw = js->camera_width / (float)width;
  int64_t seg = 0;
  uint8_t *px = pixmap;
  for (int y = 0; y < height; y++) {
    for (int x = 0; x < width; x++) {
      float d[3];
      d[0] = (float)((0.0 - (double)js->camera_width / 2.0) + (double)pw * ((double)x + 0.5));
      d[1] = (float)((0.0 + (double)js->camera_height / 2.0) - (double)ph * ((double)y + 0.5));
      d[2] = -1.0f;
      o_normalize(&c, d, d);
      float col[3];
      pxinfo pi;
      float *cin = carry_in ? &carry_in[3 * ((size_t)y * width + x)] : NULL;
      if (cin) cin[0] = cin[1] = cin[2] = 0.0f;
      o_shoot(&c, d, max_recursion, mode, col, &pi, cin);
      if (cls) cls[(size_t)y * width + x] = (uint8_t)(pi.dep ? (pi.wrote ? 3 : 2) : (pi.wrote ? 1 : 0));
      if (pi.dep) {
        c.st->dep_pixels++;
        if (pi.wrote) c.st->dep_writers++;
        seg++;
        if (seg > c.st->longest_segment) c.st->longest_segment = seg;
      } else if (pi.wrote) {
        c.st->indep_writers++;
        seg = 0;
      }
      px[0] = o_quant(col[0]);
      px[1] = o_quant(col[1]);
      px[2] = o_quant(col[2]);
      px += 3;
    }
  }
  free(sh);
  free(li);
  return 0;
}

/* Selected pixels, each from a given carry-in (the row-shard protocol model, tests/
 * test_dist.py): the pixel's colour, carry-out (next_intersecion after it), class (as in
 * rco_render_cls) and zero-normalize events.  carry_in NULL = (0,0,0) for every pixel. */
int rco_pixels(const json_data_t *js, int width, int height, int max_recursion, int mode,
               int64_t n, const int64_t *pix, const float *carry_in, uint8_t *rgb,
               float *carry_out, uint8_t *cls, int64_t *zero_events) {
  rco_stats st;
  octx c;
  memset(&c, 0, sizeof c);
  memset(&st, 0, sizeof st);
  c.st = &st;
  c.n = js->num_shapes;
  c.m = js->num_lights;
  shape_t *sh = (shape_t *)calloc((size_t)(c.n > 0 ? c.n : 1), sizeof(shape_t));
  light_t *li = (light_t *)calloc((size_t)(c.m > 0 ? c.m : 1), sizeof(light_t));
  if (!sh || !li) { free(sh); free(li); return -1; }
  const shape_t *s = js->shapes_list;
  for (int k = 0; k < c.n; k++) { if (!s) { free(sh); free(li); return -2; } sh[k] = *s; s = s->next; }
  const light_t *l = js->lights_list;
  for (int k = 0; k < c.m; k++) { if (!l) { free(sh); free(li); return -2; } li[k] = *l; l = l->next; }
  c.shapes = sh;
  c.lights = li;
  o_build_phantom(&c);
  const float ph = js->camera_height / (float)height;   /* C/raycast.c:109-110 */
  const float pw = js->camera_width / (float)width;
  for (int64_t i = 0; i < n; i++) {
    const int x = (int)(pix[i] % width), y = (int)(pix[i] / width);
    float d[3];
    d[0] = (float)((0.0 - (double)js->camera_width / 2.0) + (double)pw * ((double)x + 0.5));
    d[1] = (float)((0.0 + (double)js->camera_height / 2.0) - (double)ph * ((double)y + 0.5));
    d[2] = -1.0f;
    const int64_t z0 = st.zero_normalize;
    o_normalize(&c, d, d);
    for (int k = 0; k < 3; k++) c.carry[k] = carry_in ? carry_in[3 * i + k] : 0.0f;
    float col[3];
    pxinfo pi;
    o_shoot(&c, d, max_recursion, mode, col, &pi, NULL);
    for (int k = 0; k < 3; k++) {
      rgb[3 * i + k] = o_quant(col[k]);
      carry_out[3 * i + k] = c.carry[k];
    }
    cls[i] = (uint8_t)(pi.dep ? (pi.wrote ? 3 : 2) : (pi.wrote ? 1 : 0));
    if (zero_events) zero_events[i] = st.zero_normalize - z0;
  }
  free(sh);
  free(li);
  return 0;
}

/* ------------------------------------------------ minimal scene reader (tests) -- */
/* Reads the reference scene grammar (C/parse.c): one object per line, comma separated
 * `key: value` fields, vectors as [x, y, z].  Well-formed files only; no validation. */
static void o_trim(char *s) {
  size_t n = strlen(s);
  while (n && (s[n - 1] == ' ' || s[n - 1] == '\r' || s[n - 1] == '\t')) s[--n] = 0;
  size_t k = 0;
  while (s[k] == ' ' || s[k] == '\t') k++;
  if (k) memmove(s, s + k, strlen(s + k) + 1);
}

int rco_load_scene(const char *path, json_data_t *js) {
  FILE *f = fopen(path, "r");
  if (!f) return -1;
  memset(js, 0, sizeof *js);
  char line[4096];
  shape_t **stail = &js->shapes_list;
  light_t **ltail = &js->lights_list;
  while (fgets(line, sizeof line, f)) {
    /* split fields on commas outside brackets */
    char *fields[64];
    int nf = 0, depth = 0;
    char *p = line, *start = line;
    for (;; p++) {
      if (*p == '[') depth++;
      if (*p == ']') depth--;
      if ((*p == ',' && depth == 0) || *p == '\n' || *p == 0) {
        int end = (*p == '\n' || *p == 0);
        *p = 0;
        if (nf < 64) fields[nf++] = start;
        start = p + 1;
        if (end) break;
      }
    }
    if (nf == 0) continue;
    o_trim(fields[0]);
    const char *type = fields[0];
    float v3d[3] = {0, 0, 0}, v3s[3] = {0, 0, 0};
    shape_t sh; light_t lt;
    memset(&sh, 0, sizeof sh); memset(&lt, 0, sizeof lt);
    float theta = 0.0f;
    for (int k = 1; k < nf; k++) {
      char *colon = strchr(fields[k], ':');
      if (!colon) continue;
      *colon = 0;
      char *key = fields[k], *val = colon + 1;
      o_trim(key); o_trim(val);
      float vec[3] = {0, 0, 0}, sc = 0.0f;
      int isvec = (val[0] == '[');
      if (isvec) sscanf(val, "[%f, %f, %f]", &vec[0], &vec[1], &vec[2]);
      else sscanf(val, "%f", &sc);
      if (!strcmp(type, "camera")) {
        if (!strcmp(key, "width")) js->camera_width = sc;
        if (!strcmp(key, "height")) js->camera_height = sc;
      } else if (!strcmp(type, "light")) {
        if (!strcmp(key, "color")) memcpy(lt.color, vec, sizeof vec);
        else if (!strcmp(key, "position")) memcpy(lt.position, vec, sizeof vec);
        else if (!strcmp(key, "direction")) memcpy(lt.direction, vec, sizeof vec);
        else if (!strcmp(key, "theta")) theta = sc;
        else if (!strcmp(key, "radial-a0")) lt.radial_coef[0] = sc;
        else if (!strcmp(key, "radial-a1")) lt.radial_coef[1] = sc;
        else if (!strcmp(key, "radial-a2")) lt.radial_coef[2] = sc;
        else if (!strcmp(key, "angular-a0")) lt.a0 = sc;
      } else {
        if (!strcmp(key, "diffuse_color")) memcpy(v3d, vec, sizeof vec);
        else if (!strcmp(key, "specular_color")) memcpy(v3s, vec, sizeof vec);
        else if (!strcmp(key, "position")) memcpy(sh.position, vec, sizeof vec);
        else if (!strcmp(key, "normal") && !strcmp(type, "plane")) memcpy(sh.normal, vec, sizeof vec);
        else if (!strcmp(key, "radius") && !strcmp(type, "sphere")) sh.radius = sc;
        else if (!strcmp(key, "reflectivity")) sh.reflectivity = sc;
        else if (!strcmp(key, "refractivity")) sh.refractivity = sc;
        else if (!strcmp(key, "ior")) sh.ior = sc;
        else if (strlen(key) == 1 && key[0] >= 'a' && key[0] <= 'j' && !strcmp(type, "quadric"))
          (&sh.a)[key[0] - 'a'] = sc;
      }
    }
    if (!strcmp(type, "sphere") || !strcmp(type, "plane") || !strcmp(type, "quadric")) {
      memcpy(sh.diffuse_color, v3d, sizeof v3d);
      memcpy(sh.specular_color, v3s, sizeof v3s);
      if (!strcmp(type, "sphere")) sh.type = SPHERE;
      if (!strcmp(type, "plane")) { sh.type = PLANE; sh.refractivity = 0; sh.ior = 1; }
      if (!strcmp(type, "quadric")) { sh.type = QUADRIC; sh.refractivity = 0; sh.ior = 1; }
      shape_t *node = (shape_t *)malloc(sizeof(shape_t));
      *node = sh; node->next = NULL;
      *stail = node; stail = &node->next;
      js->num_shapes++;
    } else if (!strcmp(type, "light")) {
      if (theta != 0.0f) {
        /* C/parse.c:282 converts with 180/PI (PI = 3.141592654f, C/v3math.c:11);
         * C/objects.c:179 stores cos(theta). */
        const float PI_f = 3.141592654f;
        theta = (float)((double)theta * (180.0 / (double)PI_f));
        lt.theta = theta;
        lt.cos_theta = (float)cos((double)theta);
        lt.type = SPOTLIGHT;
      } else {
        lt.type = POINT;
        lt.a0 = 0.0f; memset(lt.direction, 0, sizeof lt.direction);
      }
      light_t *node = (light_t *)malloc(sizeof(light_t));
      *node = lt; node->next = NULL;
      *ltail = node; ltail = &node->next;
      js->num_lights++;
    }
  }
  fclose(f);
  return 0;
}

void rco_free_scene(json_data_t *js) {
  shape_t *s = js->shapes_list;
  while (s) { shape_t *n = s->next; free(s); s = n; }
  light_t *l = js->lights_list;
  while (l) { light_t *n = l->next; free(l); l = n; }
  js->shapes_list = NULL;
  js->lights_list = NULL;
}
