/*
 * rc_oracle_cuda.c — TEST INFRASTRUCTURE ONLY (see rc_oracle.h).
 *
 * CPU restatement of the reference's CUDA port (CUDA/raycast.cu, CUDA/v3math.cu): SURVEY.md
 * §8 row f4, the "CUDA-semantics" render mode (RC_MODE_CUDA).  It differs from the C port in
 *   - control flow: per pixel, no carry; a reflection miss ends the bounce loop
 *     (CUDA/raycast.cu:224-237) and the loop runs up to MAX_ITER = 50 bounces (:13);
 *   - arithmetic: powf on floats where the C port calls pow on doubles
 *     (CUDA/raycast.cu:462-528,545,572,632-634; CUDA/v3math.cu:168), so squares, lengths and
 *     discriminants round to float before they are combined.
 *
 * Arithmetic contract (what "CUDA semantics" means here, the same in the HIP kernel):
 *   every float/double operation as the source writes it, C promotion rules, no FMA
 *   contraction; powf(x, y) is the correctly rounded float power: powf(x, 2) = x*x,
 *   powf(x, 0.5) = sqrtf(x) (CR), powf(a, 20) and integer spot exponents = (float) of the
 *   double power (glibc pow here; the device's exact double-double power, equal to it on
 *   every pinned parity config).
 * PARITY UNPINNED against the CUDA binary: nvcc is not in this image, nvcc's default
 * --fmad=true contracts a*b+c where it chooses (CUDA/Makefile:7 passes no --fmad=false) and
 * CUDA's powf is specified to 2 ulp, so the real port's bytes may differ from this contract in
 * the last bit of intermediate values.  The reference ships no CUDA-rendered image to pin it.
 * The CUDA kernel's shared-memory staging race (CUDA/raycast.cu:128-150) is not
 * modelled: every shape and light is used.
 */
#include "rc_oracle.h"

#include <math.h>
#include <string.h>

typedef struct {
  const shape_t *shapes;
  const light_t *lights;
  int n, m;
} cctx;

/* CUDA/v3math.cu:33-35 */
static float c_dot(const float *a, const float *b) {
  float s = a[0] * b[0];
  s = s + a[1] * b[1];
  return s + a[2] * b[2];
}
/* powf(x, 0.5): correctly rounded sqrt of a float */
static float c_sqrtf(float x) { return (float)sqrt((double)x); }
/* CUDA/v3math.cu:167-170: powf(powf(a0,2)+powf(a1,2)+powf(a2,2), 0.5), all in float */
static float c_length(const float *a) {
  float s = a[0] * a[0];
  s = s + a[1] * a[1];
  s = s + a[2] * a[2];
  return c_sqrtf(s);
}
/* CUDA/v3math.cu:172-185: no zero-length guard (IEEE quotients) */
static void c_normalize(float *dst, const float *a) {
  float len = c_length(a);
  float t0 = a[0] / len, t1 = a[1] / len, t2 = a[2] / len;
  dst[0] = t0; dst[1] = t1; dst[2] = t2;
}
/* CUDA/v3math.cu:104-121 */
static void c_reflect(float *dst, const float *v, const float *n) {
  float s = 2.0f * c_dot(v, n);
  float p0 = n[0] * s, p1 = n[1] * s, p2 = n[2] * s;
  dst[0] = v[0] - p0; dst[1] = v[1] - p1; dst[2] = v[2] - p2;
}

/* CUDA/raycast.cu:455-477 */
static int c_sphere(const float *O, const float *D, const shape_t *s, float *t) {
  float tv[3] = {O[0] - s->position[0], O[1] - s->position[1], O[2] - s->position[2]};
  float a = D[0] * D[0];
  a = a + D[1] * D[1];
  a = a + D[2] * D[2];
  float b = 2.0f * c_dot(D, tv);
  float c = c_dot(tv, tv) - s->radius * s->radius;
  float disc = b * b - (4.0f * a) * c;
  if (disc < 0.0f) return 0;
  double den = 2.0 * (double)a;
  float sq = c_sqrtf(disc);
  float tt = (float)((double)(-b - sq) / den);
  if (tt < 0.0f) tt = (float)((double)(-b + sq) / den);
  *t = tt;
  return 1;
}

/* CUDA/raycast.cu:535-552 (the same as C/raycast.c:545-562) */
static int c_plane(const float *O, const float *D, const shape_t *s, float *t) {
  float sub[3] = {O[0] - s->position[0], O[1] - s->position[1], O[2] - s->position[2]};
  float num = c_dot(sub, s->normal);
  float den = c_dot(D, s->normal);
  if (den == 0.0f) return 0;
  float tt = (-num) / den;
  if (tt < 0.0f) return 0;
  *t = tt;
  return 1;
}

/* CUDA/raycast.cu:491-532: a_q and c_q in float (powf), b_q in double as in the C port */
static int c_quadric(const float *O, const float *D, const shape_t *q, float *t) {
  float aq = q->a * (D[0] * D[0]);
  aq = aq + q->b * (D[1] * D[1]);
  aq = aq + q->c * (D[2] * D[2]);
  aq = aq + q->d * D[0] * D[1];
  aq = aq + q->e * D[0] * D[2];
  aq = aq + q->f * D[1] * D[2];

  double acc = 2.0 * (double)q->a * (double)O[0] * (double)D[0];
  acc = acc + 2.0 * (double)q->b * (double)O[1] * (double)D[1];
  acc = acc + 2.0 * (double)q->c * (double)O[2] * (double)D[2];
  acc = acc + (double)(q->d * (O[0] * D[1] + O[1] * D[0]));
  acc = acc + (double)(q->e * (O[0] * D[2] + O[2] * D[0]));
  acc = acc + (double)(q->f * (O[1] * D[2] + O[2] * D[1]));
  acc = acc + (double)(q->g * D[0]);
  acc = acc + (double)(q->h * D[1]);
  acc = acc + (double)(q->i * D[2]);
  float bq = (float)acc;

  float cq = q->a * (O[0] * O[0]);
  cq = cq + q->b * (O[1] * O[1]);
  cq = cq + q->c * (O[2] * O[2]);
  cq = cq + q->d * O[0] * O[1];
  cq = cq + q->e * O[0] * O[2];
  cq = cq + q->f * O[1] * O[2];
  cq = cq + q->g * O[0];
  cq = cq + q->h * O[1];
  cq = cq + q->i * O[2];
  cq = cq + q->j;

  if ((double)aq == 0.0) {                                     /* :517-519 */
    *t = (float)((-1.0 * (double)cq) / (double)bq);
    return 1;
  }
  float disc = (float)((double)(bq * bq) - 4.0 * (double)aq * (double)cq);
  if ((double)disc < 0.0) return 0;
  double den = 2.0 * (double)aq;
  float sq = c_sqrtf(disc);
  float tt = (float)((double)(-bq - sq) / den);
  if (tt <= 0.0f) tt = (float)((double)(-bq + sq) / den);
  *t = tt;
  return 1;
}

/* CUDA/raycast.cu:330-430 */
static int c_nearest(const cctx *c, const float *O, const float *D, float *P, float *N, int skip,
                     int shadow) {
  float best = INFINITY, t = 0.0f;
  int idx = -1;
  for (int k = 0; k < c->n; k++) {
    if (k == skip) continue;
    const shape_t *s = &c->shapes[k];
    int hit;
    if (s->type == SPHERE) hit = c_sphere(O, D, s, &t);
    else if (s->type == PLANE) hit = c_plane(O, D, s, &t);
    else if (s->type == QUADRIC) {
      hit = c_quadric(O, D, s, &t);
      if (hit && skip != -1 && (O[2] + t * D[2]) < O[2]) continue;   /* :388-390 */
    } else continue;
    if (!hit || !(best > t && t > 0.0f)) continue;
    best = t;
    idx = k;
    if (shadow) continue;
    float p0 = O[0] + D[0] * best, p1 = O[1] + D[1] * best, p2 = O[2] + D[2] * best;
    P[0] = p0; P[1] = p1; P[2] = p2;
    if (s->type == SPHERE) {
      float inv = (float)(1.0 / (double)s->radius);
      N[0] = (p0 - s->position[0]) * inv;
      N[1] = (p1 - s->position[1]) * inv;
      N[2] = (p2 - s->position[2]) * inv;
      c_normalize(N, N);
    } else if (s->type == PLANE) {
      N[0] = s->normal[0]; N[1] = s->normal[1]; N[2] = s->normal[2];
    } else {
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
      c_normalize(N, N);
      if (c_dot(N, D) > 0.0f) {
        N[0] = N[0] * -1.0f; N[1] = N[1] * -1.0f; N[2] = N[2] * -1.0f;
      }
    }
  }
  return idx;
}

/* CUDA/raycast.cu:260-302 with the attenuation / light terms of :544-634 */
static void c_shade(const cctx *c, float *out, int idx, const float *P, const float *N,
                    const float *D) {
  const shape_t *o = &c->shapes[idx];
  float opacity = (float)((1.0 - (double)o->reflectivity) - (double)o->refractivity);
  out[0] = out[1] = out[2] = 0.0f;
  if (!(opacity > 0.0f)) return;
  for (int l = 0; l < c->m; l++) {
    const light_t *L = &c->lights[l];
    float ld[3] = {L->position[0] - P[0], L->position[1] - P[1], L->position[2] - P[2]};
    float dist = c_length(ld);
    c_normalize(ld, ld);
    if (c_nearest(c, P, ld, NULL, NULL, idx, 1) != -1) continue;
    /* :544-546: float sum, double quotient */
    float den = L->radial_coef[0] + L->radial_coef[1] * dist;
    den = den + L->radial_coef[2] * (dist * dist);
    float rad = (float)(1.0 / (double)den);
    float ang = 1.0f;                                          /* :556-573 */
    if (L->type == SPOTLIGHT) {
      float v[3] = {P[0] - L->position[0], P[1] - L->position[1], P[2] - L->position[2]};
      c_normalize(v, v);
      float alpha = c_dot(v, L->direction);
      if (alpha < L->cos_theta) ang = 0.0f;
      else ang = (float)pow((double)alpha, (double)L->a0);
    }
    float dif[3] = {0, 0, 0}, spe[3] = {0, 0, 0};
    float th = c_dot(N, ld);
    if (!(th <= 0.0)) {
      for (int k = 0; k < 3; k++) dif[k] = (o->diffuse_color[k] * L->color[k]) * th;
      float view[3] = {D[0] * -1.0f, D[1] * -1.0f, D[2] * -1.0f};
      float r[3];
      c_reflect(r, ld, N);
      double angle = (double)c_dot(view, r);
      if (!(angle > 0.0)) {                                    /* :632-634: powf(float, 20) */
        float p20 = (float)pow(angle, 20.0);
        for (int k = 0; k < 3; k++) spe[k] = (o->specular_color[k] * L->color[k]) * p20;
      }
    }
    for (int k = 0; k < 3; k++) out[k] = out[k] + ((dif[k] + spe[k]) * rad) * ang;
  }
  out[0] = out[0] * opacity; out[1] = out[1] * opacity; out[2] = out[2] * opacity;
}

/* CUDA/raycast.cu:183-246 */
static void c_shoot(const cctx *c, const float *d, int max_iter, float *out) {
  float P0[3], N0[3];
  out[0] = out[1] = out[2] = 0.0f;
  const float zero[3] = {0.0f, 0.0f, 0.0f};
  int i0 = c_nearest(c, zero, d, P0, N0, -1, 0);
  if (i0 < 0) return;
  int obj = i0, S = i0;
  float O[3] = {P0[0], P0[1], P0[2]}, D[3] = {d[0], d[1], d[2]}, N[3] = {N0[0], N0[1], N0[2]};
  float T = c->shapes[i0].reflectivity, col[3], P[3];
  for (int iter = 0; iter < max_iter; iter++) {
    if (!(c->shapes[obj].reflectivity > 0.0f)) break;
    float r[3];
    c_reflect(r, D, N);
    c_normalize(r, r);
    D[0] = r[0]; D[1] = r[1]; D[2] = r[2];
    int i = c_nearest(c, O, D, P, N, S, 0);
    if (i < 0) break;                                          /* :236-238 */
    obj = i;
    c_shade(c, col, i, P, N, D);
    col[0] = col[0] * T; col[1] = col[1] * T; col[2] = col[2] * T;
    T = T * c->shapes[obj].reflectivity;
    out[0] = out[0] + col[0]; out[1] = out[1] + col[1]; out[2] = out[2] + col[2];
    O[0] = P[0]; O[1] = P[1]; O[2] = P[2];
    S = i;
  }
  c_shade(c, col, i0, P0, N0, d);                              /* :244-245 */
  out[0] = out[0] + col[0]; out[1] = out[1] + col[1]; out[2] = out[2] + col[2];
}

/* CUDA/ppm.cu:349-358 and the uint8_t store of CUDA/raycast.cu:166-168 */
static uint8_t c_quant(float v) {
  v = v * 255.0f;
  if (v > 255.0f) v = 255.0f;
  if (v < 0.0f) v = 0.0f;
  if (v != v) return 0;
  return (uint8_t)(int32_t)v;
}

int rco_render_cuda(const json_data_t *js, int width, int height, int max_iter,
                    uint8_t *pixmap) {
  if (width <= 0 || height <= 0 || max_iter < 0) return -1;
  shape_t shapes[256];
  light_t lights[256];
  cctx c = {shapes, lights, 0, 0};
  for (const shape_t *s = js->shapes_list; s && c.n < 256; s = s->next) shapes[c.n++] = *s;
  for (const light_t *l = js->lights_list; l && c.m < 256; l = l->next) lights[c.m++] = *l;
  const float pw = js->camera_width / width, ph = js->camera_height / height;
  for (int y = 0; y < height; y++) {
    for (int x = 0; x < width; x++) {                         /* :154-158 */
      float d[3];
      d[0] = (float)(0.0 - js->camera_width / 2.0 + (double)pw * ((double)x + 0.5));
      d[1] = (float)(0.0 + js->camera_height / 2.0 - (double)ph * ((double)y + 0.5));
      d[2] = -1.0f;
      c_normalize(d, d);
      float col[3];
      c_shoot(&c, d, max_iter, col);
      uint8_t *px = pixmap + ((size_t)y * width + x) * 3;
      px[0] = c_quant(col[0]);
      px[1] = c_quant(col[1]);
      px[2] = c_quant(col[2]);
    }
  }
  return 0;
}
