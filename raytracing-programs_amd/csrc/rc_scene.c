/*
 * rc_scene.c — host side of the drop-in boundary: flatten the reference's scene lists into
 * the packed image the kernels read (layout: rc_scene.h).
 *
 * Replaces the list -> VLA copy of C/raycast.c:87-102.  The values stored are produced by
 * the same IEEE operations the reference performs at its use sites, so the device reads
 * bit-identical numbers.
 *
 * Phantom record (C/raycast.c:360,382): on a reflection miss the reference shades
 * shapes_list[-1], i.e. the 104 bytes just below the object VLA.  With gcc's VLA placement
 * (object array above the light array, each rounded to 16 B) these are the bytes
 * [R-104, R) of the light VLA, R = (72m+15) & ~15.  The light VLA holds
 * verbatim copies of the list nodes (C/raycast.c:100).  Bytes that are not reproducible
 * from the scene (stack garbage below the light VLA, VLA padding, heap pointers, the
 * fields add_new_point_light leaves uninitialised) are taken as zero and reported through
 * phantom_defined when the shading would read them.
 */
#include "rc_scene.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "raycast_hip.h"

#define LIGHT_REC 72
#define SHAPE_REC 104

/* byte classification of one light record (light_t, C/objects.h:51-61) */
static int light_byte_defined(const light_t *L, int byte, int is_last) {
  if (byte >= 64) return is_last;                  /* `next`: heap pointer, NULL on last */
  if (L->type == POINT && byte >= 36 && byte < 60) /* theta, cos_theta, a0, direction    */
    return 0;                                      /* never written for point lights     */
  return 1;
}

static void build_phantom(const light_t *const *lights, int m, shape_t *ph, int *defined) {
  unsigned char img[SHAPE_REC];
  unsigned char def[SHAPE_REC];
  const long region = ((long)LIGHT_REC * m + 15) & ~15L;
  for (long o = 0; o < SHAPE_REC; o++) {
    long off = region - SHAPE_REC + o;
    img[o] = 0;
    def[o] = 0;
    if (off < 0 || off >= (long)LIGHT_REC * m) continue;   /* stack garbage / padding */
    int li = (int)(off / LIGHT_REC), lb = (int)(off % LIGHT_REC);
    if (!light_byte_defined(lights[li], lb, li == m - 1)) continue;
    img[o] = ((const unsigned char *)lights[li])[lb];
    def[o] = 1;
  }
  memcpy(ph, img, sizeof(shape_t));
  ph->next = NULL;
  /* calc_color consumes diffuse [0,12), specular [12,24), reflectivity [36,40) and
   * refractivity [40,44) (C/raycast.c:382-383,408-412). */
  int ok = 1;
  for (int o = 0; o < 24; o++) ok &= def[o];
  for (int o = 36; o < 44; o++) ok &= def[o];
  *defined = ok;
}

static void fill_shape(rc_shape *d, const shape_t *s) {
  memset(d, 0, sizeof *d);
  d->type = (s->type == SPHERE) ? RC_SHAPE_SPHERE
          : (s->type == PLANE)  ? RC_SHAPE_PLANE
          : (s->type == QUADRIC) ? RC_SHAPE_QUADRIC : -1;
  d->refl = s->reflectivity;
  d->opacity = (float)((1.0 - (double)s->reflectivity) - (double)s->refractivity);
  d->p[0] = s->position[0]; d->p[1] = s->position[1]; d->p[2] = s->position[2];
  if (s->type == SPHERE) {
    d->r = s->radius;
    d->inv_r = (float)(1.0 / (double)s->radius);
    d->r2 = (double)s->radius * (double)s->radius;
  } else if (s->type == PLANE) {
    d->n[0] = s->normal[0]; d->n[1] = s->normal[1]; d->n[2] = s->normal[2];
  } else if (s->type == QUADRIC) {
    d->qa = s->a; d->qb = s->b; d->qc = s->c;
    d->A = (double)s->a; d->B = (double)s->b; d->C = (double)s->c;
    d->qd = s->d; d->qe = s->e; d->qf = s->f;
    d->qg = s->g; d->qh = s->h; d->qi = s->i; d->qj = s->j;
  }
  /* Origin-only terms of the intersection tests at O = (0,0,0), the primary rays' origin
   * (C/raycast.c:118-121), by the device's operations in the same order (rc_device.hpp
   * hit_sphere / hit_plane / hit_quadric with O = +0): sphere c (C/raycast.c:584-586),
   * plane numerator (:550), quadric c (:626-638). */
  const float ox = 0.0f, oy = 0.0f, oz = 0.0f;
  const float tx = ox - d->p[0], ty = oy - d->p[1], tz = oz - d->p[2];
  if (s->type == SPHERE) {
    float dd = tx * tx;
    dd = dd + ty * ty;
    dd = dd + tz * tz;
    d->o0 = (float)((double)dd - d->r2);
  } else if (s->type == PLANE) {
    float num = tx * d->n[0];
    num = num + ty * d->n[1];
    d->o0 = num + tz * d->n[2];
  } else if (s->type == QUADRIC) {
    double acc;
    acc = d->A * ((double)ox * (double)ox);
    acc = acc + d->B * ((double)oy * (double)oy);
    acc = acc + d->C * ((double)oz * (double)oz);
    acc = acc + (double)(d->qd * ox * oy);
    acc = acc + (double)(d->qe * ox * oz);
    acc = acc + (double)(d->qf * oy * oz);
    acc = acc + (double)(d->qg * ox);
    acc = acc + (double)(d->qh * oy);
    acc = acc + (double)(d->qi * oz);
    acc = acc + (double)d->qj;
    d->o0 = (float)acc;
  }
}

/* The primary-ray forms drop terms that are zero at O = 0 (rc_device.hpp nearest_primary);
 * that holds for finite coefficients only. */
static int o0_usable(const rc_shape *d) {
  const float f[] = {d->p[0], d->p[1], d->p[2], d->n[0], d->n[1], d->n[2], d->qd, d->qe,
                     d->qf, d->qg, d->qh, d->qi, d->qj, d->qa, d->qb, d->qc, d->o0};
  for (unsigned k = 0; k < sizeof f / sizeof f[0]; k++)
    if (!isfinite(f[k])) return 0;
  return isfinite(d->r2) && isfinite(d->A) && isfinite(d->B) && isfinite(d->C);
}

static void fill_light(rc_light *d, const light_t *l) {
  memset(d, 0, sizeof *d);
  d->pos[0] = l->position[0]; d->pos[1] = l->position[1]; d->pos[2] = l->position[2];
  d->type = (l->type == SPOTLIGHT) ? RC_LIGHT_SPOT : RC_LIGHT_POINT;
  d->r0 = l->radial_coef[0]; d->r1 = l->radial_coef[1]; d->r2 = l->radial_coef[2];
  if (l->type == SPOTLIGHT) {
    d->cos_theta = l->cos_theta;
    d->dir[0] = l->direction[0]; d->dir[1] = l->direction[1]; d->dir[2] = l->direction[2];
    d->a0 = l->a0;
    float r = nearbyintf(l->a0);
    if (r == l->a0 && fabsf(r) <= 64.0f) {
      d->a0_kind = RC_A0_INT;
      d->a0_int = (int32_t)r;
    } else {
      d->a0_kind = RC_A0_GENERAL;
    }
  }
}

static void fill_pair(rc_shade_pair *p, const shape_t *s, const light_t *l) {
  for (int k = 0; k < 3; k++) {
    p->dl[k] = s->diffuse_color[k] * l->color[k];
    p->sl[k] = s->specular_color[k] * l->color[k];
  }
}

rc_packed_header *rc_pack_scene(const json_data_t *js) {
  const int n = js->num_shapes, m = js->num_lights;
  if (n < 0 || m < 0) return NULL;
  const shape_t **sh = (const shape_t **)calloc((size_t)n + 1, sizeof *sh);
  const light_t **li = (const light_t **)calloc((size_t)m + 1, sizeof *li);
  if (!sh || !li) { free(sh); free(li); return NULL; }
  const shape_t *s = js->shapes_list;
  for (int k = 0; k < n; k++, s = s->next) {
    if (!s) { free(sh); free(li); return NULL; }
    sh[k] = s;
  }
  const light_t *l = js->lights_list;
  for (int k = 0; k < m; k++, l = l->next) {
    if (!l) { free(sh); free(li); return NULL; }
    li[k] = l;
  }
  shape_t phantom;
  int phantom_ok = 1;
  build_phantom(li, m, &phantom, &phantom_ok);
  const double ph_opacity = (double)(float)((1.0 - (double)phantom.reflectivity) -
                                            (double)phantom.refractivity);
  /* a phantom that is never lit (opacity <= 0) or has no light to be lit by is black */
  if (!(ph_opacity > 0.0) || m == 0) phantom_ok = 1;

  size_t off_shapes = sizeof(rc_packed_header);
  size_t off_lights = off_shapes + sizeof(rc_shape) * ((size_t)n + 1);
  size_t off_pairs = off_lights + sizeof(rc_light) * (size_t)m;
  size_t bytes = off_pairs + sizeof(rc_shade_pair) * ((size_t)n + 1) * (size_t)m;
  bytes = (bytes + 255) & ~(size_t)255;
  if (bytes > 0x7fffffff) { free(sh); free(li); return NULL; }
  unsigned char *buf = (unsigned char *)calloc(1, bytes);
  if (!buf) { free(sh); free(li); return NULL; }
  rc_packed_header *h = (rc_packed_header *)buf;
  h->n = n;
  h->m = m;
  h->cam_w = js->camera_width;
  h->cam_h = js->camera_height;
  h->off_shapes = (int32_t)off_shapes;
  h->off_lights = (int32_t)off_lights;
  h->off_pairs = (int32_t)off_pairs;
  h->bytes = (int32_t)bytes;
  h->phantom_defined = phantom_ok;
  rc_shape *ds = (rc_shape *)(buf + off_shapes);
  rc_light *dl = (rc_light *)(buf + off_lights);
  rc_shade_pair *dp = (rc_shade_pair *)(buf + off_pairs);
  h->o0_ok = 1;
  for (int k = 0; k < n; k++) {
    fill_shape(&ds[k], sh[k]);
    if (!o0_usable(&ds[k])) h->o0_ok = 0;
  }
  fill_shape(&ds[n], &phantom);
  ds[n].type = -1;                       /* never intersected, only shaded */
  for (int k = 0; k < m; k++) fill_light(&dl[k], li[k]);
  for (int k = 0; k <= n; k++)
    for (int j = 0; j < m; j++) fill_pair(&dp[(size_t)k * m + j], k < n ? sh[k] : &phantom, li[j]);
  free(sh);
  free(li);
  return h;
}
