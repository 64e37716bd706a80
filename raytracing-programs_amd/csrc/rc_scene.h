/*
 * rc_scene.h — packed scene image shared by the host flattener (rc_scene.c) and the HIP
 * kernels (rc_kernels.hip).
 *
 * The reference walks two linked lists of 104-B shape_t / 72-B light_t records copied into
 * stack VLAs (C/raycast.c:87-107).  On MI355X the whole scene is one small read-only
 * buffer whose per-shape records are read with wave-uniform scalar loads (every lane of a
 * wave tests the same shape k at the same time, C/raycast.c:449), so shape parameters land
 * in SGPRs and feed VALU ops directly as scalar operands.
 *
 * Everything the reference recomputes per test but that depends only on the scene is
 * precomputed here with the identical IEEE operation (so the value is bit-identical):
 *   sphere  r*r in double (C/raycast.c:585), (float)(1.0/r) (C/raycast.c:465)
 *   quadric a,b,c widened to double (C/raycast.c:615-638, 504-517)
 *   primary rays: the origin-only terms of each test at O = (0,0,0) (rc_shape::o0)
 *   shading opacity (float)((1.0-refl)-refr) (C/raycast.c:383) and the per (shape,light)
 *   colour products diffuse*light.color, specular*light.color (C/raycast.c:716-718,755-757)
 * Index n (one past the last shape) holds the phantom record shapes_list[-1].
 */
#ifndef RC_SCENE_H
#define RC_SCENE_H

#include <stdint.h>

#define RC_SHAPE_SPHERE 0
#define RC_SHAPE_PLANE 1
#define RC_SHAPE_QUADRIC 2

#define RC_LIGHT_POINT 0
#define RC_LIGHT_SPOT 1

/* spot-light exponent kinds for pow(alpha, a0) (C/raycast.c:695) */
#define RC_A0_INT 0      /* a0 is an integer with |a0| <= 64: exact-product power */
#define RC_A0_GENERAL 1  /* any other value: double-double exp/log power          */

/* 128 B per shape: geometry fields are read in the intersection loop. */
typedef struct rc_shape {
  int32_t type;        /* RC_SHAPE_*                                   */
  float refl;          /* reflectivity (loop test C/raycast.c:352)     */
  float opacity;       /* (float)((1.0 - refl) - refr)                 */
  float inv_r;         /* sphere: (float)(1.0 / (double)radius)        */
  float p[3];          /* sphere/plane position                        */
  float r;             /* sphere radius (unused by the math, kept)     */
  float n[3];          /* plane normal                                 */
  float qd, qe, qf;    /* quadric d, e, f                              */
  float qg, qh, qi, qj;/* quadric g, h, i, j                           */
  float qa, qb, qc;    /* quadric a, b, c (float)                      */
  float o0;            /* primary rays (origin (0,0,0)): the origin-only */
                       /* term, computed as the device would at O = 0:   */
                       /* sphere c, plane numerator, quadric c          */
  double r2;           /* sphere (double)r*(double)r                   */
  double A, B, C;      /* quadric (double)a, (double)b, (double)c      */
  double pad1;
} rc_shape;

/* 64 B per light */
typedef struct rc_light {
  float pos[3];
  int32_t type;        /* RC_LIGHT_*                                   */
  float r0, r1, r2;    /* radial coefficients                          */
  float cos_theta;
  float dir[3];
  float a0;
  int32_t a0_kind;     /* RC_A0_*                                      */
  int32_t a0_int;      /* a0 as an integer when a0_kind == RC_A0_INT   */
  float pad[2];
} rc_light;

/* per (shape, light) colour products: [ (n+1) * m ] entries, shape-major */
typedef struct rc_shade_pair {
  float dl[3];         /* diffuse_color[k] * light.color[k]  (float)   */
  float sl[3];         /* specular_color[k] * light.color[k] (float)   */
} rc_shade_pair;

/* Header of the packed image; followed in the same allocation by
 *   rc_shape shapes[n + 1]      (index n = phantom)
 *   rc_light lights[m]
 *   rc_shade_pair pairs[(n + 1) * m]                                       */
typedef struct rc_packed_header {
  int32_t n;            /* shapes                                       */
  int32_t m;            /* lights                                       */
  float cam_w, cam_h;   /* camera width/height (C/parse.c:50-56)        */
  int32_t off_shapes;   /* byte offsets from the header start           */
  int32_t off_lights;
  int32_t off_pairs;
  int32_t bytes;        /* total image size                             */
  int32_t phantom_defined;
  int32_t o0_ok;        /* every shape's o0 usable (finite coefficients) */
  int32_t pad[6];
} rc_packed_header;

#ifdef __cplusplus
extern "C" {
#endif
struct json_data_t;
/* Build the packed image from the reference lists (not consumed).  Returns a malloc'd
 * buffer of header->bytes bytes, or NULL on allocation failure / inconsistent counts. */
rc_packed_header *rc_pack_scene(const struct json_data_t *js);
#ifdef __cplusplus
}
#endif

#endif
