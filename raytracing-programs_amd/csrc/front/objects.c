/*
 * objects.c — scene list builders of the host front end.
 *
 * Same names, arguments and list semantics as the reference's C/objects.c:20-221: every
 * add_* appends one node at the TAIL (file order is render order, C/raycast.c:449) and
 * returns the head.  Nodes are zero-filled, so the fields the reference leaves
 * uninitialised (a point light's theta/cos_theta/a0/direction) read as 0.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "raycast_hip.h"

static void *node_alloc(size_t bytes) {
  void *p = calloc(1, bytes);
  if (!p) {
    fprintf(stderr, "Error: out of memory while building the scene\n");
    exit(1);
  }
  return p;
}

static shape_t *append_shape(shape_t *head, shape_t *node) {
  if (!head) return node;
  shape_t *t = head;
  while (t->next) t = t->next;
  t->next = node;
  return head;
}

static light_t *append_light(light_t *head, light_t *node) {
  if (!head) return node;
  light_t *t = head;
  while (t->next) t = t->next;
  t->next = node;
  return head;
}

static void copy3(float *dst, const float *src) {
  dst[0] = src[0];
  dst[1] = src[1];
  dst[2] = src[2];
}

shape_t *add_new_sphere(shape_t *head, float *diffuse, float *specular, float *position,
                        float radius, float reflectivity, float refractivity, float ior) {
  shape_t *s = (shape_t *)node_alloc(sizeof *s);
  copy3(s->diffuse_color, diffuse);
  copy3(s->specular_color, specular);
  copy3(s->position, position);
  s->reflectivity = reflectivity;
  s->refractivity = refractivity;
  s->ior = ior;
  s->radius = radius;
  s->type = SPHERE;
  return append_shape(head, s);
}

shape_t *add_new_plane(shape_t *head, float *diffuse, float *specular, float *position,
                       float *normal, float reflectivity) {
  shape_t *s = (shape_t *)node_alloc(sizeof *s);
  copy3(s->diffuse_color, diffuse);
  copy3(s->specular_color, specular);
  copy3(s->position, position);
  copy3(s->normal, normal);
  s->reflectivity = reflectivity;
  s->refractivity = 0.0f;   /* planes are opaque to refraction (C/objects.c:67-68) */
  s->ior = 1.0f;
  s->type = PLANE;
  return append_shape(head, s);
}

shape_t *add_new_quadric(shape_t *head, float *diffuse, float *specular, float a, float b,
                         float c, float d, float e, float f, float g, float h, float i,
                         float j, float reflectivity) {
  shape_t *s = (shape_t *)node_alloc(sizeof *s);
  copy3(s->diffuse_color, diffuse);
  copy3(s->specular_color, specular);
  const float coef[10] = {a, b, c, d, e, f, g, h, i, j};
  memcpy(&s->a, coef, sizeof coef);
  s->reflectivity = reflectivity;
  s->refractivity = 0.0f;   /* C/objects.c:108-109 */
  s->ior = 1.0f;
  s->type = QUADRIC;
  return append_shape(head, s);
}

light_t *add_new_point_light(light_t *head, float *color, float *position, float *radial_coef) {
  light_t *l = (light_t *)node_alloc(sizeof *l);
  copy3(l->color, color);
  copy3(l->position, position);
  copy3(l->radial_coef, radial_coef);
  l->type = POINT;
  return append_light(head, l);
}

light_t *add_new_spot_light(light_t *head, float *color, float *position, float theta,
                            float a0, float *direction, float *radial_coef) {
  light_t *l = (light_t *)node_alloc(sizeof *l);
  copy3(l->color, color);
  copy3(l->position, position);
  copy3(l->direction, direction);
  copy3(l->radial_coef, radial_coef);
  l->a0 = a0;
  l->theta = theta;
  l->cos_theta = (float)cos((double)theta);   /* C/objects.c:179, libm cos */
  l->type = SPOTLIGHT;
  return append_light(head, l);
}

shape_t *free_shape_list(shape_t *head) {
  while (head) {
    shape_t *n = head->next;
    free(head);
    head = n;
  }
  return NULL;
}

light_t *free_light_list(light_t *head) {
  while (head) {
    light_t *n = head->next;
    free(head);
    head = n;
  }
  return NULL;
}
