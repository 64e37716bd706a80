/*
 * parse.c — scene-file front end of the host side.
 *
 * Accepts exactly the reference grammar of C/parse.c:13-436 and produces the same lists,
 * counts, stderr messages and exit(1) behaviour:
 *   - one record per line: a type token (camera | sphere | plane | quadric | light) then
 *     comma-separated `key: value` fields; a field that opens '[' runs to the matching ']'
 *     (commas and newlines included);
 *   - keys are compared with every space removed, values with leading spaces removed, and
 *     parsed with the same sscanf formats ("%f", "[%f, %f, %f]");
 *   - the scratch values persist from record to record (the reference keeps them in locals
 *     declared once, C/parse.c:15-37), so a repeated key can stand in for a missing one;
 *   - a record's field count must match (sphere 7, plane 5, quadric 13, point light 5,
 *     spot light 8; a missing diffuse/specular colour defaults to black and counts);
 *   - `theta: 0` makes a point light; any other theta is converted with 180/PI
 *     (C/parse.c:282, PI = 3.141592654f) and makes a spot light;
 *   - exactly one camera line.
 * The implementation is table driven; the only behaviour not mirrored is the reference's
 * undefined behaviour (reads past a field with no ':' or an unterminated '[').
 */
#include <stdbool.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#include "raycast_hip.h"

static const float kPI = 3.141592654f;   /* C/v3math.c:11 */

/* ------------------------------------------------------------------ tokenizer -- */
typedef struct {
  char *buf;
  size_t len, cap;
} field_t;

static void field_push(field_t *f, char ch) {
  if (f->len + 2 > f->cap) {
    f->cap = f->cap ? 2 * f->cap : 128;
    f->buf = (char *)realloc(f->buf, f->cap);
    if (!f->buf) {
      fprintf(stderr, "Error: out of memory while parsing the scene\n");
      exit(1);
    }
  }
  f->buf[f->len++] = ch;
  f->buf[f->len] = '\0';
}

/* The reference reads into a `char`, so a 0xFF byte compares equal to EOF. */
static char next_char(FILE *in, bool *at_eof) {
  int c = fgetc(in);
  if (c == EOF) *at_eof = true;
  return (char)c;
}

/* One comma/newline-terminated field (C/parse.c:368-392).  Returns true at end of line. */
static bool read_one_field(FILE *in, field_t *f) {
  bool eof = false;
  f->len = 0;
  field_push(f, '\0');
  f->len = 0;
  char c = next_char(in, &eof);
  while (c != ',' && c != '\n' && c != (char)EOF) {
    if (c == '[') {
      while (c != ']') {
        field_push(f, c);
        c = next_char(in, &eof);
        if (eof) return true;   /* unterminated vector: the reference never returns */
      }
    }
    field_push(f, c);
    c = next_char(in, &eof);
  }
  return c == '\n' || c == (char)EOF;
}

/* name := the characters before the first ':' with every space dropped; value := the rest
 * after that colon, leading spaces dropped (C/parse.c:402-430).  Like the source, a ':'
 * reached right after skipped spaces is taken into the name and the scan goes on; a field
 * with no usable ':' stops at its end (the reference reads past it). */
static void split_key_value(const char *s, char *name, size_t ncap, const char **value) {
  size_t k = 0, i = 0;
  name[0] = '\0';
  while (s[i] != ':') {
    while (s[i] == ' ') i++;
    const char c = s[i];
    if (c == '\0') {
      *value = s + i;
      return;
    }
    if (k + 1 < ncap) {
      name[k++] = c;
      name[k] = '\0';
    }
    i++;
  }
  i++;
  while (s[i] == ' ') i++;
  *value = s + i;
}

/* ------------------------------------------------------------- record tables -- */
typedef enum { K_SCALAR, K_VEC3, K_THETA } kind_t;

typedef struct {
  float color[3], diffuse[3], specular[3], pos[3], norm[3], radial[3], direction[3];
  float reflectivity, refractivity, ior, radius, theta, a0, q[10];
  bool diffuse_found, specular_found, spotlight;
} scratch_t;

typedef struct {
  const char *key;
  kind_t kind;
  size_t offset;   /* into scratch_t */
  int flag;        /* 1: diffuse_found, 2: specular_found */
} field_spec;

#define SC(member) offsetof(scratch_t, member)

static const field_spec kSphere[] = {
    {"diffuse_color", K_VEC3, SC(diffuse), 1}, {"specular_color", K_VEC3, SC(specular), 2},
    {"position", K_VEC3, SC(pos), 0},          {"radius", K_SCALAR, SC(radius), 0},
    {"reflectivity", K_SCALAR, SC(reflectivity), 0},
    {"refractivity", K_SCALAR, SC(refractivity), 0}, {"ior", K_SCALAR, SC(ior), 0},
    {NULL, K_SCALAR, 0, 0}};
static const field_spec kPlane[] = {
    {"diffuse_color", K_VEC3, SC(diffuse), 1}, {"specular_color", K_VEC3, SC(specular), 2},
    {"position", K_VEC3, SC(pos), 0},          {"normal", K_VEC3, SC(norm), 0},
    {"reflectivity", K_SCALAR, SC(reflectivity), 0}, {NULL, K_SCALAR, 0, 0}};
static const field_spec kQuadric[] = {
    {"diffuse_color", K_VEC3, SC(diffuse), 1}, {"specular_color", K_VEC3, SC(specular), 2},
    {"reflectivity", K_SCALAR, SC(reflectivity), 0},
    {"a", K_SCALAR, SC(q[0]), 0}, {"b", K_SCALAR, SC(q[1]), 0}, {"c", K_SCALAR, SC(q[2]), 0},
    {"d", K_SCALAR, SC(q[3]), 0}, {"e", K_SCALAR, SC(q[4]), 0}, {"f", K_SCALAR, SC(q[5]), 0},
    {"g", K_SCALAR, SC(q[6]), 0}, {"h", K_SCALAR, SC(q[7]), 0}, {"i", K_SCALAR, SC(q[8]), 0},
    {"j", K_SCALAR, SC(q[9]), 0}, {NULL, K_SCALAR, 0, 0}};
static const field_spec kLight[] = {
    {"color", K_VEC3, SC(color), 0},           {"position", K_VEC3, SC(pos), 0},
    {"theta", K_THETA, SC(theta), 0},          {"radial-a0", K_SCALAR, SC(radial[0]), 0},
    {"radial-a1", K_SCALAR, SC(radial[1]), 0}, {"radial-a2", K_SCALAR, SC(radial[2]), 0},
    {"angular-a0", K_SCALAR, SC(a0), 0},       {"direction", K_VEC3, SC(direction), 0},
    {NULL, K_SCALAR, 0, 0}};

static void fail(const char *msg) {
  fprintf(stderr, "%s", msg);
  exit(1);
}

/* Read the rest of a record line, applying `table`.  Returns the counted fields. */
static int read_record(FILE *in, field_t *f, const field_spec *table, scratch_t *st) {
  int counted = 0;
  bool eol = false;
  char name[256];
  while (!eol) {
    eol = read_one_field(in, f);
    const char *value;
    split_key_value(f->buf, name, sizeof name, &value);
    for (const field_spec *fs = table; fs->key; fs++) {
      if (strcmp(name, fs->key) != 0) continue;
      float *dst = (float *)((char *)st + fs->offset);
      if (fs->kind == K_VEC3) {
        sscanf(value, "[%f, %f, %f]", &dst[0], &dst[1], &dst[2]);
      } else {
        sscanf(value, "%f", dst);
      }
      if (fs->kind == K_THETA) {
        if (*dst == 0.0f) break;                            /* point light: not counted */
        *dst = (float)((double)*dst * (180.0 / (double)kPI));
        st->spotlight = true;
      }
      if (fs->flag == 1) st->diffuse_found = true;
      if (fs->flag == 2) st->specular_found = true;
      counted++;
      break;
    }
  }
  return counted;
}

static int default_colors(scratch_t *st) {
  int added = 0;
  if (!st->specular_found) {
    set_to_black(st->specular);
    added++;
  }
  if (!st->diffuse_found) {
    set_to_black(st->diffuse);
    added++;
  }
  return added;
}

static const char kBadRefl[] =
    "Error: invalid reflectivity for a sphere. Must be between 0 and 1.\n";

void set_to_black(float *input) {
  input[0] = 0.0f;
  input[1] = 0.0f;
  input[2] = 0.0f;
}

void parse_json(FILE *json, json_data_t *json_data) {
  scratch_t st;
  memset(&st, 0, sizeof st);
  field_t f = {NULL, 0, 0};
  int cameras = 0;
  char name[256];
  for (;;) {
    st.diffuse_found = st.specular_found = false;
    read_one_field(json, &f);   /* the type token; its end-of-line flag is not used */
    const char *type = f.buf;
    if (!strcmp(type, "camera")) {
      cameras++;
      int n = 0;
      bool eol = false;
      while (!eol) {
        eol = read_one_field(json, &f);
        const char *value;
        split_key_value(f.buf, name, sizeof name, &value);
        if (!strcmp(name, "width")) {
          sscanf(value, "%f", &json_data->camera_width);
          n++;
        } else if (!strcmp(name, "height")) {
          sscanf(value, "%f", &json_data->camera_height);
          n++;
        }
      }
      if (n != 2) fail("Error: A camera width or height was not given.\n");
    } else if (!strcmp(type, "sphere")) {
      int n = read_record(json, &f, kSphere, &st) + default_colors(&st);
      if (n != 7) fail("Error: A field for a sphere was missing.\n");
      if (st.reflectivity < 0 || st.reflectivity > 1) fail(kBadRefl);
      if (st.refractivity < 0 || st.refractivity > 1)
        fail("Error: invalid refractivity for a sphere. Must be between 0 and 1.\n");
      json_data->shapes_list =
          add_new_sphere(json_data->shapes_list, st.diffuse, st.specular, st.pos, st.radius,
                         st.reflectivity, st.refractivity, st.ior);
      json_data->num_shapes += 1;
    } else if (!strcmp(type, "plane")) {
      int n = read_record(json, &f, kPlane, &st) + default_colors(&st);
      if (n != 5) fail("Error: A field for a plane was missing.\n");
      if (st.reflectivity < 0 || st.reflectivity > 1) fail(kBadRefl);
      json_data->shapes_list = add_new_plane(json_data->shapes_list, st.diffuse, st.specular,
                                             st.pos, st.norm, st.reflectivity);
      json_data->num_shapes += 1;
    } else if (!strcmp(type, "quadric")) {
      int n = read_record(json, &f, kQuadric, &st) + default_colors(&st);
      if (n != 13) fail("Error: A field for a quadric was missing.\n");
      if (st.reflectivity < 0 || st.reflectivity > 1) fail(kBadRefl);
      const float *q = st.q;
      json_data->shapes_list =
          add_new_quadric(json_data->shapes_list, st.diffuse, st.specular, q[0], q[1], q[2],
                          q[3], q[4], q[5], q[6], q[7], q[8], q[9], st.reflectivity);
      json_data->num_shapes += 1;
    } else if (!strcmp(type, "light")) {
      st.spotlight = false;
      int n = read_record(json, &f, kLight, &st);
      if ((!st.spotlight && n != 5) || (st.spotlight && n != 8))
        fail("Error: A field for a light was missing.\n");
      if (st.spotlight)
        json_data->lights_list = add_new_spot_light(json_data->lights_list, st.color, st.pos,
                                                    st.theta, st.a0, st.direction, st.radial);
      else
        json_data->lights_list =
            add_new_point_light(json_data->lights_list, st.color, st.pos, st.radial);
      json_data->num_lights += 1;
    }
    int c = fgetc(json);
    if ((char)c == (char)EOF) break;
    ungetc(c, json);
  }
  free(f.buf);
  if (cameras != 1) fail("Error: The scene must have one and only one camera.\n");
}
