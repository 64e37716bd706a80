/* front_check.c — TEST TOOL (tests/test_sanitize.py): drives the host front end
 * (csrc/front/parse.c, objects.c, ppm.c) under AddressSanitizer / UBSan: parse a scene with
 * parse_json (C/parse.c:13 semantics), print the list contents, write a W x H gradient image
 * with ppm_WriteOutP3 (C/ppm.c:168-184) and free both lists.
 *   front_check SCENE OUT.ppm W H */
#include <stdio.h>
#include <stdlib.h>

#include "raycast_hip.h"

int main(int argc, char **argv) {
  if (argc != 5) return 2;
  FILE *f = fopen(argv[1], "r");
  if (!f) return 1;
  json_data_t js;
  parse_json(f, &js);
  fclose(f);
  printf("%d %d", js.num_shapes, js.num_lights);
  for (shape_t *s = js.shapes_list; s; s = s->next)
    printf(" s%d:%.9g,%.9g,%.9g,%.9g", (int)s->type, s->position[0], s->position[1],
           s->position[2], s->reflectivity);
  for (light_t *l = js.lights_list; l; l = l->next)
    printf(" l%d:%.9g,%.9g,%.9g", (int)l->type, l->position[0], l->cos_theta, l->a0);
  printf("\n");
  const int W = atoi(argv[3]), H = atoi(argv[4]);
  PPMFormat img = {W, H, W * H * 3, 255, 3, NULL, (uint8_t *)malloc((size_t)W * H * 3)};
  for (size_t k = 0; k < (size_t)W * H * 3; k++) img.pixmap[k] = (uint8_t)(k * 7 + k / 3);
  FILE *o = fopen(argv[2], "wb");
  if (!o) return 1;
  ppm_WriteOutP3(img, o);
  fclose(o);
  free(img.pixmap);
  js.shapes_list = free_shape_list(js.shapes_list);
  js.lights_list = free_light_list(js.lights_list);
  return 0;
}
