/*
 * raytrace_main.c — the drop-in CLI, same contract as the reference's main
 * (C/raycast.c:19-69):
 *   raytrace WIDTH HEIGHT INPUT_SCENE OUTPUT_IMAGE
 * usage text on stdout + exit 0 for a wrong argument count, the scene opened "r+" and the
 * output opened "wb" before parsing (with the same error messages), the P3 image, and the
 * timing line.  Rendering goes through raycast() of libraycast_hip.so; the timed span is
 * the same as the reference's (render + P3 write + frees).
 */
#include <stdlib.h>
#include <sys/time.h>

#include "raycast_hip.h"

int main(int argc, char **argv) {
  if (argc != 5) {
    printf("Usage: raytrace WIDTH HEIGHT INPUT_SCENE OUTPUT_IMAGE\n");
    exit(0);
  }
  int width = atoi(argv[1]);
  int height = atoi(argv[2]);
  FILE *input_json = fopen(argv[3], "r+");
  if (input_json == NULL) {
    fprintf(stderr, "Error: Unable to open the input scene file: %s\n", argv[3]);
    exit(1);
  }
  FILE *output_image = fopen(argv[4], "wb");
  if (output_image == NULL) {
    fprintf(stderr, "Error: Unable to open the output image file: %s\n", argv[4]);
    exit(1);
  }
  json_data_t *json_struct = (json_data_t *)calloc(1, sizeof(json_data_t));
  if (!json_struct) exit(1);
  parse_json(input_json, json_struct);
  fclose(input_json);

  PPMFormat photo_data;
  photo_data.maxColor = 255;
  photo_data.depth = 0;
  photo_data.tupleType = NULL;
  photo_data.height = height;
  photo_data.width = width;
  photo_data.size = photo_data.width * photo_data.height * 3;
  size_t bytes = (width > 0 && height > 0) ? (size_t)width * (size_t)height * 3 : 1;
  photo_data.pixmap = (uint8_t *)malloc(bytes);
  if (!photo_data.pixmap) {
    fprintf(stderr, "Error: out of memory for a %dx%d image\n", width, height);
    exit(1);
  }
  const int num_shapes = json_struct->num_shapes, num_lights = json_struct->num_lights;

  struct timeval start, end;
  gettimeofday(&start, NULL);
  raycast(json_struct, photo_data);
  ppm_WriteOutP3(photo_data, output_image);
  free(photo_data.pixmap);
  free(json_struct);
  gettimeofday(&end, NULL);
  double elapsed = (((end.tv_sec * 1000000.0 + end.tv_usec) -
                     (start.tv_sec * 1000000.0 + start.tv_usec)) / 1000000.00);
  printf("Time (sec) to create a %dx%d image with %d shape(s) and %d light(s): %f\n", width,
         height, num_shapes, num_lights, elapsed);
  fclose(output_image);
  return 0;
}
