/* asan_main.c — drives the CPU oracle (vss_oracle.c, test infrastructure) under
 * AddressSanitizer + UndefinedBehaviorSanitizer ("race detection /
 * sanitizers": ASan on the CPU restatement).  Built by `make -C oracle asan`
 * into oracle/_ref/oracle_asan (gitignored); tests/test_oracle_asan.py runs it.
 *
 *   oracle_asan WEIGHTS_BLOB
 *
 * Exercises every entry point the tests use on edge-case geometry: 1x1 and odd
 * frames, RGBA with padded rows, a 2-frame batch on 1 and 4 threads (the
 * nested frame x channel OpenMP teams), the post chain with and without face
 * inputs, compositing and the frame-size mask upsample.  Exit 0 = clean. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  double ema, noise_cutoff, high_threshold, gamma, sigma_spatial, sigma_range;
  int use_bilateral;
} vsso_post_cfg;
typedef struct {
  int has_affine;
  double affine[6];
  int has_box;
  double box[4];
  int video_w, video_h;
} vsso_face;

int vsso_preprocess(const uint8_t* frames, int n, int h, int w, int c, long row_stride, long frame_stride, int Hm,
                    int Wm, float* out);
int vsso_forward(const uint8_t* blob, long blob_bytes, int mode, const uint8_t* frames, int n, int h, int w, int c,
                 long row_stride, long frame_stride, int Hm, int Wm, float* masks, int nthreads, float** taps);
int vsso_post_face(const float* masks, int n, int H, int W, const uint8_t* frames, int fh, int fw, int fc,
                   long row_stride, long frame_stride, const vsso_post_cfg* cfg, float* state, int* state_valid,
                   const vsso_face* faces, float* out_alpha, uint8_t* out_u8);
int vsso_composite(const uint8_t* frames, int n, int fh, int fw, int fc, long row_stride, long frame_stride,
                   const uint8_t* alpha, int H, int W, uint8_t* out);
int vsso_upsample_mask(const float* masks, int n, int H, int W, int fh, int fw, float* out);

static uint8_t* frames_of(int n, int h, int w, int c, long rs, unsigned seed) {
  uint8_t* f = (uint8_t*)malloc((size_t)n * h * rs);
  for (size_t i = 0; i < (size_t)n * h * rs; ++i) {
    seed = seed * 1664525u + 1013904223u;
    f[i] = (uint8_t)(seed >> 24);
  }
  return f;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s WEIGHTS_BLOB\n", argv[0]);
    return 2;
  }
  FILE* fp = fopen(argv[1], "rb");
  if (!fp) return 2;
  fseek(fp, 0, SEEK_END);
  long bytes = ftell(fp);
  fseek(fp, 0, SEEK_SET);
  uint8_t* blob = (uint8_t*)malloc((size_t)bytes);
  if (fread(blob, 1, (size_t)bytes, fp) != (size_t)bytes) return 2;
  fclose(fp);
  const int Hm = 48, Wm = 64, P = Hm * Wm;
  const int geo[][3] = {{1, 1, 3}, {3, 5, 4}, {37, 61, 3}, {120, 160, 4}};
  int fails = 0;
  for (int g = 0; g < 4; ++g) {
    const int h = geo[g][0], w = geo[g][1], c = geo[g][2];
    const long rs = (long)w * c + 8; /* padded rows */
    const int n = 2;
    uint8_t* f = frames_of(n, h, w, c, rs, 17u + g);
    float* x0 = (float*)malloc(sizeof(float) * 3 * P * n);
    float* m1 = (float*)malloc(sizeof(float) * P * n);
    float* m4 = (float*)malloc(sizeof(float) * P * n);
    fails += vsso_preprocess(f, n, h, w, c, rs, rs * h, Hm, Wm, x0) != 0;
    fails += vsso_forward(blob, bytes, 0, f, n, h, w, c, rs, rs * h, Hm, Wm, m1, 1, NULL) != 0;
    fails += vsso_forward(blob, bytes, 0, f, n, h, w, c, rs, rs * h, Hm, Wm, m4, 4, NULL) != 0;
    fails += memcmp(m1, m4, sizeof(float) * P * n) != 0; /* threads never change the result */
    vsso_post_cfg cfg = {0.55, 0.06, 0.95, 0.4, 1.0, 12.0, 1};
    float* state = (float*)calloc(P, sizeof(float));
    int valid = 0;
    float* alpha = (float*)malloc(sizeof(float) * P * n);
    uint8_t* u8 = (uint8_t*)malloc((size_t)P * n);
    fails += vsso_post_face(m1, n, Hm, Wm, f, h, w, c, rs, rs * h, &cfg, state, &valid, NULL, alpha, u8) != 0;
    vsso_face faces[2] = {{1, {1.0, 0.02, 1.5, -0.02, 1.0, -2.0}, 1, {0.2 * w, 0.1 * h, 0.7 * w, 0.8 * h}, w, h},
                          {0, {0}, 1, {0, 0, (double)w, (double)h}, 0, 0}};
    fails += vsso_post_face(m1, n, Hm, Wm, f, h, w, c, rs, rs * h, &cfg, state, &valid, faces, alpha, u8) != 0;
    uint8_t* rgba = (uint8_t*)malloc((size_t)n * h * w * 4);
    fails += vsso_composite(f, n, h, w, c, rs, rs * h, u8, Hm, Wm, rgba) != 0;
    float* up = (float*)malloc(sizeof(float) * n * h * w);
    fails += vsso_upsample_mask(m1, n, Hm, Wm, h, w, up) != 0;
    free(f); free(x0); free(m1); free(m4); free(state); free(alpha); free(u8); free(rgba); free(up);
  }
  free(blob);
  printf("oracle_asan: %d failures\n", fails);
  return fails ? 1 : 0;
}
