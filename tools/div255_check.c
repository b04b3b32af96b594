/* Exhaustive check of the kernels' div255() (csrc/vss_kernels.hip): for every
 * float v in [0, 256], fma(fma(-q, 255, v), 1/255, q) with q = v * (1/255)
 * equals the correctly rounded v / 255.0f.  Build: gcc -O2 -mfma -fopenmp.
 * Prints "checked N values, M mismatches"; exit status 1 on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

int main(void) {
  const float inv = 1.0f / 255.0f, lim = 256.0f;
  uint32_t last;
  memcpy(&last, &lim, 4);
  unsigned long long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
  for (long long b = 0; b <= (long long)last; ++b) {
    const uint32_t u = (uint32_t)b;
    float v;
    memcpy(&v, &u, 4);
    volatile float ref = v / 255.0f;
    const float q = v * inv;
    const float got = fmaf(fmaf(-q, 255.0f, v), inv, q);
    const float r = ref;
    if (memcmp(&got, &r, 4) != 0) ++bad;
  }
  printf("checked %llu values, %llu mismatches\n", (unsigned long long)last + 1, bad);
  return bad != 0;
}
