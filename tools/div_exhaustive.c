/* Exhaustive check that x / d == fma(fma(-q, d, x), c, q) with q = x * c and c = RN(1/d), for every
 * finite float x with |x| >= 2^-100 (the shading path's div_pi / div_two_pi, pt_common.h, and
 * rt_unorm16's x / 65535); with a second argument "2", of rtmath.h rt_div_rcp's two corrections for
 * every x with 2^-30 <= |x| <= 2^30 (the denoiser's depth weights).
 * Build: gcc -O2 -ffp-contract=off -o div_exhaustive div_exhaustive.c -lm
 * Run: ./div_exhaustive 3.14159265358979 ; ./div_exhaustive 0.01 2   (about a minute each;
 * prints bad=0 when the identity holds for all 2^32 bit patterns in range) */
#include <stdio.h>
#include <math.h>
#include <string.h>
#include <stdint.h>
#include <stdlib.h>
int main(int argc, char** argv){
  volatile float d = strtof(argv[1], 0); const float c = 1.0f / d;
  uint32_t cb, db; memcpy(&cb,&c,4); memcpy(&db,(const void*)&d,4); printf("d=%a bits=%08x c=%a bits=%08x\n", (double)d, db, c, cb);
  uint64_t bad=0;
  const int two = argc > 2 && argv[2][0] == '2';
  for (uint64_t u=0; u<(1ull<<32); ++u){ uint32_t b=(uint32_t)u; float x; memcpy(&x,&b,4); if (!isfinite(x) || fabsf(x) < 0x1p-100f) continue;
    if (two && (fabsf(x) < 0x1p-30f || fabsf(x) > 0x1p30f)) continue;
    float ref = x / d; float q = x*c; float r = fmaf(-q, d, x); float o = fmaf(r, c, q);
    if (two) o = fmaf(fmaf(-o, d, x), c, o);
    if (memcmp(&o,&ref,4)) { if (bad<4) printf("x=%a ref=%a got=%a\n", x, ref, o); ++bad; } }
  printf("bad=%llu\n",(unsigned long long)bad);
}
