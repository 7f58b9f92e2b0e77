/* Host check of the dense quantise's division (coalac.hip k_dense_quant):
 * t1 = fma(fma(-q, b, a), y, q) with q = a * y, y = 1 / b  against  t0 = a / b, on random and boundary-targeted
 * (a, b): scale exponents in [2^-90, 2^89] (mantissas all ones / zero / random), a uniform in [0, levels * b], within
 * 4 ulps of half-integer and integer quotients, or any float. Counts differing quotients (a >= 2^-100) and differing
 * rint codes. Build: gcc -O2 -mfma -o /tmp/rcp_div_check tools/rcp_div_check.c -lm; run: /tmp/rcp_div_check 1000000000
 * (round 6: bad=0 bad_rint=0). */
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <stdlib.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void){ s ^= s<<13; s ^= s>>7; s ^= s<<17; return s; }
static inline float fb(uint32_t u){ float f; memcpy(&f,&u,4); return f; }
static inline uint32_t bf(float f){ uint32_t u; memcpy(&u,&f,4); return u; }
int main(int argc,char**argv){
  long N = atol(argv[1]); long bad=0, badr=0;
  for (long i=0;i<N;i++){
    uint64_t r = xr();
    uint32_t e = 127 - 90 + (uint32_t)(r % 180);          /* scale exponent in [2^-90, 2^89] */
    uint32_t m = (uint32_t)(r >> 8) & 0x7FFFFF;
    int kind = (r>>40) & 7;
    if (kind==0) m = 0x7FFFFF; else if (kind==1) m = 0; else if (kind==2) m = 0x7FFFFF ^ ((r>>44)&0xFF);
    float b = fb((e<<23)|m);
    float y = 1.0f / b;
    uint64_t r2 = xr();
    float a;
    int ak = r2 & 3;
    float lv = (float)(1 + (r2>>2)%255);
    if (ak==0) a = (float)((double)(r2>>11) / 9007199254740992.0 * lv) * b;            /* uniform-ish */
    else if (ak==1) { float h = ((float)((r2>>3)%256) + 0.5f) * b; uint32_t hu = bf(h); int d = (int)((r2>>20)%9) - 4; a = fb(hu + d); } /* near half-integers */
    else if (ak==2) { float h = ((float)((r2>>3)%256)) * b; uint32_t hu = bf(h); int d = (int)((r2>>20)%9) - 4; a = fb(hu + d); } /* near integers */
    else a = fb(xr() & 0x7FFFFFFF) ; /* any positive float */
    if (!(a >= 0) || isinf(a)) continue;
    float t0 = a / b; if (!(t0 < 1048576.0f)) continue;
    float q = a * y;
    float rr = fmaf(-q, b, a);
    float t1 = fmaf(rr, y, q);
    if (bf(t0) != bf(t1) && a >= 0x1p-100f) { bad++; if (bad < 5) printf("mismatch a=%a b=%a t0=%a t1=%a\n", a, b, t0, t1); }
    if (rintf(t0) != rintf(t1)) badr++;
  }
  printf("N=%ld bad=%ld bad_rint=%ld\n", N, bad, badr);
}
