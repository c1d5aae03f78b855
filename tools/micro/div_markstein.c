#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <stdint.h>
static uint64_t s = 88172645463325252ull;
static uint64_t xr(void){ s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double rnd(void){ // random double with random exponent in a modest range and random mantissa
  uint64_t m = xr() & ((1ull<<52)-1);
  int e = (int)(xr() % 200) - 100 + 1023;
  uint64_t sg = xr() & 1;
  uint64_t b = (sg<<63) | ((uint64_t)e<<52) | m;
  double d; memcpy(&d,&b,8); return d;
}
#include <string.h>
int main(int argc, char**argv){
  long n = atol(argv[1]); long bad = 0;
  for (long i = 0; i < n; i++) {
    double b = (i % 4 == 0) ? 0.5 * (1.0 + (double)(xr() % 1000000) / 1e6) : rnd();
    if (i % 1000 == 1) { uint64_t bb; memcpy(&bb,&b,8); bb |= ((1ull<<52)-1); memcpy(&b,&bb,8); } // all-ones mantissa
    double y = 1.0 / b;
    for (int k = 0; k < 8; k++) {
      double a = rnd();
      double q0 = a * y;
      double r = fma(-q0, b, a);
      double q1 = fma(r, y, q0);
      double t = a / b;
      if (q1 != t) { if (bad < 10) printf("mismatch a=%a b=%a q1=%a t=%a\n", a, b, q1, t); bad++; }
    }
  }
  printf("bad %ld of %ld\n", bad, n*8);
  return 0;
}
