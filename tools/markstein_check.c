/* Exactness check of the Markstein quotient used for integer divisors (factors.hip div_n / divc,
 * zscore.hip group_var): q0 = RN(x r), e = fma(-q0, n, x), q = fma(e, r, q0) with r = RN(1 / n)
 * equals the IEEE quotient RN(x / n).  Markstein's theorem covers it (r the correctly rounded
 * reciprocal, q0 faithful); this program checks it on x whose quotient lies within 3 ulps of a
 * rounding midpoint (the hard cases) for every n <= N, 2,000 random midpoints each.
 *   gcc -O2 -ffp-contract=off tools/markstein_check.c -lm && ./a.out 8192 2000
 * measured here: N = 8192, 114,688,000 cases, 0 mismatches. */
#include <stdio.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s=88172645463325252ull;
static inline uint64_t rnd(){ s^=s<<13; s^=s>>7; s^=s<<17; return s; }
int main(int argc,char**argv){
  int N=atoi(argv[1]); long M=atol(argv[2]); long bad=0, tot=0;
  for(int n=1;n<=N;n++){
    double d=(double)n, r=1.0/d;
    for(long i=0;i<M;i++){
      uint64_t u=rnd(); uint64_t e = 1023 - 30 + (rnd()%60);
      uint64_t bits = (u & 0x000fffffffffffffull) | (e<<52);
      double q; memcpy(&q,&bits,8);
      double qn = nextafter(q, INFINITY);
      long double mid = ((long double)q + (long double)qn)/2;     // 64-bit mantissa long double
      for(int k=-3;k<=3;k++){
        double x = (double)(mid * (long double)d);
        for(int j=0;j<k;j++) x=nextafter(x,INFINITY);
        for(int j=0;j>k;j--) x=nextafter(x,-INFINITY);
        double q0=x*r; double ee=fma(-q0,d,x); double q1=fma(ee,r,q0);
        double ref=x/d; tot++;
        if(q1!=ref){ if(bad<10) printf("n=%d x=%.17g q1=%.17g ref=%.17g\n",n,x,q1,ref); bad++; }
      }
    }
  }
  printf("N=%d cases=%ld bad=%ld\n",N,tot,bad); return 0; }
