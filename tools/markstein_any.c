/* Markstein quotient for arbitrary divisors (lasso.hip div_r): q0 = RN(x r), e = fma(-q0, d, x),
 * q = RN(q0 + e r) with r = RN(1 / d) against the IEEE x / d, on quotients within 3 ulps of a
 * rounding midpoint and on random x, for random divisors, all-ones and few-bit significands.
 *   gcc -O2 -ffp-contract=off tools/markstein_any.c -lm && ./a.out 20000 2000
 * measured here: 560,000,000 cases, 0 mismatches. */
#include <stdio.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s=88172645463325252ull;
static inline uint64_t rnd(){ s^=s<<13; s^=s>>7; s^=s<<17; return s; }
static double mk(uint64_t mant, int e){ uint64_t b=(mant&0x000fffffffffffffull)|((uint64_t)(1023+e)<<52); double d; memcpy(&d,&b,8); return d; }
int main(int argc,char**argv){
  long NB=atol(argv[1]), M=atol(argv[2]); long bad=0,tot=0;
  for(long nb=0; nb<NB; nb++){
    uint64_t m;
    switch(nb%4){case 0: m=rnd(); break; case 1: m=0x000fffffffffffffull ^ (rnd()&0xff); break; case 2: m=rnd()&0xff; break; default: m=0x000fffffffffffffull;}
    double d=mk(m, (int)(rnd()%40)-20), r=1.0/d;
    for(long i=0;i<M;i++){
      double q=mk(rnd(), (int)(rnd()%60)-30);
      double qn=nextafter(q,INFINITY);
      long double mid=((long double)q+(long double)qn)/2;
      for(int k=-3;k<=3;k++){
        double x=(double)(mid*(long double)d);
        for(int j=0;j<k;j++) x=nextafter(x,INFINITY);
        for(int j=0;j>k;j--) x=nextafter(x,-INFINITY);
        double q0=x*r, ee=fma(-q0,d,x), q1=fma(ee,r,q0);
        double ref=x/d; tot++;
        if(q1!=ref){ if(bad<10) printf("d=%a x=%a q1=%a ref=%a\n",d,x,q1,ref); bad++; }
        double xr=mk(rnd(), (int)(rnd()%60)-30); q0=xr*r; ee=fma(-q0,d,xr); q1=fma(ee,r,q0); tot++;
        if(q1!=xr/d){ if(bad<10) printf("rand d=%a x=%a\n",d,xr); bad++; }
      }
    }
  }
  printf("cases=%ld bad=%ld\n",tot,bad); return 0; }
