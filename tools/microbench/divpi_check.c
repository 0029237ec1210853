// divpi_check.c -- exhaustive CPU check that x * RN(1/pi) corrected by one fma residual step equals
// the IEEE quotient x / pi for every fp32 x in [2^-100, 4] (vr_sampling.h divpi).  gcc -O2 -mfma -ffp-contract=off
#include <stdio.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
int main(){
  const float PI=3.14159265358979323846f; const float R=1.0f/PI;
  uint64_t bad=0, n=0; float fb=0;
  for (uint32_t u=0; u<=0x40800000u; ++u){ float x; memcpy(&x,&u,4);
    float q=x/PI; float q0=x*R; float r=fmaf(-q0,PI,x); float q1=fmaf(r,R,q0);
    uint32_t a,b; memcpy(&a,&q,4); memcpy(&b,&q1,4); n++;
    if(a!=b && x>0x1p-100f){ if(!bad) fb=x; bad++; } }
  printf("R=%a n=%lu bad=%lu first=%a\n",R,n,bad,fb);
}
