// Exhaustive check of arl::div255 (arl_internal.hpp): x * RN(1/255) corrected by one fma residual
// step against IEEE x / 255.f over every finite f32 (about 70 s):
//   gcc -O2 -o /tmp/div255_check scripts/div255_check.c -lm && /tmp/div255_check
// prints "bad 1 (non-denormal results 0) first 80000000": only x = -0 differs (+0 returned).
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
int main(){
  const float y=255.f; const float inv = 1.f/255.f;
  uint64_t bad=0, badnd=0; uint32_t firstbad=0;
  for (uint64_t u=0; u<0x100000000ull; ++u){
    uint32_t b=(uint32_t)u; float x; memcpy(&x,&b,4);
    if (!isfinite(x)) continue;
    float q=x*inv; float r=fmaf(-q,y,x); float q2=fmaf(r,inv,q);
    float t=x/y;
    if (memcmp(&q2,&t,4)!=0){ if(!bad) firstbad=b; ++bad; if (fabsf(t) >= 1.17549435e-38f) ++badnd; }
  }
  printf("bad %llu (non-denormal results %llu) first %08x\n",(unsigned long long)bad,(unsigned long long)badnd,firstbad);
}
