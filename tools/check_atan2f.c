/* Check that the glibc fdlibm atan2f restatement (same constants and operation order as
 * openmavis_amd/csrc/omv_device.h::glibc_atan2f, used by KannalaBrandt8::project) is bit-identical to the
 * host libm.  Random bit patterns + integer / scaled-integer grids; 200M pairs by default (0 mismatches),
 * -DN=... for a shorter run.  gcc -O2 -ffp-contract=off tools/check_atan2f.c -lm && ./a.out */
#ifndef N
#define N 200000000L
#endif
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static inline uint32_t fbits(float f){uint32_t u; memcpy(&u,&f,4); return u;}
static inline float bitsf(uint32_t u){float f; memcpy(&f,&u,4); return f;}
static const float atanhi[] = {4.6364760399e-01f,7.8539812565e-01f,9.8279368877e-01f,1.5707962513e+00f};
static const float atanlo[] = {5.0121582440e-09f,3.7748947079e-08f,3.4473217170e-08f,7.5497894159e-08f};
static const float aT[] = {3.3333334327e-01f,-2.0000000298e-01f,1.4285714924e-01f,-1.1111110449e-01f,9.0908870101e-02f,
 -7.6918758452e-02f,6.6610731184e-02f,-5.8335702866e-02f,4.9768779427e-02f,-3.6531571299e-02f,1.6285819933e-02f};
float my_atanf(float x){ float w,s1,s2,z; int32_t ix,hx,id; hx=(int32_t)fbits(x); ix=hx&0x7fffffff;
 if(ix>=0x4c000000){ if(ix>0x7f800000) return x+x; if(hx>0) return atanhi[3]+atanlo[3]; else return -atanhi[3]-atanlo[3]; }
 if(ix<0x3ee00000){ if(ix<0x31000000) return x; id=-1; }
 else { x=fabsf(x); if(ix<0x3f980000){ if(ix<0x3f300000){ id=0; x=(2.0f*x-1.0f)/(2.0f+x);} else { id=1; x=(x-1.0f)/(x+1.0f);} }
        else { if(ix<0x401c0000){ id=2; x=(x-1.5f)/(1.0f+1.5f*x);} else { id=3; x=-1.0f/x; } } }
 z=x*x; w=z*z;
 s1=z*(aT[0]+w*(aT[2]+w*(aT[4]+w*(aT[6]+w*(aT[8]+w*aT[10])))));
 s2=w*(aT[1]+w*(aT[3]+w*(aT[5]+w*(aT[7]+w*aT[9]))));
 if(id<0) return x-x*(s1+s2);
 z=atanhi[id]-((x*(s1+s2)-atanlo[id])-x); return (hx<0)?-z:z; }
static const float pi_o_4=7.8539818525e-01f, pi_o_2=1.5707963705e+00f, pi=3.1415927410e+00f, pi_lo=-8.7422776573e-08f, tiny=1.0e-30f;
float my_atan2f(float y,float x){ float z; int32_t k,m,hx,hy,ix,iy; hx=(int32_t)fbits(x); ix=hx&0x7fffffff; hy=(int32_t)fbits(y); iy=hy&0x7fffffff;
 if(ix>0x7f800000||iy>0x7f800000) return x+y;
 if(hx==0x3f800000) return my_atanf(y);
 m=((hy>>31)&1)|((hx>>30)&2);
 if(iy==0){ switch(m){case 0: case 1: return y; case 2: return pi+tiny; case 3: return -pi-tiny;} }
 if(ix==0) return (hy<0)? -pi_o_2-tiny: pi_o_2+tiny;
 if(ix==0x7f800000){ if(iy==0x7f800000){ switch(m){case 0: return pi_o_4+tiny; case 1: return -pi_o_4-tiny; case 2: return 3.0f*pi_o_4+tiny; case 3: return -3.0f*pi_o_4-tiny;} }
   else { switch(m){case 0: return 0.0f; case 1: return -0.0f; case 2: return pi+tiny; case 3: return -pi-tiny;} } }
 if(iy==0x7f800000) return (hy<0)? -pi_o_2-tiny: pi_o_2+tiny;
 k=(iy-ix)>>23;
 if(k>60) z=pi_o_2+0.5f*pi_lo; else if(hx<0&&k<-60) z=0.0f; else z=my_atanf(fabsf(y/x));
 switch(m){ case 0: return z; case 1: return bitsf(fbits(z)^0x80000000u); case 2: return pi-(z-pi_lo); default: return (z-pi_lo)-pi; } }
static uint64_t s=88172645463325252ull; static inline uint64_t xr(){ s^=s<<13; s^=s>>7; s^=s<<17; return s; }
int main(){ long bad=0, n=0;
 for(long i=0;i<N;i++){ uint64_t r=xr(); float y,x;
   if(i%3==0){ y=bitsf((uint32_t)r); x=bitsf((uint32_t)(r>>32)); if(isnan(x)||isnan(y)) continue; }
   else { y=(float)((int32_t)(r&0xffffff)-(1<<23))*(i%3==1?1.0f:0.001f); x=(float)((int32_t)((r>>24)&0xffffff)-(1<<23))*(i%3==1?1.0f:0.001f); }
   volatile float a=atan2f(y,x); float b=my_atan2f(y,x); n++;
   if(fbits(a)!=fbits(b)){ if(bad<5) printf("mismatch y=%a x=%a libm=%a mine=%a\n",y,x,a,b); bad++; } }
 printf("n %ld bad %ld\n",n,bad); }
