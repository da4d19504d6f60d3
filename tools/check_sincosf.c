/* Exhaustive check that the glibc 2.35 sinf/cosf restatement (same constants and fma placement as
 * openmavis_amd/csrc/omv_device.h::glibc_sincosf) is bit-identical to the host libm over every float
 * in [0, 2*pi].  gcc -O2 -ffp-contract=off -DUSEFMA tools/check_sincosf.c -lm && ./a.out */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
typedef struct { double sign[4]; double hpi_inv, hpi, c0,c1,c2,c3,c4, s1,s2,s3; } tab_t;
/* order in glibc struct: sign, hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3 */
static const tab_t T[2] = {
 {{1.0,-1.0,-1.0,1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0,
  0x1p0, -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16,
  -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
 {{1.0,-1.0,-1.0,1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0,
  -0x1p0, 0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16,
  -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};
static inline uint32_t top12(float x){uint32_t u; memcpy(&u,&x,4); return (u>>20)&0x7ff;}
#ifdef USEFMA
#define MA(a,b,c) fma(a,b,c)
#else
#define MA(a,b,c) ((a)*(b)+(c))
#endif
static inline float poly(double x,double x2,const tab_t*p,int n){
  if((n&1)==0){ double x3=x*x2; double s1=MA(x2,p->s3,p->s2); double x7=x3*x2; double s=MA(x3,p->s1,x); return (float)MA(x7,s1,s);}
  else { double x4=x2*x2; double c2=MA(x2,p->c4,p->c3); double c1=MA(x2,p->c1,p->c0); double x6=x4*x2; double c=MA(x4,p->c2,c1); return (float)MA(x6,c2,c);}
}
static inline double red(double x,const tab_t*p,int*np){ double r=x*p->hpi_inv; int n=((int32_t)r+0x800000)>>24; *np=n; return MA(-(double)n,p->hpi,x);}
float mycos(float y){ double x=y; const tab_t*p=&T[0]; int n;
  if(top12(y)<top12(0x1.921FB6p-1f)){ if(top12(y)<top12(0x1p-12f)) return 1.0f; return poly(x,x*x,p,1);}
  x=red(x,p,&n); double s=p->sign[n&3]; if(n&2) p=&T[1]; return poly(x*s,x*x,p,n^1);}
float mysin(float y){ double x=y; const tab_t*p=&T[0]; int n;
  if(top12(y)<top12(0x1.921FB6p-1f)){ if(top12(y)<top12(0x1p-12f)) return y; return poly(x,x*x,p,0);}
  x=red(x,p,&n); double s=p->sign[n&3]; if(n&2) p=&T[1]; return poly(x*s,x*x,p,n);}
#ifndef STRIDE
#define STRIDE 1
#endif
int main(){ long bc=0,bs=0,tot=0; float lim=6.2831855f; uint32_t u0=0, u1; memcpy(&u1,&lim,4);
 for(uint32_t u=u0; u<=u1; u+=STRIDE){ float x; memcpy(&x,&u,4); tot++;
   volatile float c=cosf(x), s=sinf(x); float mc=mycos(x), ms=mysin(x);
   if(memcmp((const void*)&c,&mc,4)) { if(bc<5) printf("cos mismatch %a %a %a\n",x,c,mc); bc++;}
   if(memcmp((const void*)&s,&ms,4)) { if(bs<5) printf("sin mismatch %a %a %a\n",x,s,ms); bs++;} }
 printf("tot %ld cos_bad %ld sin_bad %ld\n",tot,bc,bs); }
