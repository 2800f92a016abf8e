// Host check of the PL-ICP float atan bracket (csrc/plicp_kernels.hip pl_fatan01 / pl_fatan / pl_fatan2): the
// worst error must stay well under PL_ATAN_EPS = 2e-6.  gcc -O2 -fopenmp tools/check_fatan.c -lm (about 3 min)
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static inline float f01(float t, int fma_){
  float z=t*t, q=-0.003962602f;
  const float c[7]={0.021518489f,-0.055396412f,0.096028686f,-0.13892588f,0.19943212f,-0.33329552f,0.99999923f};
  for(int i=0;i<7;i++) q = fma_ ? fmaf(z,q,c[i]) : c[i]+z*q;
  return t*q;
}
static inline float fat(float x,int m){ return x>1.0f ? 1.5707963f - f01(1.0f/x,m) : f01(x,m);}
static inline float fat2(float y,float x,int m){ float ax=fabsf(x),ay=fabsf(y);
  float r = ay>ax ? 1.5707963f - f01(ax/ay,m) : f01(ay/ax,m); if(x<0.0f) r=3.1415927f-r; return y<0.0f?-r:r;}
int main(){
  for(int m=0;m<2;m++){
    double worst=0; float wx=0;
    #pragma omp parallel
    { double lw=0; float lx=0;
      #pragma omp for schedule(static)
      for(int64_t b=0;b<0x7F800000LL;b++){ uint32_t u=(uint32_t)b; float x; memcpy(&x,&u,4);
        double e=fabs((double)fat(x,m)-atan((double)x)); if(e>lw){lw=e;lx=x;} }
      #pragma omp critical
      if(lw>worst){worst=lw;wx=lx;}
    }
    printf("fma=%d atan max err %.3e at %g\n",m,worst,wx);
    // atan2: random pairs incl. double->float rounding of args
    srand48(1); double w2=0;
    for(long i=0;i<200000000L;i++){ double y=(drand48()-0.5)*pow(10,drand48()*12-6), x=(drand48()-0.5)*pow(10,drand48()*12-6);
      if(i%4==1) y = x*(1+1e-9*(drand48()-0.5)); if(i%4==2) y=-x*(1+1e-7*(drand48()-.5));
      float fx=(float)x, fy=(float)y; if(fx==0||fy==0) continue;
      double e=fabs((double)fat2(fy,fx,m)-atan2(y,x)); if(e>2*M_PI-1) e=fabs(e-2*M_PI); if(e>w2) w2=e; }
    printf("fma=%d atan2 max err %.3e\n",m,w2);
  }
}
