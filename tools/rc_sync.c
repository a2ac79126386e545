// rc_sync.c — does the fqz range chain re-synchronise from a wrong start?
// Simulates range = renorm(floor(range/T) * f) over synthetic (f, T) events
// and restarts it at 200 points from a guessed range.
// gcc -O2 -o /tmp/rc_sync tools/rc_sync.c && /tmp/rc_sync
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
static uint64_t s=88172645463325252ull; static inline uint64_t rnd(){ s^=s<<13; s^=s>>7; s^=s<<17; return s; }
int main(int argc,char**argv){
  int N=2000000; uint32_t *f=malloc(N*4),*T=malloc(N*4);
  double P[4]={.85,.10,.04,.01};
  for(int i=0;i<N;i++){ uint32_t t=4096+rnd()%61000; double u=(rnd()%1000000)/1e6; int k=u<.85?0:u<.95?1:u<.99?2:3; uint32_t ff=(uint32_t)(P[k]*t); if(!ff)ff=1; f[i]=ff; T[i]=t; }
  uint32_t *R=malloc((N+1)*4); uint32_t r=0xFFFFFFFFu; R[0]=r;
  for(int i=0;i<N;i++){ uint32_t q=r/T[i]; r=q*f[i]; while(r<(1u<<24)) r<<=8; R[i+1]=r; }
  // start guesses at many points
  long tot=0; int fails=0, M=200; long mx=0;
  for(int j=0;j<M;j++){ int st=1000+j*9000; uint32_t g=(argc>1)?(uint32_t)(rnd()|0x01000000u):0xFFFFFFFFu; int i=st; for(;i<N && g!=R[i];i++){ uint32_t q=g/T[i]; g=q*f[i]; while(g<(1u<<24)) g<<=8; }
    if(i>=N) fails++; else { tot+=i-st; if(i-st>mx) mx=i-st; } }
  printf("merged %d/%d, mean steps %.1f, max %ld\n", M-fails, M, (double)tot/(M-fails>0?M-fails:1), mx);
}
