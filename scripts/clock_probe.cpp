// Clock-read costs on a host (profiles/box_r5_clock/): g++ -O2 -o clock_probe scripts/clock_probe.cpp
#include <cstdio>
#include <ctime>
#include <cstdint>
#include <x86intrin.h>
static inline int64_t ns(clockid_t c){timespec t;clock_gettime(c,&t);return t.tv_sec*1000000000LL+t.tv_nsec;}
int main(){
  const int N=5000000; volatile int64_t sink=0;
  clockid_t ids[4]={CLOCK_MONOTONIC,CLOCK_REALTIME,CLOCK_MONOTONIC_COARSE,CLOCK_REALTIME_COARSE};
  const char* names[4]={"MONOTONIC","REALTIME","MONOTONIC_COARSE","REALTIME_COARSE"};
  for(int k=0;k<4;k++){int64_t t0=ns(CLOCK_MONOTONIC);for(int i=0;i<N;i++)sink+=ns(ids[k]);int64_t t1=ns(CLOCK_MONOTONIC);printf("%s %.2f ns\n",names[k],double(t1-t0)/N);}
  int64_t t0=ns(CLOCK_MONOTONIC);for(int i=0;i<N;i++)sink+=__rdtsc();int64_t t1=ns(CLOCK_MONOTONIC);printf("rdtsc %.2f ns\n",double(t1-t0)/N);
  unsigned a; t0=ns(CLOCK_MONOTONIC);for(int i=0;i<N;i++)sink+=__rdtscp(&a);t1=ns(CLOCK_MONOTONIC);printf("rdtscp %.2f ns\n",double(t1-t0)/N);
  timespec r; clock_getres(CLOCK_REALTIME_COARSE,&r); printf("coarse res %ld ns\n", r.tv_nsec);
  return 0;}
