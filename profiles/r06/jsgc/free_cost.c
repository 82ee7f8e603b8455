#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sys/mman.h>
static double now(){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec*1e3+t.tv_nsec/1e6;}
int main(){
  for(int r=0;r<3;r++){
    size_t n=32u<<20;
    char*p=calloc(1,n); memset(p,1,n);
    double t0=now(); free(p); double t1=now();
    char*q=mmap(0,n,PROT_READ|PROT_WRITE,MAP_PRIVATE|MAP_ANONYMOUS,-1,0); madvise(q,n,MADV_HUGEPAGE); memset(q,1,n);
    double t2=now(); munmap(q,n); double t3=now();
    printf("free(32MiB 4K pages) %.3f ms   munmap(32MiB THP) %.3f ms\n",t1-t0,t3-t2);
  }
}
