/* parmacs.h — the PARMACS macros SPLASH-2 FFT is written in
 * (tests/benchmarks/fft/fft.C), as C preprocessor macros over the trace
 * capture runtime (fft_capture_rt.cpp).  The reference expands them with m4
 * and tests/benchmarks/splash_support/c.m4.null.POSIX (m4 is not installed
 * here); these definitions restate that file's semantics — pthreads,
 * CREATE = spawn P-1 threads then run the function on the main thread,
 * WAIT_FOR_END = join them, a counting barrier, malloc for G_MALLOC — with
 * three capture hooks: thread ids are handed out in a fixed order (the main
 * thread takes ProcID 0, spawned thread i takes i), BARRIER records its
 * position in the calling thread's trace, and heap memory comes from one
 * arena so recorded addresses do not depend on ASLR.
 * Force-included (-include) ahead of fft.C; used only by this capture tool.  */
#ifndef GG_PARMACS_H
#define GG_PARMACS_H
#include <pthread.h>
#include <stdlib.h>
#include <sys/time.h>
#include <unistd.h>

#ifdef __cplusplus
extern "C" {
#endif
void* gg_cap_malloc(size_t n);
void  gg_cap_create(void (*fn)(void), long p);
void  gg_cap_wait(long p);
void  gg_cap_lock(pthread_mutex_t* l);
void  gg_cap_unlock(pthread_mutex_t* l);
void  gg_cap_barrier_init(long n);
void  gg_cap_barrier(void);
void  CarbonEnableModels(void);
void  CarbonDisableModels(void);
#ifdef __cplusplus
}
#endif

#define MAIN_ENV
#define MAIN_INITENV(a, b) {;}
#define MAIN_END {return(0);}
#define CREATE(fn, p) { gg_cap_create((void (*)(void))(fn), (p)); }
#define WAIT_FOR_END(p) { gg_cap_wait(p); }
#define LOCKDEC(l) pthread_mutex_t l;
#define LOCKINIT(l) {pthread_mutex_init(&(l), NULL);}
#define LOCK(l) { gg_cap_lock(&(l)); }
#define UNLOCK(l) { gg_cap_unlock(&(l)); }
#define BARDEC(b) long b;
#define BARINIT(b, n) { gg_cap_barrier_init(n); }
#define BARRIER(b, n) { gg_cap_barrier(); }
#define BARINCLUDE(b) {;}
#define G_MALLOC(n) gg_cap_malloc(n);
#define CLOCK(t) { struct timeval FullTime; gettimeofday(&FullTime, NULL); \
                   (t) = (unsigned long)(FullTime.tv_usec + FullTime.tv_sec * 1000000); }
/* the per-thread malloc of SlaveStart (upriv) from the same arena */
#define malloc(n) gg_cap_malloc(n)
#endif
