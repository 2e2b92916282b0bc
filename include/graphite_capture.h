/*
 * graphite_capture.h — C ABI of the trace-capture front end (libgg_capture.so).
 *
 * Replaces the reference's Pin-based capture of application memory operands
 * (pin/lite/memory_modeling.cc:13-89, which hands every load/store to
 * Core::initiateMemoryAccess, tile/core/core.cc:139-266) for the SPLASH-2 FFT
 * of BASELINE configs[0] (tests/benchmarks/fft/fft.C, -p16 -m20): the FFT is
 * instrumented at the source level and its 8-byte shared-array accesses are
 * written as per-thread traces in the gg_trace format of graphite_gpu.h
 * (thread t = tile t; meta = WRITE bit | gap cycles << 1).
 */
#ifndef GRAPHITE_CAPTURE_H
#define GRAPHITE_CAPTURE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Run a forward six-step FFT of 2^m complex points on p threads (m even,
 * 2 <= m <= 24; p a power of two <= 2^(m/2)) and capture its traces.
 * Returns a handle, NULL on a bad argument.                                */
void* gg_fft_capture_create(uint32_t m, uint32_t p);
/* counts[t] = records of thread t (p entries).                             */
void  gg_fft_capture_counts(void* h, uint64_t* counts);
/* Thread-major trace: addr[], meta[] sized by the sum of the counts.       */
void  gg_fft_capture_copy(void* h, uint64_t* addr, uint32_t* meta);
/* The transform X[k] (re, im), natural order, 2 * 2^m doubles.             */
void  gg_fft_capture_output(void* h, double* out);
/* The input x[j] (re, im) of an m-sized capture, 2 * 2^m doubles.          */
void  gg_fft_capture_input(uint32_t m, double* out);
void  gg_fft_capture_destroy(void* h);

#ifdef __cplusplus
}
#endif
#endif
