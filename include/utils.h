/*
 * include/utils.h -- drop-in replacement for `Sord Radix y Merge/include/utils.h`.
 *
 * Provides what the reference's callers rely on (utils.h:20-48) without any
 * CUDA header: the C/C++ standard headers main.cpp uses for malloc/rand/srand/
 * free/clock_gettime, the CUDA_CHK/gpuAssert error policy (print "GPUassert: ..."
 * and exit with the code) and the MS wall-clock macro, token-identical to the
 * copy performanceTest.cpp:9-17 re-defines (so that redefinition is benign).
 */
#ifndef LAB_UTILS_H
#define LAB_UTILS_H

#include "math.h"
#include <algorithm>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <stdlib.h>

/* from liblabsort.so (include/labsort.h); declared here so callers see no other symbol */
extern "C" const char *labsort_hip_error_string(int hip_error);

/* CUDA_CHK(ans): `ans` is a hipError_t (or any int status of the HIP runtime). */
#define CUDA_CHK(ans) { gpuAssert((ans), __FILE__, __LINE__); }
inline void gpuAssert(int code, const char *file, int line, bool abort=true)
{
    if (code != 0)
    {
        fprintf(stderr,"GPUassert: %s %s %d\n", labsort_hip_error_string(code), file, line);
        if (abort) exit(code);
    }
}

#define MS(f,elap)                                                                                           \
        double elap=0;                                                                                       \
        {                                                                                                    \
        struct timespec t_ini,t_fin;                                                                         \
            clock_gettime(CLOCK_MONOTONIC, &t_ini);                                                          \
            f;                                                                                               \
            clock_gettime(CLOCK_MONOTONIC, &t_fin);                                                          \
            elap = 1000 * (t_fin.tv_sec - t_ini.tv_sec) + (t_fin.tv_nsec - t_ini.tv_nsec)/1000000.0;         \
        }

#endif /* LAB_UTILS_H */
