/*
 * include/lab.h -- drop-in replacement for the reference's `Sord Radix y Merge/include/lab.h`.
 *
 * Same two declarations with the same C++ linkage (mangled _Z11order_arrayPii and
 * _Z16order_with_trustPii), so the reference's main.cpp and performanceTest.cpp
 * compile and link unchanged against liblabsort.so.
 *
 *   order_array      lab.h:9  / lab.cu:303  sort `length` ints in place (host
 *                    pointer, synchronous) on the MI355X; default algorithm
 *                    LABSORT_ALGO_AUTO (merge path up to 2^16 keys and past the
 *                    radix limit, LSD radix between); LABSORT_ALGO=radix|merge|radix1
 *                    selects one; LABSORT_GPUS=p sorts across devices 0..p-1.
 *   order_with_trust lab.h:10 / lab.cu:404  thrust::sort on the host pointer
 *                    (rocThrust, sequential CPU backend: the reference's semantics).
 */
#ifndef LAB_LAB_H
#define LAB_LAB_H

#include "utils.h"
void order_array (int * srcCpu, int length);
void order_with_trust(int * src, int length);

#endif /* LAB_LAB_H */
