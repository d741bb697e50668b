// thrust_host.hip -- order_with_trust (lab.cu:404-406), the reference's comparator.
//
// thrust::sort on raw host pointers dispatches to Thrust's host (sequential CPP)
// backend -- a single-core radix sort on the CPU, not a GPU sort.
// Compiled against rocThrust (ROCm 7.2), which keeps that dispatch, so this is
// the same algorithm the reference timed as "Trust".
#include <thrust/sort.h>

void order_with_trust(int *src, int length) { thrust::sort(src, src + length); }
