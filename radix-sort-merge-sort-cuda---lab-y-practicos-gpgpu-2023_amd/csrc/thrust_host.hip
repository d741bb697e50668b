// thrust_host.hip -- order_with_trust (lab.cu:404-406), the reference's comparator.
//
// thrust::sort on raw host pointers dispatches to Thrust's host (sequential CPP)
// backend -- a single-core radix sort on the CPU, not a GPU sort.
// Compiled against rocThrust (ROCm 7.2), which keeps that dispatch, so this is
// the same algorithm the reference timed as "Trust".  LABSORT_VERIFY=1 checks the
// result as for order_array (api.hip).
#include <thrust/sort.h>

#include "common.h"

void order_with_trust(int *src, int length) {
    if (length <= 0) return;
    const bool verify = labsort::verify_enabled();
    labsort::KeyPrint before{};
    if (verify) before = labsort::key_print(src, (size_t)length);
    thrust::sort(src, src + length);
    if (verify) labsort::verify_or_exit("order_with_trust", src, (size_t)length, before);
}
