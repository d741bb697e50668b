#!/bin/bash
# r4: merge pass with 1024-thread workgroups (MGX_BLOCK=1024: 8192-key tiles) against the
# shipped 512: per-class launch times alternating; then the merge tests on the variant.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  for L in base b1024; do
    ALGO=merge LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$L.so" timeout -k 10 120 python "$R/harness/exp/hist_time.py" || exit 1
  done
done
LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_b1024.so" timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sort.py -k "merge or tile" > gpurun_out/b1024_tests.log 2>&1 || { tail -30 gpurun_out/b1024_tests.log; exit 1; }
echo "b1024: $(tail -1 gpurun_out/b1024_tests.log)"
