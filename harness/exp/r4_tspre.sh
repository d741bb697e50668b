#!/bin/bash
# r4: tile sort with a per-wave, per-pass pre-check for wave-uniform digits (MGX_TSPRE) so
# the common case ranks with branch-free returning atomics; alternating with the shipped
# build, then the merge / tile / pairs tests on the variant.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  for L in base tspre; do
    ALGO=merge LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$L.so" timeout -k 10 120 python "$R/harness/exp/hist_time.py" || exit 1
  done
done
LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_tspre.so" timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sort.py -k "merge or tile or pairs" > gpurun_out/tspre_tests.log 2>&1 || { tail -30 gpurun_out/tspre_tests.log; exit 1; }
echo "tspre: $(tail -1 gpurun_out/tspre_tests.log)"
