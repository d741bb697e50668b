#!/bin/bash
# r4: onesweep scatter with nontemporal 16-B stores (OSX_NT build): per-class launch times,
# alternating with the base build; then the radix GPU tests on the variant.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  for L in base osnt2; do
    ALGO=radix LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$L.so" timeout -k 10 120 python "$R/harness/exp/hist_time.py" || exit 1
  done
done
L=osnt2
LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$L.so" timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sort.py -k "radix" > gpurun_out/osx_tests_$L.log 2>&1 || { tail -30 gpurun_out/osx_tests_$L.log; exit 1; }
echo "$L: $(tail -1 gpurun_out/osx_tests_$L.log)"
