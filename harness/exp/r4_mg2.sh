#!/bin/bash
# r4: merge pass with nontemporal loads (MGX_NT) and 8192-key tiles (MGX_KPT=16) against the
# shipped build: per-class launch times, alternating; then the merge tests on each variant.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  for L in base mnt k16 k16nt; do
    ALGO=merge LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$L.so" timeout -k 10 120 python "$R/harness/exp/hist_time.py" || exit 1
  done
done
for L in mnt k16 k16nt; do
  LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$L.so" timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sort.py -k "merge or tile" > gpurun_out/mg2_tests_$L.log 2>&1 || { tail -30 gpurun_out/mg2_tests_$L.log; exit 1; }
  echo "$L: $(tail -1 gpurun_out/mg2_tests_$L.log)"
done
