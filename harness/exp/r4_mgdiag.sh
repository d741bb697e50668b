#!/bin/bash
# r4: merge-pass time split (timing-only builds, invalid output): MGX_NOMERGE (real co-ranks,
# geometry, loads and stores; the LDS merge replaced by a copy) and MGX_PROLOGUE_ONLY.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
for i in 1 2 3; do
  for L in base nomerge pro net net8; do
    ALGO=merge LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$L.so" timeout -k 10 120 python "$R/harness/exp/hist_time.py" || exit 1
  done
done
LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_net.so" timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sort.py -k "merge or tile" > gpurun_out/net_tests.log 2>&1 || { tail -30 gpurun_out/net_tests.log; exit 1; }
echo "net: $(tail -1 gpurun_out/net_tests.log)"
LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_net8.so" timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sort.py -k "merge or tile" > gpurun_out/net8_tests.log 2>&1 || { tail -30 gpurun_out/net8_tests.log; exit 1; }
echo "net8: $(tail -1 gpurun_out/net8_tests.log)"
