#!/bin/bash
# r6: onesweep pass A/B -- the working tree's build against harness/bin/ab builds named in
# VARS: radix tests with each variant as the library, then alternating 2^28 keys-only
# sorts (pairs_ab.py MODE=keys) and per-kernel rocprof times.
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
TAG=${TAG:-osab}
VARS="${VARS:-base}"
for v in $VARS; do
  LABSORT_LIBRARY="$R/harness/bin/ab/liblabsort_$v.so" timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_sort.py -k "sort_device or order_array or sort_host or pass_structure or segment" > "$O/${TAG}_${v}_tests.log" 2>&1
  tail -1 "$O/${TAG}_${v}_tests.log"
  LABSORT_LIBRARY="$R/harness/bin/ab/liblabsort_$v.so" timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_fullsize.py -k "fullsize_sha or inplace_repeat" > "$O/${TAG}_${v}_full.log" 2>&1
  tail -1 "$O/${TAG}_${v}_full.log"
done
MODE=keys timeout -k 10 300 python3 -u harness/exp/pairs_ab.py radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so \
  $(for v in $VARS; do echo harness/bin/ab/liblabsort_$v.so; done) ${REPS:-4} > "$O/${TAG}_ab.log" 2>&1
cat "$O/${TAG}_ab.log"
