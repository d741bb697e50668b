#!/bin/bash
# r6: write-path probe, per-pass onesweep times by n (item 3b: does a
# pass over an Infinity-Cache-sized array run faster per key?), and the GPU tests touched
# by this round's first changes.  Every GPU step has its own time limit; the first failure
# ends the script.
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
timeout -k 10 120 "$R/harness/bin/write_probe" > "$O/r6_write_probe.txt" 2>&1
for lg in 22 23 24 25 26 27 28; do
  LABSORT_RADIX_IMPL=onesweep timeout -k 10 150 python3 bench.py --log2n $lg --steps 20 --warmup 3 --no-merge \
    --no-cpu-baseline --no-host-path > "$O/r6_ic_$lg.json" 2> "$O/r6_ic_$lg.err"
  echo "2^$lg done"
done
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dist.py tests/test_gpu_multi.py "tests/test_gpu_sort.py::test_c_abi_sort_symbols_match_std_sort" \
  "tests/test_gpu_fullsize.py::test_fullsize_sha_i32" "tests/test_gpu_fullsize.py::test_fullsize_order_array_i32_2e30" \
  > "$O/r6_tests1.log" 2>&1
tail -3 "$O/r6_tests1.log"
