#!/bin/bash
# r4: key/value merge pass with the transposed nontemporal stores (product build) against
# the r28 base build (keys only): the pairs tests, then bench --algo pairs --pair-algo merge
# alternating.  Each step has its own limit; the first failure ends it.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sort.py -k "pairs or merge or tile" > gpurun_out/kv_tests.log 2>&1 || { tail -30 gpurun_out/kv_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/kv_tests.log)"
for i in 1 2; do
  for L in "$R/harness/exp/libs/liblabsort_base.so" "$R/radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so"; do
    LABSORT_LIBRARY="$L" timeout -k 10 300 python bench.py --algo pairs --pair-algo merge --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/kv_bench.json 2> gpurun_out/kv_bench.err || { tail -20 gpurun_out/kv_bench.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/kv_bench.json').read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], d['roofline']['achieved'], d['roofline'].get('copy_frac'))
" "$L"
  done
done
