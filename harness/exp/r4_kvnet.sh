#!/bin/bash
# r4: key/value merge pass with the (key, slot) network (MGX_KVNET build) against the shipped
# build: the pairs / merge tests on the variant, then bench --algo pairs --pair-algo merge
# alternating.  Each step has its own limit; the first failure ends it.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_kvnet.so" timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sort.py -k "pairs or merge or tile" > gpurun_out/kvnet_tests.log 2>&1 || { tail -30 gpurun_out/kvnet_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/kvnet_tests.log)"
for i in 1 2; do
  for L in base kvnet; do
    LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$L.so" timeout -k 10 300 python bench.py --algo pairs --pair-algo merge --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/kvnet_bench.json 2> gpurun_out/kvnet_bench.err || { tail -20 gpurun_out/kvnet_bench.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/kvnet_bench.json').read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], d['value'], d['roofline']['achieved'])
" "$L"
  done
done
