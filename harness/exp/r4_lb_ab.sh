#!/bin/bash
# r4 A/B: the onesweep pass's look-back window loaded at the end of the previous
# iteration, with a fixed count of tile loads (harness/exp/libs/liblabsort_lbtop4.so) vs
# the product (liblabsort_base.so).  Radix / pairs tests with the variant first; each GPU
# step has its own time limit.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
V="harness/exp/libs/liblabsort_lbtop4.so"
LABSORT_LIBRARY="$R/$V" timeout -k 10 500 python -u -m pytest "$R/tests/test_gpu_sort.py" "$R/tests/test_gpu_fullsize.py" -m gpu -x -q \
    -k "radix or sort_device or onesweep or pairs or segment or timing" --timeout 150 --timeout-method thread -p no:cacheprovider > "$O/lb_pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/lb_pytest.log"; [ $rc -eq 0 ] || exit $rc
bash "$R/harness/exp/ab_libs.sh" radix harness/exp/libs/liblabsort_base.so "$V" 4 || exit 1
for L in harness/exp/libs/liblabsort_base.so "$V" harness/exp/libs/liblabsort_base.so "$V"; do
  LABSORT_LIBRARY="$R/$L" timeout -k 10 200 python "$R/bench.py" --algo pairs --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > "$O/lb_pairs.json" 2>"$O/lb_pairs.err" || { tail -5 "$O/lb_pairs.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lb_pairs.json')); print('$L'.split('/')[-1], 'pairs radix ms', d['ms_per_step'], d['roofline'].get('avg_launch_ms'))"
done
