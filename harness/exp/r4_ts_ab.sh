#!/bin/bash
# r4 A/B of the tile sort (LABSORT_TS_IMPL=p: persistent pipelined 512 x 64) on the merge
# sort: correctness tests of the merge path with the variant, then the bench's merge leg.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
LABSORT_TS_IMPL=p timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_sort.py" -m gpu -x -q -k "tile or merge or small or sort_device" --timeout 150 --timeout-method thread -p no:cacheprovider > "$O/ts_ab_pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$O/ts_ab_pytest.log"
[ $rc -le 1 ] || exit $rc
for impl in p x p x; do
  LABSORT_TS_IMPL=$impl timeout -k 10 200 python "$R/bench.py" --algo merge --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > "$O/ts_ab_$impl.json" 2>"$O/ts_ab_$impl.err" || { tail -5 "$O/ts_ab_$impl.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/ts_ab_$impl.json')); print('$impl', d['ms_per_step'], d['roofline'].get('avg_launch_ms'))"
done
