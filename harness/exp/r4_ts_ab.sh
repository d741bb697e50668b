#!/bin/bash
# r4 A/B of the merge sort's tile sort (LABSORT_TS_IMPL): 3 = three 11/11/10-bit LDS
# passes (512 x 64), p = persistent pipelined 512 x 64 with four 8-bit passes, x = the
# shipped 1024 x 32 four-pass kernel.  Merge-path tests with each variant, then the
# bench's merge leg alternating the variants.  Each GPU step has its own time limit.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for impl in ${TS_IMPLS:-3 p}; do
  LABSORT_TS_IMPL=$impl timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_sort.py" "$R/tests/test_gpu_fullsize.py" -m gpu -x -q \
      -k "tile_sort or merge or sort_device_uniform or sort_device_distributions" --timeout 150 --timeout-method thread -p no:cacheprovider > "$O/ts_ab_pytest_$impl.log" 2>&1
  rc=$?; echo "pytest $impl rc=$rc"; tail -3 "$O/ts_ab_pytest_$impl.log"
  [ $rc -eq 0 ] || exit $rc
done
for impl in x ${TS_IMPLS:-3 p} x ${TS_IMPLS:-3 p}; do
  LABSORT_TS_IMPL=$impl ALGO=merge timeout -k 10 200 python "$R/harness/exp/hist_time.py" >> "$O/ts_ab_classes.jsonl" 2>"$O/ts_ab_$impl.err" || { tail -5 "$O/ts_ab_$impl.err"; exit 1; }
  tail -1 "$O/ts_ab_classes.jsonl"
  LABSORT_TS_IMPL=$impl timeout -k 10 200 python "$R/bench.py" --algo merge --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > "$O/ts_ab_$impl.json" 2>"$O/ts_ab_$impl.err" || { tail -5 "$O/ts_ab_$impl.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ts_ab_$impl.json')); print('$impl', d['ms_per_step'], d['roofline'].get('avg_launch_ms'))"
done
