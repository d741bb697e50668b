#!/bin/bash
# r3_tail.sh -- A/B of the radix launch sequence at 2^28: shipped (look-back clear folded
# into the plan launch), LABSORT_PLAN_ZERO=0 (separate k_zero), and the tail-writeback
# variant library; then the radix parity tests on the shipped build
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-host-path --no-merge --steps 40 --warmup 5"
one() { timeout -k 10 200 env "$@" python3 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('config2',{}).get('ms_per_sort'))"; }
for i in 1 2 3; do
  one X=shipped || exit 1
  one LABSORT_PLAN_ZERO=0 || exit 1
  one LABSORT_LIBRARY=$R/harness/exp/libs/liblabsort_tailwb.so || exit 1
done
timeout -k 10 600 python -u -m pytest "$R/tests/test_gpu_fullsize.py" "$R/tests/test_gpu_sort.py" "$R/tests/test_gpu_graph.py" -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > "$O/tail_pytest.log" 2>&1 || { tail -30 "$O/tail_pytest.log"; exit 1; }
tail -1 "$O/tail_pytest.log"
