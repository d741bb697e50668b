#!/bin/bash
# r3_seg.sh -- gsweep/onesweep parity tests, then the chain layout of the later passes at
# 2^28: digit-group segments (default) vs one chain (LABSORT_SEG=first)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_gsweep.py" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/gsweep_pytest3.log" 2>&1 || { tail -40 "$O/gsweep_pytest3.log"; exit 1; }
tail -1 "$O/gsweep_pytest3.log"
B="$R/bench.py --no-cpu-baseline --no-host-path --no-merge --steps 40 --warmup 5"
one() { timeout -k 10 200 env "$@" python3 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], d['roofline']['avg_launch_ms'])"; }
for i in 1 2; do
  one LABSORT_SEG=on || exit 1
  one LABSORT_SEG=first || exit 1
done
