#!/bin/bash
# r3_fused2.sh -- fused path: gsweep parity tests, 2^20 timing (fused 2 vs 0), kernel trace
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_gsweep.py" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/gsweep_pytest2.log" 2>&1 || { tail -40 "$O/gsweep_pytest2.log"; exit 1; }
tail -1 "$O/gsweep_pytest2.log"
for f in 2 0; do
  echo "== LABSORT_GS_FUSED=$f"
  LABSORT_GS_FUSED=$f NS="262144 1048576" IMPLS="radix:gather" timeout -k 10 120 python3 "$R/harness/exp/small_n.py" || exit 1
done
NS=1048576 IMPLS=radix:gather bash "$R/harness/exp/ktrace.sh" f20 5 "$R/harness/exp/small_n.py" || exit 1
