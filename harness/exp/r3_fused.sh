#!/bin/bash
# r3_fused.sh -- fused small gathered path: parity tests, then 2^16..2^20 timing with and
# without the fusion (LABSORT_GS_FUSED=0), then a kernel trace of one fused 2^20 sort
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "$R/tests/test_gpu_gsweep.py" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/fused_pytest.log" 2>&1 || { tail -40 "$O/fused_pytest.log"; exit 1; }
tail -2 "$O/fused_pytest.log"
for f in 1 0; do
  echo "== LABSORT_GS_FUSED=$f"
  LABSORT_GS_FUSED=$f NS="65536 262144 1048576" IMPLS="radix:gather" timeout -k 10 120 python3 "$R/harness/exp/small_n.py" || exit 1
done
NS=1048576 IMPLS=radix:gather bash "$R/harness/exp/ktrace.sh" f20 12 "$R/harness/exp/small_n.py" || exit 1
LABSORT_GS_FUSED=0 NS=1048576 IMPLS=radix:gather bash "$R/harness/exp/ktrace.sh" u20 12 "$R/harness/exp/small_n.py"
