#!/bin/bash
# r3_fused.sh -- fused small gathered path: parity tests (memset-free default and the
# memset variant), then 2^16..2^20 timing of LABSORT_GS_FUSED=2/1/0, then kernel traces
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
for f in 2 1; do
  LABSORT_GS_FUSED=$f timeout -k 10 300 python -u -m pytest "$R/tests/test_gpu_gsweep.py" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/fused_pytest_$f.log" 2>&1 || { tail -40 "$O/fused_pytest_$f.log"; exit 1; }
  echo "fused=$f: $(tail -1 "$O/fused_pytest_$f.log")"
done
for f in 2 1 0; do
  echo "== LABSORT_GS_FUSED=$f"
  LABSORT_GS_FUSED=$f NS="65536 262144 1048576" IMPLS="radix:gather" timeout -k 10 120 python3 "$R/harness/exp/small_n.py" || exit 1
done
LABSORT_GS_FUSED=2 NS=1048576 IMPLS=radix:gather bash "$R/harness/exp/ktrace.sh" f20 6 "$R/harness/exp/small_n.py" || exit 1
