#!/bin/bash
# r4 A/B of the merge pass's prefetch depth (LABSORT_MG_PF=2: the next two tiles' keys in
# flight instead of one): merge tests with it, then alternating timings of both.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
LABSORT_MG_PF=2 timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_sort.py" "$R/tests/test_gpu_fullsize.py" -m gpu -x -q \
    -k "merge or sort_device_uniform or sort_device_distributions" --timeout 150 --timeout-method thread -p no:cacheprovider > "$O/mg_ab_pytest.log" 2>&1
rc=$?; echo "pytest MG_PF=2 rc=$rc"; tail -3 "$O/mg_ab_pytest.log"
[ $rc -eq 0 ] || exit $rc
for pf in 1 2 1 2; do
  LABSORT_MG_PF=$pf LABSORT_TS_IMPL=${TS:-x} ALGO=merge timeout -k 10 200 python "$R/harness/exp/hist_time.py" > "$O/mg_ab_$pf.json" 2>"$O/mg_ab_$pf.err" || { tail -5 "$O/mg_ab_$pf.err"; exit 1; }
  echo "MG_PF=$pf $(cat "$O/mg_ab_$pf.json")"
done
