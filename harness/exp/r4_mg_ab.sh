#!/bin/bash
# r4 A/B of a merge-pass variant (harness/exp/libs/liblabsort_$1.so) vs the product
# (liblabsort_base.so): merge / pairs tests with the variant, then alternating timings.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
V="harness/exp/libs/liblabsort_$1.so"
LABSORT_LIBRARY="$R/$V" timeout -k 10 500 python -u -m pytest "$R/tests/test_gpu_sort.py" "$R/tests/test_gpu_fullsize.py" "$R/tests/test_gpu_multi.py" -m gpu -x -q \
    -k "merge or sort_device or pairs or tile" --timeout 150 --timeout-method thread -p no:cacheprovider > "$O/mg_pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/mg_pytest.log"; [ $rc -eq 0 ] || exit $rc
bash "$R/harness/exp/ab_libs.sh" merge harness/exp/libs/liblabsort_base.so "$V" 4
