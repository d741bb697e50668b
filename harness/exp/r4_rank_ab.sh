#!/bin/bash
# r4 A/B of the branch-free rank loop: harness/exp/libs/liblabsort_tsrank.so (the tile
# sort) and liblabsort_osprank.so (also the onesweep pass) against liblabsort_base.so
# (the product).  Tests first; each GPU step has its own time limit.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
P="harness/exp/libs/liblabsort_tsrank.so"
LABSORT_LIBRARY="$R/$P" timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_sort.py" "$R/tests/test_gpu_fullsize.py" -m gpu -x -q \
    -k "tile_sort or merge or sort_device_uniform or sort_device_distributions" --timeout 150 --timeout-method thread -p no:cacheprovider > "$O/rank_pytest_ts.log" 2>&1
rc=$?; echo "pytest ts rc=$rc"; tail -2 "$O/rank_pytest_ts.log"; [ $rc -eq 0 ] || exit $rc
LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_osprank.so" timeout -k 10 500 python -u -m pytest "$R/tests/test_gpu_sort.py" "$R/tests/test_gpu_fullsize.py" -m gpu -x -q \
    -k "radix or sort_device or onesweep or pairs" --timeout 150 --timeout-method thread -p no:cacheprovider > "$O/rank_pytest_osp.log" 2>&1
rc=$?; echo "pytest osp rc=$rc"; tail -2 "$O/rank_pytest_osp.log"; [ $rc -eq 0 ] || exit $rc
bash "$R/harness/exp/ab_libs.sh" merge harness/exp/libs/liblabsort_base.so "$P" 3 || exit 1
bash "$R/harness/exp/ab_libs.sh" radix harness/exp/libs/liblabsort_base.so harness/exp/libs/liblabsort_osprank.so 3
