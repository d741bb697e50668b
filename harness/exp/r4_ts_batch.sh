#!/bin/bash
# r4: k_tile_sort's counter reads batched ahead of its reorder stores (and the key/value
# merge pass's payload reads): merge / tile-sort / pairs tests with the product build,
# then alternating timings against harness/exp/libs/liblabsort_base.so (before).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
P="radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so"
timeout -k 10 500 python -u -m pytest "$R/tests/test_gpu_sort.py" "$R/tests/test_gpu_fullsize.py" -m gpu -x -q \
    -k "tile or merge or sort_device or pairs" --timeout 150 --timeout-method thread -p no:cacheprovider > "$O/tsb_pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/tsb_pytest.log"; [ $rc -eq 0 ] || exit $rc
bash "$R/harness/exp/ab_libs.sh" merge harness/exp/libs/liblabsort_base.so "$P" 3 || exit 1
for L in harness/exp/libs/liblabsort_base.so "$P" harness/exp/libs/liblabsort_base.so "$P"; do
  LABSORT_LIBRARY="$R/$L" timeout -k 10 200 python "$R/bench.py" --algo pairs --pair-algo merge --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > "$O/tsb_pairs.json" 2>"$O/tsb_pairs.err" || { tail -5 "$O/tsb_pairs.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/tsb_pairs.json')); print('$L'.split('/')[-1], 'pairs merge ms', d['ms_per_step'])"
done
