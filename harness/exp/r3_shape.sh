#!/bin/bash
# r3_shape.sh -- the 768 x 20 onesweep shape (shipped) against 1024 x 16 (o1024k16):
# radix keys (u32, sorted), key/value pairs; then the whole GPU suite on the shipped build
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
L=radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so
LIBS="harness/exp/libs/liblabsort_o1024k16.so $L" DISTS="u32 sorted" bash harness/exp/lib_ab.sh || exit 1
for lib in harness/exp/libs/liblabsort_o1024k16.so $L harness/exp/libs/liblabsort_o1024k16.so $L; do
  LABSORT_LIBRARY="$R/$lib" timeout -k 10 200 python bench.py --algo pairs --no-cpu-baseline --no-host-path > "$O/kv.json" 2> "$O/kv.err" || { echo "FAIL $lib"; tail -5 "$O/kv.err"; exit 1; }
  echo "$(basename $lib) pairs $(grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*' "$O/kv.json" | tr '\n' ' ')"
done
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > "$O/pytest_gpu_shape.log" 2>&1; rc=$?
tail -3 "$O/pytest_gpu_shape.log"; exit $rc
