#!/bin/bash
# r3_kv.sh -- key/value persistent onesweep A/B: key prefetch (PF) and payloads scattered
# from LDS (LDSV): kv11 = shipped, kv10, kv01, kv00 (= the first r26 version)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
L=radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so
for lib in $L harness/exp/libs/liblabsort_kv10.so harness/exp/libs/liblabsort_kv01.so harness/exp/libs/liblabsort_kv00.so $L; do
  LABSORT_LIBRARY="$R/$lib" timeout -k 10 200 python bench.py --algo pairs --no-cpu-baseline --no-host-path > "$O/kv.json" 2> "$O/kv.err" || { echo "FAIL $lib"; tail -5 "$O/kv.err"; exit 1; }
  echo "$(basename $lib) $(grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*' "$O/kv.json" | tr '\n' ' ')"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort.py -k pairs -m gpu 2>&1 | tail -2
