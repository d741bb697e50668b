#!/bin/bash
# r3_kv2.sh -- key/value pass shapes: 1024 x 16 (shipped) vs 512 x 32 with / without the
# next tile's keys prefetched (kv512pf / kv512), same 16384-pair tiles; KVLIBS / KVTEST
# override the libraries timed and tested
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
L=radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so
for lib in ${KVLIBS:-$L harness/exp/libs/liblabsort_kv512pf.so harness/exp/libs/liblabsort_kv512.so $L harness/exp/libs/liblabsort_kv512pf.so}; do
  LABSORT_LIBRARY="$R/$lib" timeout -k 10 200 python bench.py --algo pairs --no-cpu-baseline --no-host-path > "$O/kv.json" 2> "$O/kv.err" || { echo "FAIL $lib"; tail -5 "$O/kv.err"; exit 1; }
  echo "$(basename $lib) $(grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*' "$O/kv.json" | tr '\n' ' ')"
done
for v in ${KVTEST:-kv512pf kv512}; do
  LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$v.so" timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort.py -k pairs -m gpu 2>&1 | tail -1
done
