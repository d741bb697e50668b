#!/bin/bash
# lib_ab.sh -- A/B of diagnostic library builds on the headline bench: for each
# library in $LIBS (default: the shipped one first), ms per sort and the dominant
# kernel's average launch time, for the key distributions in $DISTS.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
P=radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so
for lib in $P $LIBS; do
  for dist in ${DISTS:-u32}; do
    LABSORT_LIBRARY="$R/$lib" timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --no-host-path --dist $dist ${BENCH_ARGS} > "$O/ab.json" 2> "$O/ab.err" || { echo "FAIL $lib $dist"; tail -5 "$O/ab.err"; exit 1; }
    echo "$(basename $lib) $dist $(grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*\|"ms_per_sort": [0-9.]*' "$O/ab.json" | tr '\n' ' ')"
  done
done
