#!/bin/bash
# r3_run3.sh -- onesweep tile-size A/B (16K tiles with / without prefetch, 20K and 24K
# tiles), then the round's profiles (2^28 only) and the SQ/LDS counters of the onesweep
# pass and the tile sort.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
L=radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so
echo "== tile A/B"
for lib in $L harness/exp/libs/liblabsort_kpt16np.so harness/exp/libs/liblabsort_kpt20np.so harness/exp/libs/liblabsort_kpt24np.so harness/exp/libs/liblabsort_kpt24pf.so $L; do
  LABSORT_LIBRARY="$R/$lib" timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-path --no-merge > "$O/ab.json" 2> "$O/ab.err" || { echo "FAIL $lib"; tail -5 "$O/ab.err"; exit 1; }
  echo "$(basename $lib) $(grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*' "$O/ab.json" | tr '\n' ' ')"
done
echo "== profiles"
timeout -k 10 700 bash harness/exp/profile_round.sh r26 || exit 1
echo "== SQ/LDS counters"
BENCH_ARGS="--no-merge" timeout -k 10 300 bash harness/exp/pmc_kernel.sh k_onesweep_p onesweep_r26 > /dev/null 2>&1 || echo "pmc onesweep failed"
BENCH_ARGS="--algo merge --no-merge" timeout -k 10 300 bash harness/exp/pmc_kernel.sh k_tile_sort tile_sort_r26 > /dev/null 2>&1 || echo "pmc tile sort failed"
cat "$O/pmc_onesweep_r26.txt" "$O/pmc_tile_sort_r26.txt" 2>/dev/null
