#!/bin/bash
# A/B experiment (first used for XCD-grouped acquisition): GPU sort tests ($TESTS), then bench + per-pass times for
# the library (XCD groups) and harness/exp/liblabsort_stamps_x0.so (one global counter),
# each with LABSORT_SEG=first (default) and on.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
P=radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -m pytest ${TESTS:-"$R/tests/test_gpu_sort.py"} -x -q -p no:cacheprovider > "$O/xt.log" 2>&1 || { tail -30 "$O/xt.log"; exit 1; }
  tail -2 "$O/xt.log"
fi
for lib in $P ${LIBS-harness/exp/liblabsort_stamps_x0.so}; do
  for seg in ${SEGS:-first on}; do
    echo "== $lib SEG=$seg"
    LABSORT_SEG=$seg LABSORT_LIBRARY="$R/$lib" timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --no-host-path > "$O/xe.json" 2> "$O/xe.err" || { tail -5 "$O/xe.err"; exit 1; }
    grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*' "$O/xe.json" | tr '\n' ' '; echo
    LABSORT_SEG=$seg LABSORT_LIBRARY="$R/$lib" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/xe_prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > "$O/xe_prof.log" 2>&1 || { tail -5 "$O/xe_prof.log"; exit 1; }
    python3 "$R/harness/exp/pass_times.py" "$O/xe_prof/run_kernel_trace.csv"
    rm -rf "$O/xe_prof"
  done
done
