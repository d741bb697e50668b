#!/bin/bash
# bench.py (radix, 2^28) once per diagnostic library given on the command line.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
for lib in "$@"; do
  echo "== $lib"
  LABSORT_LIBRARY="$R/$lib" timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --no-host-path ${BENCH_ARGS:-} > "$R/gpurun_out/rl.json" 2> "$R/gpurun_out/rl.err" || { tail -5 "$R/gpurun_out/rl.err"; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*' "$R/gpurun_out/rl.json" | tr '\n' ' '; echo
done
