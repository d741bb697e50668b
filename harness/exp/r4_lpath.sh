#!/bin/bash
# r4: the local-pass radix on the GPU: its radix tests, a radix-only bench, a kernel trace.
# Each GPU step has its own time limit; a crash or time-out ends the script.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"
TAG="${1:-r4l}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "$R/tests/test_gpu_sort.py" "$R/tests/test_gpu_gsweep.py" "$R/tests/test_gpu_fullsize.py" \
    -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > "$O/${TAG}_pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 "$O/${TAG}_pytest.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python "$R/bench.py" --no-cpu-baseline --no-host-path --no-merge ${BENCH_ARGS:-} > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err"
rc=$?
echo "bench rc=$rc"; cut -c1-1200 "$O/${TAG}_bench.json"; tail -5 "$O/${TAG}_bench.err"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${TAG}_prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-host-path --no-merge > "$O/${TAG}_prof.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
f=$(find "$O/${TAG}_prof" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
exit $rc
