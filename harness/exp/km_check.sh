#!/bin/bash
# GPU check of the K-way merge: merge unit tests, merge bench, per-kernel rocprof stats.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 120 --timeout-method thread -k "merge" > gpurun_out/kt.log 2>&1
timeout -k 10 120 python bench.py --algo merge --no-cpu-baseline --no-host-path --steps 10 --warmup 2 > gpurun_out/km_bench.json 2> gpurun_out/km_bench.err
rm -rf gpurun_out/kmprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kmprof" -o run -- python3 "$R/bench.py" --algo merge --no-cpu-baseline --no-host-path --steps 5 --warmup 1 > "$R/gpurun_out/kmprof.log" 2>&1
