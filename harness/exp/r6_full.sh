#!/bin/bash
# r6: the whole GPU test suite, then bench.py --gpus 8 --backend gloo started plainly (its own
# 8 ranks on this one GPU: the launcher and the 8-rank config-5 line rehearsed), then the
# default bench line.  Each step has its own time limit; the first failure ends the script.
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
TAG=${TAG:-r31}
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/${TAG}_pytest_gpu.log" 2>&1
  tail -2 "$O/${TAG}_pytest_gpu.log"
fi
timeout -k 10 600 python3 -u bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --no-host-path > "$O/${TAG}_bench_gloo8.json" 2> "$O/${TAG}_bench_gloo8.err"
tail -c 600 "$O/${TAG}_bench_gloo8.json"; echo
timeout -k 10 600 python3 -u bench.py > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err"
tail -c 1500 "$O/${TAG}_bench.json"; echo
