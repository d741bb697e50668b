#!/bin/bash
# r3_run2.sh -- the GPU tests touched in round 3 (multi-GPU, dist, key/value), the gloo
# 2-rank bench rehearsal, the PMC calibration probe, and a full default bench run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
echo "== tests"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_sort.py -k "dist or pairs" > "$O/t_r2.log" 2>&1 || { echo "TESTS FAILED"; tail -30 "$O/t_r2.log"; exit 1; }
tail -2 "$O/t_r2.log"
echo "== gloo bench"
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --log2n 24 --no-host-path > "$O/b_gloo2.json" 2> "$O/b_gloo2.err" || { echo "GLOO BENCH FAILED"; tail -20 "$O/b_gloo2.err"; exit 1; }
head -c 800 "$O/b_gloo2.json"; echo
echo "== pmc calibration timing"
timeout -k 10 60 harness/bin/pmc_cal || exit 1
echo "== bench"
timeout -k 10 400 python bench.py > "$O/bench_r3a.json" 2> "$O/bench_r3a.err" || { echo "BENCH FAILED"; tail -20 "$O/bench_r3a.err"; exit 1; }
head -c 3000 "$O/bench_r3a.json"
