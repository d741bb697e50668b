#!/bin/bash
# r4 (r28) N>1 evidence for the final build on one GPU: bench --gpus 2 over gloo (both
# exchanges, 2^22 per rank), then the config-5 form at 2^28 total (strong scaling).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
STEPS="dist" bash "$R/harness/gpu_check.sh" r28dist || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --total-log2n 28 --no-weak > gpurun_out/bench_dist2_config5.log 2>&1 || { tail -30 gpurun_out/bench_dist2_config5.log; exit 1; }
grep '"metric"' gpurun_out/bench_dist2_config5.log | cut -c1-600
