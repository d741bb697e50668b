#!/bin/bash
# harness/gpu_check.sh -- one gpurun call: GPU parity tests, smoke, bench, rocprofv3
# kernel-trace summary and separate PMC passes (FETCH_SIZE / WRITE_SIZE) of the bench.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
TAG="${1:-r01}"
STEPS="${STEPS:-all}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() { echo "== $(date +%T) $*" | tee -a "$O/steps.log"; }
ok=0
if [[ "$STEPS" == all || "$STEPS" == *tests* ]]; then
  run pytest
  timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest "$R/tests" -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > "$O/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
  tail -3 "$O/pytest_gpu.log"
  run smoke
  timeout -k 10 300 python -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 1; }
  cat "$O/smoke.log"
fi
if [[ "$STEPS" == all || "$STEPS" == *bench* ]]; then
  run bench
  timeout -k 10 400 python "$R/bench.py" > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" || { cat "$O/bench_$TAG.err"; exit 1; }
  cat "$O/bench_$TAG.json"
fi
if [[ "$STEPS" == all || "$STEPS" == *prof* ]]; then
  run rocprof stats
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > "$O/prof_$TAG.log" 2>&1 || { tail -30 "$O/prof_$TAG.log"; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    run rocprof pmc $c
    timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_${c}_$TAG" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > "$O/pmc_${c}_$TAG.log" 2>&1 || { tail -30 "$O/pmc_${c}_$TAG.log"; exit 1; }
  done
fi
run done
if [[ "$STEPS" == *dist* ]]; then
  for ex in splitters pairwise; do
    run "bench gloo 2 ranks on one GPU ($ex)"
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 "$R/bench.py" --gpus 2 --steps 3 --warmup 1 --backend gloo --log2n 22 --exchange $ex > "$O/bench_dist2_$ex.log" 2>&1 || { tail -30 "$O/bench_dist2_$ex.log"; exit 1; }
    grep '"metric"' "$O/bench_dist2_$ex.log" | cut -c1-400
  done
fi
if [[ "$STEPS" == *mprof* ]]; then
  run rocprof stats merge
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/mprof_$TAG" -o run -- python3 "$R/bench.py" --algo merge --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > "$O/mprof_$TAG.log" 2>&1 || { tail -30 "$O/mprof_$TAG.log"; exit 1; }
fi
