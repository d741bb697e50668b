#!/bin/bash
# r3_run1.sh -- round-3 GPU batch: onesweep A/B (HEAD kernels vs the flat-load fix vs
# buffer-descriptor loads/stores), key/value persistent vs non-persistent passes, then
# the multi-GPU / key/value GPU tests and the gloo 2-rank bench rehearsal.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
L=radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so
echo "== radix A/B"
for lib in harness/exp/libs/liblabsort_base.so harness/exp/libs/liblabsort_flatfix.so $L harness/exp/libs/liblabsort_base.so $L; do
  LABSORT_LIBRARY="$R/$lib" timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-path --no-merge > "$O/ab.json" 2> "$O/ab.err" || { echo "FAIL $lib"; tail -5 "$O/ab.err"; exit 1; }
  echo "$(basename $lib) $(grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*' "$O/ab.json" | tr '\n' ' ')"
done
echo "== pairs"
for osp in 1 0; do
  LABSORT_PAIRS_OSP=$osp timeout -k 10 200 python bench.py --algo pairs --no-cpu-baseline --no-host-path > "$O/pairs_$osp.json" 2> "$O/pairs_$osp.err" || { echo "FAIL pairs $osp"; tail -5 "$O/pairs_$osp.err"; exit 1; }
  echo "pairs osp=$osp $(grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*' "$O/pairs_$osp.json" | tr '\n' ' ')"
done
echo "== tests"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_dist.py "tests/test_gpu_sort.py" -k "multi or dist or pairs or ranks" > "$O/t_multi.log" 2>&1 || { echo "TESTS FAILED"; tail -30 "$O/t_multi.log"; exit 1; }
tail -3 "$O/t_multi.log"
echo "== gloo bench"
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --log2n 24 --no-host-path > "$O/b_gloo2.json" 2> "$O/b_gloo2.err" || { echo "GLOO BENCH FAILED"; tail -20 "$O/b_gloo2.err"; exit 1; }
head -c 600 "$O/b_gloo2.json"
