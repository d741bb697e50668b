#!/bin/bash
# r4: the multi-rank plan phase after the splitter selection / pinned staging / host-clock
# work split: the multi and dist GPU tests, then the bench (its config-5 host-path line
# carries plan_work / plan_wait).  Each step has its own limit; the first failure ends it.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_multi.py tests/test_gpu_dist.py > gpurun_out/plan_tests.log 2>&1 || { tail -30 gpurun_out/plan_tests.log; exit 1; }
tail -3 gpurun_out/plan_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/plan_bench.json 2> gpurun_out/plan_bench.err || { tail -30 gpurun_out/plan_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/plan_bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['value'])
print(json.dumps(d['host_path']['config5_8ranks_one_gpu']['phases_ms']))
"
