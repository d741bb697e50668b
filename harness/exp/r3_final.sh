#!/bin/bash
# r3_final.sh -- fused-path parity tests, the default bench (copy ceiling), the round's
# profiles (profile_round.sh r27)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_gsweep.py" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/gsweep_pytest.log" 2>&1 || { tail -40 "$O/gsweep_pytest.log"; exit 1; }
tail -1 "$O/gsweep_pytest.log"
timeout -k 10 400 python "$R/bench.py" > "$O/bench_r27b.json" 2> "$O/bench_r27b.err" || { tail -20 "$O/bench_r27b.err"; exit 1; }
cut -c1-900 "$O/bench_r27b.json"
bash "$R/harness/exp/profile_round.sh" r27
