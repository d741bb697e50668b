#!/bin/bash
# r6: validation and the round's committed measurements on one box: the whole GPU test suite,
# smoke(), the rocprofv3 kernel-stats + HBM counter passes (profile_round.sh TAG), the default bench line.
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
TAG=${TAG:-r31}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/${TAG}_pytest_gpu.log" 2>&1
tail -2 "$O/${TAG}_pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/${TAG}_smoke.log" 2>&1
tail -1 "$O/${TAG}_smoke.log"
timeout -k 10 600 python3 -u bench.py > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err"
tail -c 400 "$O/${TAG}_bench.json"; echo
timeout -k 10 900 bash "$R/harness/exp/profile_round.sh" "$TAG"
