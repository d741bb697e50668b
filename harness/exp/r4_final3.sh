#!/bin/bash
# r4 (r28) late validation of the shipped build (GPU suite, smoke, bench, committed
# profiles), then the merge-pass co-rank bracket A/B.  First failure ends it.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
bash "$R/harness/exp/r4_final2.sh" || exit $?
bash "$R/harness/exp/r4_br.sh" > "$R/gpurun_out/r4_br.txt" 2>&1
