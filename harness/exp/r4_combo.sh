#!/bin/bash
# one GPU call for the r4 A/Bs: the tile sort (LABSORT_TS_IMPL) and the merge pass's
# prefetch depth (LABSORT_MG_PF); each script stops at its first failing GPU step
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
TS_IMPLS="${TS_IMPLS:-3 q}" bash "$R/harness/exp/r4_ts_ab.sh" || exit $?
bash "$R/harness/exp/r4_mg_ab.sh"
