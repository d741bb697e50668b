#!/bin/bash
# one GPU call for the r4 experiments: the local-pass radix, then the tile-sort A/B
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
bash "$R/harness/exp/r4_lpath.sh" r4l || exit $?
bash "$R/harness/exp/r4_ts_ab.sh"
