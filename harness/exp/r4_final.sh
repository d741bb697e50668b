#!/bin/bash
# r4 (r28) final call: the GPU suite, smoke and bench of the product (gpu_check.sh), the
# committed profiles (kernel stats, HBM PMC, SQ/LDS counters), then the rank-loop A/B of
# the variant libraries.  Each step has its own time limit; the first failure ends it.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
STEPS="tests bench" bash "$R/harness/gpu_check.sh" r28 || exit $?
bash "$R/harness/exp/r4_profiles.sh" || exit $?
bash "$R/harness/exp/r4_rank_ab.sh"
