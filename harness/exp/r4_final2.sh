#!/bin/bash
# r4 (r28) final validation of the shipped build: GPU suite, smoke, bench (gpu_check.sh),
# then the committed profiles (kernel stats, HBM PMC, SQ/LDS counters).  Each step has its
# own time limit; the first failure ends it.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
STEPS="tests bench" bash "$R/harness/gpu_check.sh" r28 || exit $?
bash "$R/harness/exp/r4_profiles.sh"
