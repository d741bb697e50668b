#!/bin/bash
# r4 (r28) committed profiles: kernel-trace stats and HBM PMC passes of the radix and merge
# benches (profile_round.sh), then the SQ / LDS counter passes of k_tile_sort (merge bench)
# and k_onesweep_p (radix bench).  Each step has its own time limit; the first failure ends it.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
bash "$R/harness/exp/profile_round.sh" r28 || exit $?
BENCH_ARGS="--algo merge --no-merge" bash "$R/harness/exp/pmc_kernel.sh" k_tile_sort tile_sort_sq || exit $?
BENCH_ARGS="--no-merge" bash "$R/harness/exp/pmc_kernel.sh" k_onesweep_p onesweep_sq || exit $?
BENCH_ARGS="--algo merge --no-merge" bash "$R/harness/exp/pmc_kernel.sh" k_merge_pass_p merge_sq
