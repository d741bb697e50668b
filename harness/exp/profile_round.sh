#!/bin/bash
# profile_round.sh TAG -- the round's committed profiles, each at 2^28 keys only (the
# small config legs of the default bench would pollute per-kernel averages):
#   prof_TAG / prof_TAG_merge      rocprofv3 --kernel-trace --stats: radix bench, merge bench
#   pmc_{FETCH,WRITE}_SIZE_TAG[_merge]   one --pmc pass each (HBM bytes per launch)
#   cal_{FETCH,WRITE}_SIZE_TAG     the same counters on harness/bin/pmc_cal (known bytes
#                                  per access shape) for profiles/pmc_summary.py
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
TAG="$1"
B="$R/bench.py --no-cpu-baseline --no-host-path --no-merge"
for leg in "" "_merge"; do
  A=""; [ "$leg" = "_merge" ] && A="--algo merge"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG$leg" -o run -- python3 $B $A --steps 10 --warmup 2 > "$O/prof_$TAG$leg.log" 2>&1 || { echo "stats pass $leg failed"; tail -20 "$O/prof_$TAG$leg.log"; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_${c}_$TAG$leg" -o run -- python3 $B $A --steps 2 --warmup 1 > "$O/pmc_${c}_$TAG$leg.log" 2>&1 || { echo "pmc $c $leg failed"; tail -20 "$O/pmc_${c}_$TAG$leg.log"; exit 1; }
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$O/cal_${c}_$TAG" -o run -- "$R/harness/bin/pmc_cal" > "$O/cal_${c}_$TAG.log" 2>&1 || { echo "cal $c failed"; tail -20 "$O/cal_${c}_$TAG.log"; exit 1; }
done
echo "profiles done: $TAG"
