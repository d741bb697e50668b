#!/bin/bash
# r3_cal.sh TAG -- the pmc_cal calibration passes of profile_round.sh alone
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$O/cal_${c}_$1" -o run -- "$R/harness/bin/pmc_cal" > "$O/cal_${c}_$1.log" 2>&1 || { echo "cal $c failed"; tail -20 "$O/cal_${c}_$1.log"; exit 1; }
done
echo "cal done"
