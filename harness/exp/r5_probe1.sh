#!/bin/bash
# r5: key/value pass A/B (r27 build vs HEAD build) and the digit-width probe, one call.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 python -u "$R/harness/exp/pairs_ab.py" harness/bin/ab/liblabsort_r27.so harness/bin/ab/liblabsort_head.so 4 > "$O/pairs_ab.log" 2>&1 || { cat "$O/pairs_ab.log"; exit 1; }
cat "$O/pairs_ab.log"
timeout -k 10 200 "$R/harness/bin/digit_probe" > "$O/digit_probe.log" 2>&1 || { cat "$O/digit_probe.log"; exit 1; }
cat "$O/digit_probe.log"
