#!/bin/bash
# r5: merge A/B (pairwise only / four-way / four-way + 16K tiles) and per-kernel times of the four-way pass
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
bash "$R/harness/exp/r5_merge_ab.sh" || exit 1
export ALGO=merge
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/m4prof_b" -o run -- python3 "$R/harness/exp/hist_time.py" > "$O/m4prof_b.log" 2>&1 || { tail -20 "$O/m4prof_b.log"; exit 1; }
cut -d, -f1-4 "$O"/m4prof_b/run_kernel_stats.csv
