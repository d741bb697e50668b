#!/bin/bash
# r5: merge sort A/B at 2^28: pairwise passes only (m2) / four-way passes (HEAD) / four-way +
# 16K-key tile sort at 2 workgroups per CU (ts512); output equality checked per row.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
MODE=merge timeout -k 10 240 python -u "$R/harness/exp/pairs_ab.py" harness/bin/ab/liblabsort_m2np.so harness/bin/ab/liblabsort_m2.so radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so harness/bin/ab/liblabsort_ts512.so 3 > "$O/merge_ab.log" 2>&1 || { cat "$O/merge_ab.log"; exit 1; }
cat "$O/merge_ab.log"
