#!/bin/bash
# r6: SQ counters of the four-way merge kernel for each build in VARS ("product" = the in-tree
# library, others harness/bin/ab/liblabsort_<v>.so), two rocprofv3 --pmc passes each over one
# 2^28 merge sort (bench.py --algo merge --steps 1 --warmup 1); summaries in gpurun_out/pmc_<TAG>_<v>.txt
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
TAG=${TAG:-m4}
for v in ${VARS:-product}; do
  lib=""; [ "$v" != product ] && lib="$R/harness/bin/ab/liblabsort_$v.so"
  SQ_ONLY=1 LABSORT_LIBRARY="$lib" BENCH_ARGS="--algo merge ${EXTRA_ARGS:-}" bash "$R/harness/exp/pmc_kernel.sh" "${KRE:-k_m4_merge}" "${TAG}_$v" > /dev/null
  echo "== $v"; cat "$R/gpurun_out/pmc_${TAG}_$v.txt"
done
