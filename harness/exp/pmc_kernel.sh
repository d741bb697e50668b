#!/bin/bash
# pmc_kernel.sh KRE TAG -- SQ/LDS counter passes (one rocprofv3 --pmc run each) on the
# kernels matching KRE during `bench.py $BENCH_ARGS --steps 1 --warmup 1`; per-counter
# averages printed and kept in gpurun_out/pmc_TAG.txt
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
KRE="$1"; TAG="$2"
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
      "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
      "FETCH_SIZE" "WRITE_SIZE")
[ -n "${SQ_ONLY:-}" ] && SETS=("${SETS[@]:0:2}")  # the two SQ passes only
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "$KRE" --output-format csv -d "$O/pmc_${TAG}_$i" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-host-path ${BENCH_ARGS:-} > "$O/pmc_${TAG}_$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$O/pmc_${TAG}_$i.log"; exit 1; }
done
python3 - "$O" "$TAG" <<'PY' | tee "$O/pmc_$2.txt"
import csv, sys, glob, collections
O, tag = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(f"{O}/pmc_{tag}_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:40s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
