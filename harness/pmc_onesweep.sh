#!/bin/bash
# harness/pmc_onesweep.sh -- SQ/LDS/TA counter passes (one rocprofv3 --pmc run each)
# on the onesweep kernel of one 2^28 bench step; summaries in gpurun_out/pmc_os_*.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
i=0
SETS=("${PMC_SETS[@]}")
if [ ${#SETS[@]} -eq 0 ]; then
  SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
        "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE")
fi
[ -n "$PMC_SET1" ] && SETS=("$PMC_SET1")
rm -rf "$O"/pmc_os_*
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "${KRE:-onesweep_p}" --output-format csv -d "$O/pmc_os_$i" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-host-path ${BENCH_ARGS:-} > "$O/pmc_os_$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$O/pmc_os_$i.log"; exit 1; }
done
python3 - "$O" <<'PY'
import csv, sys, glob, collections
O = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(O + "/pmc_os_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:40s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
