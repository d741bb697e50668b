#!/bin/bash
# r5: per-kernel times of the four-way merge pass (k_m4_rank vs k_m4_merge) and SQ counters.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
export ALGO=merge
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/m4prof" -o run -- python3 "$R/harness/exp/hist_time.py" > "$O/m4prof.log" 2>&1 || { tail -20 "$O/m4prof.log"; exit 1; }
cat "$O"/m4prof/*kernel_stats.csv 2>/dev/null || find "$O/m4prof" -name "*stats*"
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
      "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
      "FETCH_SIZE" "WRITE_SIZE")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "k_m4_" --output-format csv -d "$O/pmc_m4_$i" -o run -- python3 "$R/harness/exp/hist_time.py" > "$O/pmc_m4_$i.log" 2>&1 || { echo "pmc $i failed"; tail -5 "$O/pmc_m4_$i.log"; exit 1; }
done
echo pmc done
