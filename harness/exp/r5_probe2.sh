#!/bin/bash
# r5: key/value readback order A/B (r27 / HEAD / HEAD with keys-then-payloads readback) and
# the digit-width probe with its contiguous-write control, then SQ + HBM counters of the
# probe's pass kernel at 8 and 11 bits (one rocprofv3 --pmc run per counter set).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 python -u "$R/harness/exp/pairs_ab.py" harness/bin/ab/liblabsort_r27.so harness/bin/ab/liblabsort_head.so harness/bin/ab/liblabsort_head2.so 3 > "$O/pairs_ab2.log" 2>&1 || { cat "$O/pairs_ab2.log"; exit 1; }
cat "$O/pairs_ab2.log"
timeout -k 10 200 "$R/harness/bin/digit_probe" > "$O/digit_probe2.log" 2>&1 || { cat "$O/digit_probe2.log"; exit 1; }
cat "$O/digit_probe2.log"
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
      "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
      "FETCH_SIZE" "WRITE_SIZE")
for b in 8 11; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $set --kernel-include-regex "k_pass" --output-format csv -d "$O/pmc_dp${b}_$i" -o run -- "$R/harness/bin/digit_probe" $b s > "$O/pmc_dp${b}_$i.log" 2>&1 || { echo "pmc $b $i failed"; tail -5 "$O/pmc_dp${b}_$i.log"; exit 1; }
  done
done
echo pmc done
