#!/bin/bash
# Round 3: kernel-level PMC passes for gemm_sk (stall breakdown, instruction mix, LDS) on lin320 / lin320r / geglu320
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3p; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_DATA_FIFO_FULL"
P3="TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum FETCH_SIZE"
RX="gemm_sk"
for op in lin320 lin320r geglu320; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv -d $O/${op}_p$i -o p -- python3 scripts/kprof.py --op $op --iters 5 > $O/${op}_p$i.log 2>&1 || { echo "pass $i of $op failed"; tail -5 $O/${op}_p$i.log; exit 1; }
  done
  python3 scripts/pmc_dump.py "$RX" $O/${op}_p1 $O/${op}_p2 $O/${op}_p3 > $O/${op}_pmc.txt
  echo "== $op"; cat $O/${op}_pmc.txt
  rm -rf $O/${op}_p1 $O/${op}_p2 $O/${op}_p3
done
