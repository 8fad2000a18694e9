#!/bin/bash
# Where does a large-tile GEMM/conv spend its time?  gemm_dbg: 1 skip epilogue, 2 skip MFMAs, 3 both;
# per pipeline mode (gemm_deep 0: 2-stage BK64, 1: BK32 ring, 2: BK64 3-stage ring where it fits).
set -o pipefail
O=gpurun_out/diag; mkdir -p $O; : > $O/res.txt
for dp in 0 1 2; do for d in 0 1 2 3; do
  timeout -k 10 60 python3 scripts/kshape.py conv 16 64 64 320 0 320 3 --opt gemm_deep=$dp --opt gemm_dbg=$d >> $O/res.txt 2>&1 || exit 1
  timeout -k 10 60 python3 scripts/kshape.py gemm 65536 320 320 --opt gemm_deep=$dp --opt gemm_dbg=$d >> $O/res.txt 2>&1 || exit 1
  timeout -k 10 60 python3 scripts/kshape.py gemm 65536 2560 320 --opt gemm_deep=$dp --opt gemm_dbg=$d >> $O/res.txt 2>&1 || exit 1
  timeout -k 10 60 python3 scripts/kshape.py conv 16 32 32 640 0 640 3 --opt gemm_deep=$dp --opt gemm_dbg=$d >> $O/res.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/res.txt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for pm in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $pm --output-format csv -d $O/pmc$n -o p -- python3 scripts/kshape.py conv 16 64 64 320 0 320 3 --iters 5 > $O/pmc$n.log 2>&1 || { tail -3 $O/pmc$n.log; exit 1; }
done
find $O -name "*counter_collection.csv" | head
