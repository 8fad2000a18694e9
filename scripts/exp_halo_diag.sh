#!/bin/bash
# halo conv: where does the time go (gemm_dbg 1 no epilogue, 2 no MFMA, 3 both) + SQ PMC passes.
set -o pipefail
O=gpurun_out/halodiag; mkdir -p $O; : > $O/res.txt
for d in 0 1 2 3; do
  timeout -k 10 60 python3 scripts/kshape.py conv 16 64 64 320 0 320 3 --iters 20 --opt gemm_dbg=$d >> $O/res.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/res.txt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
n=0
for pm in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $pm --output-format csv -d $O/pmc$n -o p -- python3 scripts/kshape.py conv 16 64 64 320 0 320 3 --iters 5 > $O/pmc$n.log 2>&1 || { tail -3 $O/pmc$n.log; exit 1; }
done
echo done
