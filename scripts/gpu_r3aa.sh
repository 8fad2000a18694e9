#!/bin/bash
# Round 3: fp16 batch-invariance: in-kernel split-K reductions (dense and halo) both off
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3aa; mkdir -p $O
for o in "--opt splitk_inkernel=0 --opt halo_split=0" "--opt large_dense=32 --opt splitk_inkernel=0 --opt halo_split=0" "--opt large_dense=32 --opt gn_parts=0 --opt ln_fold=0"; do
  timeout -k 10 200 python -u scripts/diag_bi2.py --dtype fp16 --res 256 $o > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0" $O/d.txt | cut -c1-250 | tee -a $O/bisect.txt
done
