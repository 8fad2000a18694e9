#!/bin/bash
# Round 3: fp16 batch-invariance bisection within the dense large-tile GEMMs
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3t; mkdir -p $O
for o in "--opt ln_fold=0 --opt gemm_sk=0 --opt gn_parts=0 --opt splitk_inkernel=0 --opt tile_256x320=0 --opt attn_hm=0" \
         "--opt gemm_deep=1" "--opt gemm_small=1" "--opt ln_fold=0 --opt gemm_sk=0"; do
  timeout -k 10 200 python -u scripts/diag_bi2.py --dtype fp16 --res 256 $o > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0" $O/d.txt | cut -c1-250 | tee -a $O/bisect.txt
done
