#!/bin/bash
# Round 3: fp16 batch-invariance bisection: which GEGLU level (large tiles for GEGLU at K 320 / 640 / >= 1280 only)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3z; mkdir -p $O
for m in 4 16 32 59 47 31; do
  timeout -k 10 200 python -u scripts/diag_bi2.py --dtype fp16 --res 256 --opt large_dense=$m > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0" $O/d.txt | cut -c1-250 | tee -a $O/bisect.txt
done
