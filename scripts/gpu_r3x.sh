#!/bin/bash
# Round 3: fp16 batch-invariance bisection by dense GEMM class on large tiles (1 N<=1280, 2 head-split, 4 GEGLU, 8 other)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3x; mkdir -p $O
for m in 1 2 4 8 14 13 11 7; do
  timeout -k 10 200 python -u scripts/diag_bi2.py --dtype fp16 --res 256 --opt large_dense=$m > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0" $O/d.txt | cut -c1-250 | tee -a $O/bisect.txt
done
