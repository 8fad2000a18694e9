#!/bin/bash
# Round 3: fp16 batch-invariance bisection, large tiles for dense GEMMs only / convs only
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3s; mkdir -p $O
for o in "--opt large_mask=1" "--opt large_mask=2" "--opt large_mask=2 --opt gn_parts=0"; do
  timeout -k 10 200 python -u scripts/diag_bi2.py --dtype fp16 --res 256 $o > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0" $O/d.txt | cut -c1-200 | tee -a $O/bisect.txt
done
