#!/bin/bash
# Round 3: fp16 batch-invariance vs the split point (partial-tile hypothesis), GEGLU K >= 1280 on large tiles only
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3ab; mkdir -p $O
for c in 4 2 1 7; do
  timeout -k 10 200 python -u scripts/diag_bi2.py --dtype fp16 --res 256 --split $c --opt large_dense=32 > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0" $O/d.txt | cut -c1-250 | tee -a $O/bisect.txt
done
