#!/bin/bash
# Round 3: fp16 batch-invariance bisection by forced dense tile (gemm_force = BM*100000 + BN*100 + splits)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3u; mkdir -p $O
for o in "--opt gemm_force=12832001" "--opt gemm_force=25632001" "--opt gemm_force=12812801" "--opt gemm_force=25625601" "--opt gemm_force=12825601"; do
  timeout -k 10 200 python -u scripts/diag_bi2.py --dtype fp16 --res 256 $o > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0" $O/d.txt | cut -c1-250 | tee -a $O/bisect.txt
done
