#!/bin/bash
# Round 3: GEMM-op row-wise batch invariance at the 256x256 UNet shapes; 64x320 tile timing (forced)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3v; mkdir -p $O
timeout -k 10 200 python -u scripts/diag_gemm_rows.py > $O/gemm_rows.txt 2>&1; grep -v amdgpu.ids $O/gemm_rows.txt
for op in lin320 lin320r qkv320; do
  for f in 0 6432001; do
    timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 20 --opt gemm_force=$f > $O/kp.txt 2>&1 || { cat $O/kp.txt; exit 1; }
    grep "us per" $O/kp.txt | sed "s/^/force$f /" >> $O/kprof.txt
  done
done
cat $O/kprof.txt
