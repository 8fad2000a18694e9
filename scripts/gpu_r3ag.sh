#!/bin/bash
# Round 3: tile / split sweep for the C x C projections at the 32x32 and 16x16 levels (gemm_force = BM*1e5 + BN*100 + splits)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3ag; mkdir -p $O
for op in lin1280 lin640; do
  for f in 0 12812801 12812802 12832001 12832002 12832004 12825601 12825602 25632001 25632002 25625601 25612801 25612802; do
    timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 30 --opt gemm_force=$f > $O/kp.txt 2>&1 || { cat $O/kp.txt | tail -2; continue; }
    grep "us per" $O/kp.txt | sed "s/^/force$f /" >> $O/kprof.txt
  done
done
cat $O/kprof.txt
