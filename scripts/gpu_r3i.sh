#!/bin/bash
# Round 3: fp16 batch-invariance diagnosis, default bench (CPU baseline 4 images), rocprof stats, large-tile decomposition
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3i; mkdir -p $O
for o in "" "--opt ln_fold=0" "--opt halo_pipe=0" "--opt conv_halo=0"; do
  timeout -k 10 120 python -u scripts/diag_bi.py --dtype fp16 --res 256 $o >> $O/diag_bi.txt 2>&1 || { tail $O/diag_bi.txt; exit 1; }
done
grep "whole" $O/diag_bi.txt
timeout -k 10 560 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > $O/bench_prof.log 2>&1 || { tail $O/bench_prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv; rm -rf $O/prof
head -14 $O/kernel_stats.csv | cut -c1-200
for op in geglu320 ff1_320 ff2_320 lin320 lin1280 conv320; do
  for d in 0 1 2 3; do
    timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 20 --opt gemm_dbg=$d > $O/kp.txt 2>&1 || { cat $O/kp.txt; exit 1; }
    grep "us per" $O/kp.txt | sed "s/^/dbg$d /" >> $O/decomp.txt
  done
done
cat $O/decomp.txt
