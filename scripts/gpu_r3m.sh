#!/bin/bash
# Round 3: gemm_sk time decomposition (diagnostic builds: 1 no epilogue, 2 no MFMA, 3 neither, 4 no A DMA) and the
# fp16 batch-invariance stage diagnosis under several options
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3m; mkdir -p $O
for op in lin320 lin320r geglu320; do
  for d in 0 1 2 3 4; do
    lib=""; [ $d -gt 0 ] && lib="--lib scripts/_skdbg/libirx_skdbg$d.so"
    timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 20 $lib > $O/kp.txt 2>&1 || { cat $O/kp.txt; exit 1; }
    grep "us per" $O/kp.txt | sed "s/^/dbg$d /" >> $O/decomp.txt
  done
done
cat $O/decomp.txt
for o in "--dtype bf16" "--dtype fp16 --opt gemm_sk=0" "--dtype fp16 --opt attn_xcd=0" "--dtype fp16 --opt gn_parts=0" "--dtype fp16 --opt ln_fold=0"; do
  timeout -k 10 200 python -u scripts/diag_bi2.py --res 256 $o > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0" $O/d.txt | cut -c1-220 | tee -a $O/diag_bi2.txt
done
