#!/bin/bash
# Round 3: stale-read hunt — the UNet workspace poisoned with 0xFF (NaN) before every forward, stage-wise diag
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3q; mkdir -p $O
for o in "--dtype fp16 --res 256" "--dtype bf16 --res 256" "--dtype fp16 --res 128"; do
  IRX_WS_POISON=1 timeout -k 10 200 python -u scripts/diag_bi2.py $o > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "max|d|" $O/d.txt | cut -c1-200 | tee -a $O/diag_poison.txt
done
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm_sk" > $O/tests_sk.log 2>&1
rc=$?; tail -2 $O/tests_sk.log
