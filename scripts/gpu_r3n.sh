#!/bin/bash
# Round 3: gemm_sk v4 (every A / residual / statistics transfer LDS-DMA with exact waits; no compiler waits in the loop)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3n; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm_sk" > $O/tests_sk.log 2>&1
rc=$?; tail -2 $O/tests_sk.log; grep -E "FAILED|Error|assert" $O/tests_sk.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
for op in lin320 lin320r qkv320 geglu320; do
  for d in 0 1 2 4; do
    lib=""; [ $d -gt 0 ] && lib="--lib scripts/_skdbg/libirx_skdbg$d.so"
    timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 20 $lib > $O/kp.txt 2>&1 || { cat $O/kp.txt; exit 1; }
    grep "us per" $O/kp.txt | sed "s/^/dbg$d /" >> $O/kprof.txt
  done
  timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 20 --opt gemm_sk=0 > $O/kp.txt 2>&1 || { cat $O/kp.txt; exit 1; }
  grep "us per" $O/kp.txt | sed "s/^/sk0 /" >> $O/kprof.txt
done
cat $O/kprof.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_models_gpu.py tests/test_ln_fold_gpu.py tests/test_e2e_golden_gpu.py tests/test_graph_gpu.py > $O/tests_models.log 2>&1
rc=$?; tail -2 $O/tests_models.log; grep -E "FAILED|^E2E" $O/tests_models.log | cut -c1-200 | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
grep -E "ms/step" $O/bench.err | head -24; cat $O/bench.json
for o in "--dtype fp16 --res 128" "--dtype fp16 --res 512"; do
  timeout -k 10 200 python -u scripts/diag_bi2.py $o > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0" $O/d.txt | cut -c1-220 | tee -a $O/diag_bi2.txt
done
