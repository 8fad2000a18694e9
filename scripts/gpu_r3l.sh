#!/bin/bash
# Round 3: gemm_sk v3 (exact vmcnt accounting incl. the epilogue stores): tests, timing, bench; stage-wise batch-invariance
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3l; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm_sk" > $O/tests_sk.log 2>&1
rc=$?; tail -2 $O/tests_sk.log; grep -E "FAILED|Error|assert" $O/tests_sk.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
for op in lin320 lin320r qkv320 geglu320; do
  for v in 0 1 2; do
    timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 20 --opt gemm_sk=$v > $O/kp.txt 2>&1 || { cat $O/kp.txt; exit 1; }
    grep "us per" $O/kp.txt | sed "s/^/sk$v /" >> $O/kprof.txt
  done
done
cat $O/kprof.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_models_gpu.py tests/test_ln_fold_gpu.py tests/test_e2e_golden_gpu.py tests/test_graph_gpu.py > $O/tests_models.log 2>&1
rc=$?; tail -2 $O/tests_models.log; grep -E "FAILED|^E2E" $O/tests_models.log | cut -c1-200 | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
grep -E "ms/step" $O/bench.err | head -24; cat $O/bench.json
timeout -k 10 200 python -u scripts/diag_bi2.py --dtype fp16 --res 256 > $O/diag_bi2.txt 2>&1; cat $O/diag_bi2.txt | grep "max|d|" | cut -c1-200
