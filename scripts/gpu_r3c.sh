#!/bin/bash
# Round 3: ping-pong halo + LayerNorm fold — op / model / e2e tests, kernel timing, bench, rocprof summary
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3c; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_ops_gpu.py -k "halo or layer_norm or gemm" > $O/tests_ops.log 2>&1
rc=$?; tail -2 $O/tests_ops.log; grep -E "FAILED|Error" $O/tests_ops.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 $PT -s tests/test_ln_fold_gpu.py tests/test_rccl_gpu.py tests/test_graph_gpu.py > $O/tests_fold.log 2>&1
rc=$?; tail -2 $O/tests_fold.log; grep -E "FAILED|Error|^ln_fold" $O/tests_fold.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/kbench.py --only conv --variants halo1,halo2 --iters 20 > $O/kbench_conv.txt 2>&1 || { tail $O/kbench_conv.txt; exit 1; }
cat $O/kbench_conv.txt
timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_e2e_golden_gpu.py > $O/tests_e2e.log 2>&1
rc=$?; grep -E "^E2E|PASSED|FAILED" $O/tests_e2e.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
grep -E "ms/step" $O/bench.err | head -16; cat $O/bench.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --opt halo_pipe=0 > $O/bench_halo1.json 2> $O/bench_halo1.err || { tail $O/bench_halo1.err; exit 1; }
cat $O/bench_halo1.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --opt ln_fold=0 > $O/bench_nofold.json 2> $O/bench_nofold.err || { tail $O/bench_nofold.err; exit 1; }
cat $O/bench_nofold.json
