#!/bin/bash
# Round 3: ping-pong dense GEMM / im2col conv main loop — bit-exact vs round 2, op / model / e2e tests, timing, bench
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3f; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_ops_gpu.py > $O/tests_ops.log 2>&1
rc=$?; tail -2 $O/tests_ops.log; grep -E "FAILED|Error" $O/tests_ops.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u scripts/kbench.py --only gemm --variants pp0,pp1 --iters 20 > $O/kbench_gemm.txt 2>&1 || { tail $O/kbench_gemm.txt; exit 1; }
cat $O/kbench_gemm.txt
timeout -k 10 600 python -u scripts/kbench.py --only conv --variants pp0,pp1 --iters 20 > $O/kbench_conv.txt 2>&1 || { tail $O/kbench_conv.txt; exit 1; }
cat $O/kbench_conv.txt
timeout -k 10 900 $PT -s tests/test_models_gpu.py tests/test_ln_fold_gpu.py tests/test_e2e_golden_gpu.py > $O/tests_models.log 2>&1
rc=$?; tail -2 $O/tests_models.log; grep -E "FAILED|^E2E" $O/tests_models.log | cut -c1-200 | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
grep -E "ms/step" $O/bench.err | head -20; cat $O/bench.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --opt gemm_pp=0 > $O/bench_pp0.json 2> $O/bench_pp0.err || { tail $O/bench_pp0.err; exit 1; }
grep -E "ms/step" $O/bench_pp0.err | head -12; cat $O/bench_pp0.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --opt ln_fold=0 > $O/bench_nofold.json 2> $O/bench_nofold.err || { tail $O/bench_nofold.err; exit 1; }
grep -E "ms/step" $O/bench_nofold.err | head -16; cat $O/bench_nofold.json
timeout -k 10 900 python3 scripts/pmc_top.py run --dir $O/top --timeout 280 || exit 1
python3 scripts/pmc_top.py summarize --dir $O/top --out $O/pmc_top.json --top 12
rm -rf $O/top/*/*.db
