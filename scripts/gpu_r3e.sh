#!/bin/bash
# Round 3: unrolled-tap ping-pong halo conv + fast-erf GEGLU — op tests, kernel timing, bench A/B
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3e; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_ops_gpu.py -k "halo or geglu or gemm_large" > $O/tests_ops.log 2>&1
rc=$?; tail -2 $O/tests_ops.log; grep -E "FAILED|Error" $O/tests_ops.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/kbench.py --only conv --variants halo1,halo2 --iters 20 > $O/kbench_conv.txt 2>&1 || { tail $O/kbench_conv.txt; exit 1; }
cat $O/kbench_conv.txt
for op in geglu320 conv320 lin320 lin1280; do timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 20 || exit 1; done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
grep -E "ms/step" $O/bench.err | head -16; cat $O/bench.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --opt ln_fold=0 > $O/bench_nofold.json 2> $O/bench_nofold.err || { tail $O/bench_nofold.err; exit 1; }
cat $O/bench_nofold.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > $O/bench2.json 2> $O/bench2.err || { tail $O/bench2.err; exit 1; }
cat $O/bench2.json
timeout -k 10 900 python3 scripts/pmc_top.py run --dir $O/top --timeout 280 || exit 1
python3 scripts/pmc_top.py summarize --dir $O/top --out $O/pmc_top.json --top 12
rm -rf $O/top/*/*.db
