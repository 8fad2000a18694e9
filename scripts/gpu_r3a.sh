#!/bin/bash
# Round 3, first pass: pipelined halo conv (bit-exact vs round 2 + conv tests), RCCL world-of-one, graph rebind,
# full-length e2e goldens; halo kernel timing (round-2 loop vs pipelined); default bench without the CPU leg
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3a; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_ops_gpu.py -k "halo" tests/test_rccl_gpu.py tests/test_graph_gpu.py > $O/tests_ops.log 2>&1
rc=$?; tail -3 $O/tests_ops.log; grep -E "FAILED|Error" $O/tests_ops.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/kbench.py --only conv --variants halo1,halo2 --iters 20 > $O/kbench_conv.txt 2>&1 || { tail $O/kbench_conv.txt; exit 1; }
cat $O/kbench_conv.txt
timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_e2e_golden_gpu.py > $O/tests_e2e.log 2>&1
rc=$?; grep -E "^E2E|PASSED|FAILED" $O/tests_e2e.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
grep -E "ms/step" $O/bench.err | head -14; cat $O/bench.json
