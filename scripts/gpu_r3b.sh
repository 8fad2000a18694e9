#!/bin/bash
# Round 3: ping-pong halo conv — bit-exact vs the round-2 loop, conv tests, kernel timing; RCCL + graph tests
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3b; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_ops_gpu.py -k "halo" > $O/tests_ops.log 2>&1
rc=$?; tail -2 $O/tests_ops.log; grep -E "FAILED|Error" $O/tests_ops.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/kbench.py --only conv --variants halo1,halo2 --iters 20 > $O/kbench_conv.txt 2>&1 || { tail $O/kbench_conv.txt; exit 1; }
cat $O/kbench_conv.txt
timeout -k 10 600 $PT tests/test_rccl_gpu.py tests/test_graph_gpu.py > $O/tests_rccl_graph.log 2>&1
rc=$?; tail -2 $O/tests_rccl_graph.log; grep -E "FAILED|Error" $O/tests_rccl_graph.log | head
exit $rc
