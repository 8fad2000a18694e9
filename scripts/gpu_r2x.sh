#!/bin/bash
# single-launch GroupNorm for small tensors: op / model parity, batch invariance, bench A/B
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "group_norm" -q --timeout 120 --timeout-method thread > $O/tests_op.log 2>&1
rc=$?; tail -2 $O/tests_op.log; grep -E "FAILED" $O/tests_op.log | head
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_models_gpu.py tests/test_batch_invariance_gpu.py tests/test_graph_gpu.py tests/test_fullsize_gpu.py::test_unet_512 tests/test_fullsize_gpu.py::test_bf16_baseline_batches -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "FAILED" $O/tests.log | head
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
grep -E "gn_" $O/bench.err; cat $O/bench.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --opt gn_small=0 > $O/bench_nosmall.json 2> $O/bench_nosmall.err || exit $?
cat $O/bench_nosmall.json
