#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_predictions_gpu.py tests/test_batch_invariance_gpu.py tests/test_models_gpu.py "tests/test_ops_gpu.py::test_attention" tests/test_fullsize_gpu.py::test_attention_spike_at_4096 tests/test_fullsize_gpu.py::test_bf16_baseline_batches -v --timeout 300 --timeout-method thread > gpurun_out/r2f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2f_tests.log; grep FAILED gpurun_out/r2f_tests.log | head
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/attn3bench.py --iters 10 --dtypes bf16 --variants v3,v3-hm,r1 > gpurun_out/r2f_attn.txt 2>&1 || exit $?
cat gpurun_out/r2f_attn.txt
