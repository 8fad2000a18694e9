#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_predictions_gpu.py tests/test_batch_invariance_gpu.py "tests/test_ops_gpu.py::test_attention" tests/test_ops_gpu.py::test_attention_v3_vs_v2_and_head_major tests/test_ops_gpu.py::test_gemm tests/test_ops_gpu.py::test_gemm_large tests/test_fullsize_gpu.py::test_attention_production_shapes tests/test_fullsize_gpu.py::test_attention_spike_at_4096 tests/test_fullsize_gpu.py::test_unet_512 tests/test_models_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r2e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2e_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/attn3bench.py --iters 10 --dtypes bf16 > gpurun_out/r2e_attn.txt 2>&1 || exit $?
cat gpurun_out/r2e_attn.txt
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r2e_bench.json 2> gpurun_out/r2e_bench.err || exit $?
head -16 gpurun_out/r2e_bench.err; cat gpurun_out/r2e_bench.json
