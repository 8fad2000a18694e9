#!/bin/bash
# d = 512 flash attention (VAE mid block): op parity, VAE parity, full-size VAE, pipelines, bench
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "d512" -v --timeout 120 --timeout-method thread > $O/tests_op.log 2>&1
rc=$?; tail -2 $O/tests_op.log; grep -E "FAILED|Error" $O/tests_op.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_models_gpu.py tests/test_fullsize_gpu.py::test_vae_512 tests/test_fullsize_gpu.py::test_bf16_baseline_batches tests/test_fullsize_gpu.py::test_fp16_colorize_768_config5 tests/test_pipeline_gpu.py tests/test_batch_invariance_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "FAILED" $O/tests.log | head
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
grep -E "attnw|TFLOP/img" $O/bench.err; cat $O/bench.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --opt vae_flash=0 > $O/bench_noflash.json 2> $O/bench_noflash.err || exit $?
cat $O/bench_noflash.json
