#!/bin/bash
# attn3 (double-buffered LDS) + head-major engine layout: tests, micro-bench, bench, and SQ counters for the
# d = 40 self-attention kernel (separate rocprofv3 --pmc passes, each under its own time limit).
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_batch_invariance_gpu.py "tests/test_ops_gpu.py::test_attention" tests/test_ops_gpu.py::test_attention_v3_vs_v2_and_head_major tests/test_fullsize_gpu.py::test_attention_spike_at_4096 tests/test_fullsize_gpu.py::test_unet_512 tests/test_models_gpu.py tests/test_pipeline_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r2d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2d_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/attn3bench.py --iters 10 --dtypes bf16 > gpurun_out/r2d_attn.txt 2>&1 || exit $?
cat gpurun_out/r2d_attn.txt
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r2d_bench.json 2> gpurun_out/r2d_bench.err || exit $?
head -14 gpurun_out/r2d_bench.err; cat gpurun_out/r2d_bench.json
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass -d gpurun_out/pmc_$tag -o pmc --output-format csv -- python3 scripts/attn3bench.py --iters 3 --rounds 1 --dtypes bf16 --only "self d40 L4096" --variants v3 > gpurun_out/pmc_$tag.log 2>&1
  echo "pmc pass $tag rc=$?"
done
exit 0
