#!/bin/bash
# GroupNorm partial fold inside gn_apply for small partial sets: parity, batch invariance, bench, trace
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_models_gpu.py tests/test_batch_invariance_gpu.py tests/test_graph_gpu.py tests/test_fullsize_gpu.py::test_unet_512 tests/test_fullsize_gpu.py::test_vae_512 tests/test_fullsize_gpu.py::test_bf16_baseline_batches -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "FAILED" $O/tests.log | head
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
head -6 $O/bench.err; cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > $O/bench_trace.log 2>&1 || { tail $O/bench_trace.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace.csv
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv; rm -rf $O/prof
python3 scripts/trace_summary.py $O/kernel_trace.csv 80 5 > $O/trace_summary.txt; head -24 $O/trace_summary.txt; grep -E "gn_|ln_" $O/trace_summary.txt | tail -20
rm -f $O/kernel_trace.csv
