#!/bin/bash
# GroupNorm-fused halo conv: parity tests, A/B bench, kernel trace (launch gaps) of the fused build
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -k "gn_conv3 or group_norm or conv_halo" tests/test_models_gpu.py tests/test_batch_invariance_gpu.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_fused.json 2> $O/bench_fused.err || exit $?
head -20 $O/bench_fused.err; cat $O/bench_fused.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --opt gn_fuse=0 > $O/bench_unfused.json 2> $O/bench_unfused.err || exit $?
cat $O/bench_unfused.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_trace.log 2>&1 || { tail $O/bench_trace.log; exit 1; }
f=$(find $O/kt -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace.csv; rm -rf $O/kt
python3 scripts/gap_summary.py $O/kernel_trace.csv 20 > $O/gaps.txt; cat $O/gaps.txt
python3 scripts/trace_summary.py $O/kernel_trace.csv 30 3 > $O/trace_summary.txt; head -25 $O/trace_summary.txt
