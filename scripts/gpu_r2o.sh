#!/bin/bash
# graph recorded right after the first eager loop: graph tests + default bench (W = 1)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_pipeline_gpu.py tests/test_predictions_gpu.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED" $O/tests.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/bench_10.json 2> $O/bench_10.err || { tail $O/bench_10.err; exit 1; }
cat $O/bench_10.json
