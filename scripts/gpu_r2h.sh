#!/bin/bash
# kernel trace of bench steps (launch-gap share) + rocprofv3 stats of the default bench
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2h; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/bench_trace.log 2>&1 || { tail $O/bench_trace.log; exit 1; }
f=$(find $O/kt -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace.csv; rm -rf $O/kt
python3 scripts/gap_summary.py $O/kernel_trace.csv 20 > $O/gaps.txt; cat $O/gaps.txt
python3 scripts/trace_summary.py $O/kernel_trace.csv 30 3 > $O/trace_summary.txt; head -25 $O/trace_summary.txt
