#!/bin/bash
# Round 3 checkpoint at HEAD (re-used for the later passes): every -m gpu test, smoke(), the default bench (CPU baseline on 4 images + parity
# leg), rocprofv3 kernel stats of the bench
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3final3; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "FAILED" $O/tests.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > $O/bench_prof.log 2>&1 || { tail $O/bench_prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv; rm -rf $O/prof
head -14 $O/kernel_stats.csv | cut -c1-200
