#!/bin/bash
# LayerNorm statistics, 8 lanes per row (ln_stats8): bit-exactness vs ln_kernel mode 2, bench A/B, kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3v; mkdir -p $O
timeout -k 10 400 python -u -m pytest -p tests.conftest scripts/scratch_ln_stats8.py -k stats8 -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --opt ln_stats8=1 > $O/bench_s1.txt 2>&1 || { tail -20 $O/bench_s1.txt; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_s0.txt 2>&1 || exit 1
tail -1 $O/bench_s1.txt | cut -c1-330; tail -1 $O/bench_s0.txt | cut -c1-330
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --opt ln_stats8=1 > $O/bench_prof.log 2>&1 || { tail $O/bench_prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv; rm -rf $O/prof
grep -E "ln_stats8|ln_kernel" $O/kernel_stats.csv | cut -c1-220
