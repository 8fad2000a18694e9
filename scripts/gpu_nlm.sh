#!/bin/bash
# NLM / filter GPU pass: parity tests, v2 (default) vs v1 bench, rocprofv3 kernel stats, SQ PMC pass.
set -e -o pipefail
O=gpurun_out/nlm4; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_nlm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 200 python scripts/nlm_bench.py --cpu > $O/bench.json 2> $O/bench.err; cat $O/bench.json
timeout -k 10 200 python scripts/nlm_bench.py --v2 0 > $O/bench_v1.json 2> $O/bench_v1.err; cat $O/bench_v1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o nlm -- python3 scripts/nlm_bench.py > $O/prof.log 2>&1
python3 scripts/rocpd_stats.py $(ls $O/prof/*results.db | head -1) $O/kernel_stats.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex nlm2_kernel -d $O/pmc -o p -- python3 scripts/nlm_bench.py --iters 1 > $O/pmc.log 2>&1
rm -f $O/prof/*.db
echo done
