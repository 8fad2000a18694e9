#!/bin/bash
# resident-K/V cross-attention: parity, kernel A/B, bench
set -o pipefail
O=gpurun_out/r3q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attention" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for q in 0 1; do
  timeout -k 10 120 python -u scripts/kprof.py --op cross40 --opt attn_qrep=$q > $O/kprof_q$q.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_q1.txt 2>&1 || { tail -20 $O/bench_q1.txt; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --opt attn_qrep=0 > $O/bench_q0.txt 2>&1 || exit 1
tail -1 $O/bench_q1.txt; tail -1 $O/bench_q0.txt; cat $O/kprof_q*.txt
