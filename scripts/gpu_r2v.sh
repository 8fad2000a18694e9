#!/bin/bash
# BASELINE configs 3-5 as per-GPU shards (bench --task), with the roofline entry
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2v; mkdir -p $O
for t in sr inpaint colorize; do
  timeout -k 10 600 python -u bench.py --task $t --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$t.json 2> $O/bench_$t.err || { tail $O/bench_$t.err; exit 1; }
  cat $O/bench_$t.json
done
