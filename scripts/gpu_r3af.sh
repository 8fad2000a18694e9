#!/bin/bash
# Round 3: per-shape kernel table of the default bench step; attention MFMA priority A/B
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3af; mkdir -p $O
for op in attn40 cross40; do
  for v in 0 1; do
    timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 20 --opt attn_prio=$v > $O/kp.txt 2>&1 || { cat $O/kp.txt; exit 1; }
    grep "us per" $O/kp.txt | sed "s/^/prio$v /" >> $O/kprof.txt
  done
done
cat $O/kprof.txt
IRX_PROF_TOP=90 timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --opt prof_shapes=1 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
grep -E "ms/step" $O/bench.err | sed 's/irx::(anonymous namespace):://' | cut -c1-200 > $O/shapes.txt; head -70 $O/shapes.txt
