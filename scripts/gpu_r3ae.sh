#!/bin/bash
# Round 3: per-shape kernel time table of the default bench step (profiler keys with shapes)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3ae; mkdir -p $O
IRX_PROF_TOP=90 timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --opt prof_shapes=1 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
grep -E "ms/step" $O/bench.err | sed 's/irx::(anonymous namespace):://' | cut -c1-230
