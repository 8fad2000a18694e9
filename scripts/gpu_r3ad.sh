#!/bin/bash
# Round 3: N-major tile order (weights-heavy small-M shapes): per-shape timing, op tests, bench
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3ad; mkdir -p $O
timeout -k 10 600 python -u scripts/kbench.py --variants nm0,nm1,nm2 --iters 20 > $O/kbench.txt 2>&1 || { tail $O/kbench.txt; exit 1; }
grep -v amdgpu.ids $O/kbench.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm or conv" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
grep -E "ms/step" $O/bench.err | head -14; cat $O/bench.json | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --opt gemm_nmajor=0 > $O/bench0.json 2> $O/bench0.err || { tail $O/bench0.err; exit 1; }
cat $O/bench0.json | cut -c1-300
