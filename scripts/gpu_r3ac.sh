#!/bin/bash
# Round 3: GEGLU fusion only on whole per-image row tiles: batch-invariance diag + the batch-invariance tests + bench
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3ac; mkdir -p $O
for c in 3 1; do
  timeout -k 10 200 python -u scripts/diag_bi2.py --dtype fp16 --res 256 --split $c > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0\|lat2" $O/d.txt | cut -c1-250 | tee -a $O/bisect.txt
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_batch_invariance_gpu.py tests/test_models_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep FAILED $O/tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json | cut -c1-400
