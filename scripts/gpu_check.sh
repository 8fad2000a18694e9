#!/bin/bash
# Full GPU check (through gpurun): -m gpu tests, smoke, default bench + option A/B lines.
set -o pipefail
O=gpurun_out/check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo smoke ok
for m in "" "--opt gemm_small=1" "--opt gemm_deep=2" "--opt gn_v2=0"; do
  timeout -k 10 400 python bench.py --no-cpu-baseline $m > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  echo "== $m"; cat $O/bench.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  grep "ms/step" $O/bench.err | head -14
done
