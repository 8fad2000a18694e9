#!/bin/bash
set -o pipefail
O=gpurun_out/attn; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 2; do
timeout -k 10 400 python bench.py --no-cpu-baseline --opt attn_d40=$v > $O/bench$v.json 2> $O/bench$v.err || { tail $O/bench$v.err; exit 1; }
echo "== attn_d40=$v"; python -c "import json; d=json.load(open('$O/bench$v.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
grep "attn2" $O/bench$v.err | head -4
done
