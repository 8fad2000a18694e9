#!/bin/bash
set -o pipefail
O=gpurun_out/attn; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
grep "ms/step" $O/bench.err | head -8
