#!/bin/bash
# Quick GPU iteration: selected tests (-k expr in $1), then the default bench line (+ kernel table).
set -o pipefail
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${1:-.}" > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
shift
timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
grep "ms/step" $O/bench.err | head -14
