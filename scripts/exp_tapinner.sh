#!/bin/bash
# conv K walk A/B: tap-outer (conv_tap_inner=0) vs channel-chunk-outer / tap-inner (=1); op tests first.
set -o pipefail
O=gpurun_out/tapin; mkdir -p $O; : > $O/res.txt
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "conv" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for sh in "16 64 64 320 0 320 3" "16 64 64 640 320 320 3" "16 32 32 640 0 640 3" "16 32 32 1280 640 640 3" "16 16 16 1280 0 1280 3" "8 128 128 512 0 512 3" "8 256 256 256 0 256 3" "8 512 512 128 0 128 3" "8 64 64 512 0 512 3"; do
  for t in 0 1; do
    timeout -k 10 60 python3 scripts/kshape.py conv $sh --iters 20 --opt conv_tap_inner=$t >> $O/res.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/res.txt
for t in 1 0; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --opt conv_tap_inner=$t > $O/bench$t.json 2> $O/bench$t.err || { tail $O/bench$t.err; exit 1; }
  echo "== tap_inner=$t"; python -c "import json; d=json.load(open('$O/bench$t.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  grep "ms/step" $O/bench$t.err | head -8
done
