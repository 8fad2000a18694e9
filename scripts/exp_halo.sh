#!/bin/bash
# halo conv tiles: op tests, per-shape A/B (conv_halo=0/1), bench A/B.
set -o pipefail
O=gpurun_out/halo; mkdir -p $O; : > $O/res.txt
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "halo or conv" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for sh in "16 64 64 320 0 320 3" "16 64 64 640 320 320 3" "16 64 64 320 320 320 3" "8 128 128 512 0 512 3" "8 64 64 512 0 512 3" "8 128 128 256 0 256 3"; do
  for t in 0 1; do
    timeout -k 10 60 python3 scripts/kshape.py conv $sh --iters 20 --opt conv_halo=$t >> $O/res.txt 2>&1 || exit 1
  done
done
for d in 1 2 3; do timeout -k 10 60 python3 scripts/kshape.py conv 16 64 64 320 0 320 3 --iters 20 --opt gemm_dbg=$d >> $O/res.txt 2>&1 || exit 1; done
grep -v amdgpu.ids $O/res.txt
for t in 1; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --opt conv_halo=$t > $O/bench$t.json 2> $O/bench$t.err || { tail $O/bench$t.err; exit 1; }
  echo "== halo=$t"; python -c "import json; d=json.load(open('$O/bench$t.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  grep "ms/step" $O/bench$t.err | head -10
done
