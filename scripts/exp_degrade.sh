#!/bin/bash
set -o pipefail
O=gpurun_out/degrade; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_degrade_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python scripts/degrade_bench.py 2>&1 | grep -v amdgpu.ids | tee $O/bench.txt
