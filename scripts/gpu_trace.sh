#!/bin/bash
# Per-dispatch kernel trace of one bench step (CSV, grid sizes included) + library reference timings.
set -o pipefail
O=gpurun_out/trace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
find $O/kt -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/kt
timeout -k 10 600 python3 scripts/kbench.py --ref --variants s2 > $O/kbench.txt 2>&1; grep -v amdgpu.ids $O/kbench.txt
