#!/bin/bash
# 8x8-level conv split-K sweep (forced tile / splits) vs the policy's choice (s2)
set -o pipefail
O=gpurun_out/r3t; mkdir -p $O
timeout -k 10 300 python -u scripts/kbench.py --only conv --match @8 --iters 20 \
  --variants s2,f128x320s8,f128x320s4,f128x320s2,f256x320s8,f256x320s4,f128x256s4,f128x256s8,f256x256s4,f128x128s4,f128x128s8,f128x128s2 > $O/kbench8.txt 2>&1 || { tail -20 $O/kbench8.txt; exit 1; }
cat $O/kbench8.txt
