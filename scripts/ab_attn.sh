#!/bin/bash
# A/B of the attention kernels: the current library vs a saved baseline (scripts/_ab/libirx_base.so), kbench attn shapes
# (the baseline: `mkdir -p scripts/_ab && cp image_restoration_and_enhancement_amd/libirx.so scripts/_ab/libirx_base.so`
#  before the change is built; *.so files are git-ignored)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-ab_attn}; mkdir -p "$O"
for r in 1 2; do
  timeout -k 10 120 python -u scripts/kbench.py --only attn --iters 50 > "$O/new_$r.txt" 2>&1 || exit $?
  IRX_LIB=scripts/_ab/libirx_base.so timeout -k 10 120 python -u scripts/kbench.py --only attn --iters 50 > "$O/base_$r.txt" 2>&1 || exit $?
done
tail -n 12 "$O"/*.txt
