#!/bin/bash
# library references (hipBLASLt / MIOpen / SDPA) beside the irx kernels at the UNet's batch-16 shapes
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/kbench.py --iters 10 --ref --variants s2 > gpurun_out/r2g_kbench.txt 2>&1 || exit $?
cat gpurun_out/r2g_kbench.txt
