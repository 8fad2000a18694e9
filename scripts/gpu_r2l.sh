#!/bin/bash
# GEMM / conv pipeline variants at the UNet shapes (A/B for a per-shape policy) + gn_conv3 test fix
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "gn_conv3" -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 500 python -u scripts/kbench.py --iters 10 --only gemm --variants s2,ring32,ring64,small > $O/kbench_gemm.txt 2>&1 || exit $?
cat $O/kbench_gemm.txt
timeout -k 10 500 python -u scripts/kbench.py --iters 10 --only conv --variants s2,ring32,ring64 > $O/kbench_conv.txt 2>&1 || exit $?
cat $O/kbench_conv.txt
