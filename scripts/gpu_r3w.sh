#!/bin/bash
# Round 3: GEMM-op row-wise batch invariance at the 256x256 UNet shapes with the canonical image count passed
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3w; mkdir -p $O
timeout -k 10 200 python -u scripts/diag_gemm_rows.py > $O/gemm_rows.txt 2>&1; grep -v amdgpu.ids $O/gemm_rows.txt
timeout -k 10 200 python -u scripts/diag_gemm_rows.py splitk_inkernel=0 > $O/gemm_rows2.txt 2>&1; grep -v amdgpu.ids $O/gemm_rows2.txt
