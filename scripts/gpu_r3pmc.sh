#!/bin/bash
# Round 3 final: rocprofv3 PMC passes (MFMA busy, FETCH / WRITE) for the top kernels of the default bench at HEAD
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3pmcf; mkdir -p $O
timeout -k 10 900 python3 scripts/pmc_top.py run --dir $O/top --timeout 280 || exit 1
python3 scripts/pmc_top.py summarize --dir $O/top --out $O/pmc_top.json --top 14
rm -rf $O/top/*/*.db
