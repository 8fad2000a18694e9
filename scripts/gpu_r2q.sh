#!/bin/bash
# HBM traffic (FETCH_SIZE x2 + WRITE_SIZE, separate passes) of the bench's dominant kernel (halo conv)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2q; mkdir -p $O
KRE='gemm2_kernel<unsigned short, 256, 160, 4, 2, 64, 3, true, false, false, true>'
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gemm2_kernel<unsigned short, 256, 160" --output-format csv -d $O/pmc_fetch -o f -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $O/pmc_fetch.log 2>&1 || { tail $O/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gemm2_kernel<unsigned short, 256, 160" --output-format csv -d $O/pmc_write -o w -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $O/pmc_write.log 2>&1 || { tail $O/pmc_write.log; exit 1; }
python3 scripts/pmc_traffic.py --fetch $O/pmc_fetch --write $O/pmc_write --kernel "$KRE" --out $O/pmc_traffic_halo.json
