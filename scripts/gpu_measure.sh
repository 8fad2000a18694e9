#!/bin/bash
# One GPU measurement pass (run through gpurun): pipeline tests, default bench line (with CPU baseline),
# rocprofv3 kernel-trace stats of the same bench, and two PMC passes for the dominant kernel's traffic.
# Usage: bash scripts/gpu_measure.sh <tag> [kernel-regex]
set -e -o pipefail
TAG=${1:-r01}
KRE=${2:-gemm2_kernel<128, 320, 2, 4, 64, 2, true, false, false>}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err
echo "bench: $(cat $O/bench.json)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
echo "prof bench: $(cat $O/bench_prof.json)"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $O/pmc_fetch -o f -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $O/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $O/pmc_write -o w -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $O/pmc_write.log 2>&1
python3 scripts/rocpd_stats.py $(ls $O/prof/*results.db | head -1) $O/kernel_stats.csv
python3 scripts/pmc_traffic.py --fetch $O/pmc_fetch --write $O/pmc_write --kernel "$KRE" --out $O/pmc_traffic.json
rm -f $O/prof/*.db
echo done
