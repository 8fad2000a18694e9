#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel-filtered) for one kernel of the default bench.
# Usage: bash scripts/gpu_pmc.sh <tag> <kernel-regex> <name-for-json>
set -e -o pipefail
TAG=$1; KRE=$2; NAME=$3
O=gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d $O/pmc_fetch -o f -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $O/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d $O/pmc_write -o w -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $O/pmc_write.log 2>&1
python3 scripts/pmc_traffic.py --fetch $O/pmc_fetch --write $O/pmc_write --kernel "$NAME" --out $O/pmc_traffic.json
rm -f $O/pmc_fetch/*.db $O/pmc_write/*.db
cat $O/pmc_traffic.json
