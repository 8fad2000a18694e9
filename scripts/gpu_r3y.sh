#!/bin/bash
# Round 3: workspace overrun hunt (64 KiB guards after every arena allocation, checked at free)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3y; mkdir -p $O
timeout -k 10 400 python -u scripts/diag_bi2.py --dtype fp16 --res 256 --opt arena_guard=1 > $O/d.txt 2>&1 || { tail -5 $O/d.txt; exit 1; }
grep -c "arena guard" $O/d.txt; grep "arena guard" $O/d.txt | sort | uniq -c | head -30; grep "eps0" $O/d.txt | cut -c1-220
