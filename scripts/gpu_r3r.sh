#!/bin/bash
# Round 3: fp16 batch-invariance bisection over structural options (stage-wise diag, eps0 line)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3r; mkdir -p $O
for o in "--opt large_tiles=0" "--opt splitk_inkernel=0" "--opt halo_split=0" "--opt tile_256x320=0" "--opt attn_hm=0" "--opt gn_v2=0"; do
  timeout -k 10 200 python -u scripts/diag_bi2.py --dtype fp16 --res 256 $o > $O/d.txt 2>&1 || { tail -3 $O/d.txt; exit 1; }
  grep "eps0" $O/d.txt | cut -c1-200 | tee -a $O/bisect.txt
done
