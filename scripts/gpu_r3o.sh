#!/bin/bash
# Round 3: attention row-wise diagnosis (distinct K/V per row); gemm_sk persistent-grid size sweep; CU count
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3o; mkdir -p $O
python3 -c "import torch; p=torch.cuda.get_device_properties(0); print('CUs', p.multi_processor_count, p.name)"
timeout -k 10 200 python -u scripts/diag_attn_rows.py > $O/attn_rows.txt 2>&1; cat $O/attn_rows.txt | grep -v amdgpu.ids
for op in lin320 geglu320; do
  for b in 32 31 30 28 24 16; do
    timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 20 --opt gemm_sk_blocks=$b > $O/kp.txt 2>&1 || { cat $O/kp.txt; exit 1; }
    grep "us per" $O/kp.txt | sed "s/^/blocks$b /" >> $O/kprof.txt
  done
done
cat $O/kprof.txt
