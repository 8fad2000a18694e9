#!/bin/bash
# Round 3: time decomposition of the large-tile kernels (gemm_dbg 1 = no epilogue, 2 = no MFMAs, 3 = neither)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r3g; mkdir -p $O
for op in conv320 lin320 geglu320 ff1_320 ff2_320 lin1280; do
  for d in 0 1 2 3; do
    timeout -k 10 120 python -u scripts/kprof.py --op $op --iters 20 --opt gemm_dbg=$d 2>&1 | grep "us per" | sed "s/^/dbg$d /" || exit 1
  done
done | tee $O/decomp.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "layer_norm" > $O/tests_ln.log 2>&1; tail -1 $O/tests_ln.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --opt ln_fold=0 > $O/bench_nofold.json 2> $O/bench_nofold.err || { tail $O/bench_nofold.err; exit 1; }
grep -E "ln_kernel" $O/bench_nofold.err; cat $O/bench_nofold.json
