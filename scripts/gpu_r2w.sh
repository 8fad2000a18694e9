#!/bin/bash
# attn3: full key tiles without mask code, d = 40 at 3 waves/SIMD — parity + microbench + bench
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -k "attention" tests/test_fullsize_gpu.py::test_attention_production_shapes tests/test_models_gpu.py::test_clip -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "FAILED" $O/tests.log | head
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/attn3bench.py --iters 10 --dtypes bf16 --variants v3-hm > $O/attn.txt 2>&1 || exit $?
cat $O/attn.txt
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
grep -E "attn3" $O/bench.err; cat $O/bench.json
