#!/bin/bash
# d = 512 flash attention (K/V register prefetch): op parity + timing at the VAE shape, VAE tests, bench
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r2u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "d512" -q --timeout 120 --timeout-method thread > $O/tests_op.log 2>&1
rc=$?; tail -2 $O/tests_op.log; grep -E "FAILED|Error" $O/tests_op.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u - > $O/attnw.txt 2>&1 <<'PY'
import math, torch
from image_restoration_and_enhancement_amd import _lib as L
from tests import opref as O
L.load()
dev = torch.device("cuda")
for dt in (torch.bfloat16, torch.float16):
    for B, Lq in ((8, 4096), (8, 9216)):
        qkv = (torch.randn(B, Lq, 1536, device=dev) * 0.5).to(dt)
        q, k, v = qkv[..., :512], qkv[..., 512:1024], qkv[..., 1024:]
        fl = 4.0 * B * Lq * Lq * 512
        for qg in (1,):
            for _ in range(2): O.attention(q, k, v, 1)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5): O.attention(q, k, v, 1)
            e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 5
            print(f"{str(dt):16s} B{B} L{Lq} qg{qg}: {ms*1e3:8.1f} us {fl/ms/1e9:7.1f} TF/s", flush=True)
PY
cat $O/attnw.txt
timeout -k 10 900 python -u -m pytest tests/test_models_gpu.py -k "vae" tests/test_fullsize_gpu.py::test_vae_512 -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "FAILED" $O/tests.log | head
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
grep -E "attnw|TFLOP/img" $O/bench.err; cat $O/bench.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --opt vae_flash=0 > $O/bench_noflash.json 2> $O/bench_noflash.err || exit $?
cat $O/bench_noflash.json
