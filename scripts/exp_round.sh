# op tests + kernel benches + bench lines (used for quick GPU iterations)
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py -x -q > gpurun_out/tests.log 2>&1; tail -3 gpurun_out/tests.log
timeout -k 10 300 python scripts/kbench.py --only conv > gpurun_out/kb.txt 2>&1; timeout -k 10 300 python scripts/kbench.py --only gemm >> gpurun_out/kb.txt 2>&1; timeout -k 10 300 python scripts/kbench.py --only attn >> gpurun_out/kb.txt 2>&1; grep -v amdgpu.ids gpurun_out/kb.txt
for m in gemm_deep=0 gemm_deep=2 gemm_small=1; do
timeout -k 10 600 python bench.py --no-cpu-baseline --opt $m > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err; echo "== $m"; cat gpurun_out/bench_$m.json; grep "ms/step" gpurun_out/bench_$m.err | head -14
done
