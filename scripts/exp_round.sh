# op tests + kernel benches + one bench line (used for quick GPU iterations)
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py -x -q > gpurun_out/tests.log 2>&1; tail -3 gpurun_out/tests.log
timeout -k 10 300 python scripts/kbench.py > gpurun_out/kb.txt 2>&1; grep -v amdgpu.ids gpurun_out/kb.txt
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; cat gpurun_out/bench.json; grep "ms/step" gpurun_out/bench.err | head -14
