set -e
O=gpurun_out/exp1; mkdir -p $O
for d in 0 1 2 3; do
  timeout -k 10 120 python3 scripts/kshape.py gemm 65536 2560 320 --opt gemm_deep=0 --opt gemm_dbg=$d >> $O/res.txt 2>&1
  timeout -k 10 120 python3 scripts/kshape.py conv 16 64 64 320 0 320 3 --opt gemm_deep=0 --opt gemm_dbg=$d >> $O/res.txt 2>&1
  timeout -k 10 120 python3 scripts/kshape.py gemm 65536 320 320 --opt gemm_deep=0 --opt gemm_dbg=$d >> $O/res.txt 2>&1
done
for k in 640 1280 2560; do
  timeout -k 10 120 python3 scripts/kshape.py gemm 65536 2560 $k --opt gemm_deep=0 >> $O/res.txt 2>&1
done
cat $O/res.txt | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc1 -o p -- python3 scripts/kshape.py gemm 65536 2560 320 --opt gemm_deep=0 --iters 5 > $O/pmc1.log 2>&1
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc2 -o p -- python3 scripts/kshape.py conv 16 64 64 320 0 320 3 --opt gemm_deep=0 --iters 5 > $O/pmc2.log 2>&1
echo done
