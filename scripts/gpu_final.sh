#!/bin/bash
# Round-end GPU pass: every -m gpu test, smoke(), then the measurement pass (bench + rocprof + PMC).
set -o pipefail
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo smoke ok
bash scripts/gpu_measure.sh ${1:-r01v6} "${2:-gemm2_kernel<128, 320, 2, 4, 64, 2, true, false, false, false>}"
