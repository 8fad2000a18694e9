#!/bin/bash
# One GPU session: pytest selection (a failing assertion does not stop the session; a crash, abort,
# fault or timeout does), then optional bench runs.  Usage: scripts/gpu_round.sh TAG "pytest args" "bench args"...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
tests=$1; shift
mkdir -p gpurun_out
if [ -n "$tests" ]; then
  timeout -k 10 1000 python -u -m pytest $tests -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/${tag}_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
i=0
for b in "$@"; do
  i=$((i+1))
  timeout -k 10 600 python -u bench.py $b > gpurun_out/${tag}_bench$i.json 2> gpurun_out/${tag}_bench$i.err
  rc=$?
  tail -3 gpurun_out/${tag}_bench$i.err; cat gpurun_out/${tag}_bench$i.json
  if [ $rc -ne 0 ]; then echo "bench rc=$rc: stopping"; exit $rc; fi
done
