#!/bin/bash
# Same-box A/B of the default bench step: the current library vs a saved baseline (scripts/_ab/libirx_base.so),
# alternated twice; each line -> gpurun_out/<tag>/{new,base}_<i>.json
# (the baseline: `mkdir -p scripts/_ab && cp image_restoration_and_enhancement_amd/libirx.so scripts/_ab/libirx_base.so`
#  before the change is built; *.so files are git-ignored)
set -u
export IRX_PROF_TOP=${IRX_PROF_TOP:-80}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-ab_bench}; shift || true
mkdir -p "$O"
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > "$O/new_$r.json" 2> "$O/new_$r.err" || exit $?
  IRX_LIB=scripts/_ab/libirx_base.so timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > "$O/base_$r.json" 2> "$O/base_$r.err" || exit $?
done
for f in "$O"/*.json; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'])" "$f"; done
