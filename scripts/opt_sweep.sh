#!/bin/bash
# Bench-step option sweep on one box: each argument is one variant ("default" or a comma-separated list of
# irx options name=value), each run bench.py --steps 10 --warmup 2 --no-cpu-baseline; lines -> gpurun_out/<tag>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
O=gpurun_out/$tag; mkdir -p "$O"
i=0
for v in "$@"; do
  i=$((i + 1))
  opts=()
  if [ "$v" != default ]; then IFS=',' read -ra kv <<< "$v"; for x in "${kv[@]}"; do opts+=(--opt "$x"); done; fi
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline "${opts[@]}" > "$O/v$i.json" 2> "$O/v$i.err" || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(f\"{d['ms_per_step']:8.2f} ms/step {d['value']:8.3f} img/s  {sys.argv[2]}\")" "$O/v$i.json" "$v"
done
