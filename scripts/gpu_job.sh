#!/bin/bash
# One GPU session as a list of steps, each under its own time limit; the session stops at the first step that fails
# (a failing test, a crash, an abort, a fault or a timeout), so nothing more runs on a GPU in an unknown state.
#
#   scripts/gpu_job.sh TAG STEP [STEP ...]       (outputs under gpurun_out/TAG/)
#
# steps (fields separated by '|'):
#   tests|<pytest args>[|<-k expr>]     python -u -m pytest <args> [-k <expr>] -v --timeout 300 --timeout-method thread
#   smoke                               __graft_entry__.smoke()
#   bench|<name>|<bench.py args>        bench line -> <name>.json, log -> <name>.err
#   prof|<name>|<bench.py args>         rocprofv3 --kernel-trace --stats of bench.py -> <name>_kernel_stats.csv
#   trace|<name>|<bench.py args>        rocprofv3 --kernel-trace of bench.py, GPU idle inside the last two steps
#                                       (scripts/step_gaps.py) -> <name>.txt
#   pmc|<name>|<pmc_top.py run args>    PMC passes of the bench's top kernels (scripts/pmc_top.py) -> <name>.json
#   kpmc|<name>|<regex>|<counters>|<kprof.py args>   one rocprofv3 --pmc pass over scripts/kprof.py (one hot op looped),
#                                       kernels matching <regex> -> <name>.txt (mean per dispatch, scripts/pmc_dump.py)
#   py|<name>|<script> <args>           any python script -> <name>.txt
#   run|<name>|<program> <args>         any program (no shell) -> <name>.txt
#   sec|<seconds>                       time limit of the following steps (default 600)
#   torchrun|<name>|<nproc>|<bench.py args>   bench.py on <nproc> GPUs of one node, one rank per GPU over RCCL
#                                       (python -m torch.distributed.run ... --master-addr 127.0.0.1) -> <name>.json
#
# BASELINE.json's multi-GPU configs (the round-end driver runs the 1/2/4/8 scaling itself; these are the same runs):
#   configs[3] inpaint 512x512, batch 32 over 4 GPUs:  scripts/gpu_job.sh cfg3 "torchrun|inpaint4|4|--task inpaint"
#   configs[4] colorize 768x768 fp16, batch 64 over 8: scripts/gpu_job.sh cfg4 "torchrun|colorize8|8|--task colorize"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export IRX_PROF_TOP=${IRX_PROF_TOP:-60}   # bench.py: kernels listed in the profiled step's log
tag=$1; shift
O=gpurun_out/$tag
mkdir -p "$O"
lim=600
fail() { echo "step '$1' failed (rc=$2)"; exit "$2"; }
for step in "$@"; do
  IFS='|' read -r kind name rest <<< "$step"
  echo "== $(date +%T) $kind $name"
  case "$kind" in
    sec) lim=$name ;;
    tests)
      kx=(); [ -n "$rest" ] && kx=(-k "$rest")
      timeout -k 10 "$lim" python -u -m pytest $name "${kx[@]}" -v --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1
      rc=$?; tail -4 "$O/tests.log"; [ $rc -eq 0 ] || fail tests $rc ;;
    smoke)
      timeout -k 10 "$lim" python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
      rc=$?; tail -3 "$O/smoke.log"; [ $rc -eq 0 ] || fail smoke $rc ;;
    bench)
      timeout -k 10 "$lim" python -u bench.py $rest > "$O/$name.json" 2> "$O/$name.err"
      rc=$?; tail -3 "$O/$name.err"; cut -c1-400 "$O/$name.json"; [ $rc -eq 0 ] || fail "$name" $rc ;;
    prof)
      timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o prof -- \
        python3 bench.py $rest > "$O/$name.log" 2>&1
      rc=$?; [ $rc -eq 0 ] || { tail "$O/$name.log"; fail "$name" $rc; }
      f=$(find "$O/prof_$name" -name "*kernel_stats.csv" | head -1)
      cp "$f" "$O/${name}_kernel_stats.csv" && rm -rf "$O/prof_$name"
      head -12 "$O/${name}_kernel_stats.csv" | cut -c1-200 ;;
    trace)
      timeout -k 10 "$lim" rocprofv3 --kernel-trace --output-format csv -d "$O/trace_$name" -o tr -- \
        python3 bench.py $rest > "$O/$name.log" 2>&1
      rc=$?; [ $rc -eq 0 ] || { tail "$O/$name.log"; fail "$name" $rc; }
      f=$(find "$O/trace_$name" -name "*kernel_trace.csv" | head -1)
      python3 scripts/step_gaps.py "$f" --steps 2 > "$O/$name.txt"; cat "$O/$name.txt"
      rm -rf "$O/trace_$name" ;;
    pmc)
      timeout -k 10 "$lim" python3 scripts/pmc_top.py run --dir "$O/pmc_$name" $rest
      rc=$?; [ $rc -eq 0 ] || fail "$name" $rc
      python3 scripts/pmc_top.py summarize --dir "$O/pmc_$name" --out "$O/$name.json" --top 14
      rm -rf "$O/pmc_$name"/*/*.db ;;
    kpmc)
      IFS='|' read -r rx ctrs kargs <<< "$rest"
      timeout -s KILL "$lim" rocprofv3 --pmc $ctrs --kernel-include-regex "$rx" --output-format csv \
        -d "$O/kpmc_$name" -o p -- python3 scripts/kprof.py $kargs > "$O/$name.log" 2>&1
      rc=$?; [ $rc -eq 0 ] || { tail "$O/$name.log"; fail "$name" $rc; }
      python3 scripts/pmc_dump.py "$rx" "$O/kpmc_$name" > "$O/$name.txt"; cat "$O/$name.txt"
      rm -rf "$O/kpmc_$name" ;;
    py)
      timeout -k 10 "$lim" python3 -u $rest > "$O/$name.txt" 2>&1
      rc=$?; tail -40 "$O/$name.txt"; [ $rc -eq 0 ] || fail "$name" $rc ;;
    run)
      timeout -k 10 "$lim" $rest > "$O/$name.txt" 2>&1
      rc=$?; tail -40 "$O/$name.txt"; [ $rc -eq 0 ] || fail "$name" $rc ;;
    torchrun)
      IFS='|' read -r np bargs <<< "$rest"
      timeout -k 10 "$lim" python -m torch.distributed.run --nnodes=1 --nproc-per-node "$np" --master-addr 127.0.0.1 \
        --master-port "${IRX_MASTER_PORT:-29531}" bench.py --gpus "$np" $bargs > "$O/$name.json" 2> "$O/$name.err"
      rc=$?; tail -3 "$O/$name.err"; cut -c1-400 "$O/$name.json"; [ $rc -eq 0 ] || fail "$name" $rc ;;
    *) echo "unknown step kind '$kind'"; exit 2 ;;
  esac
done
echo "== $(date +%T) done"
