set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/ab_gnfa; mkdir -p $O
export IRX_PROF_TOP=80
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/def_$r.json 2> $O/def_$r.err || exit $?
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --opt gn_fa=1073741824 > $O/vae_$r.json 2> $O/vae_$r.err || exit $?
done
for f in $O/*.json; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'])" $f; grep -E "gn_fa|gn_apply|gn_finalize" ${f%.json}.err; done
