# Env-switch A/B at one rank's share of a view: each line of $CASES is
# "<label> <VAR=val ...>", run as bench.py --H $H --streams $ST.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
H=${H:-64}; ST=${ST:-3}
while read -r label envs; do
  [ -z "$label" ] && continue
  env $envs timeout -k 10 200 python bench.py --H $H --streams $ST --cpu-rays 0 --ref-gpu-rays 0 --steps 60 --warmup 5 > $OUT/ab_$label.log 2>&1 || { echo "$label failed"; tail -5 $OUT/ab_$label.log; exit 1; }
  python -c "import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(r['ms_per_step'],3), round(r['value']/1e6,2), 'Mrays/s', {k: round(v,3) for k,v in r['stage_ms'].items()})" $OUT/ab_$label.log $label
done <<< "$CASES"
