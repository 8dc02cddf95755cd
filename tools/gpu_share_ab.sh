# Env-switch A/B on one rank's band of the 512x512 view (bench --rank-share RS): each
# line of $CASES is "<label> <VAR=val ...>".
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
for rs in ${RS:-8 4}; do
while read -r label envs; do
  [ -z "$label" ] && continue
  env $envs timeout -k 10 200 python bench.py --rank-share $rs --streams ${ST:-1} --cpu-rays 0 --ref-gpu-rays 0 --steps 60 --warmup 5 > $OUT/sab_${rs}_$label.log 2>&1 || { echo "$label failed"; tail -5 $OUT/sab_${rs}_$label.log; exit 1; }
  python -c "import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('share', sys.argv[3], sys.argv[2], round(r['ms_per_step'],4), {k: round(v,4) for k,v in r['stage_ms'].items()})" $OUT/sab_${rs}_$label.log $label $rs
done <<< "$CASES"
done
