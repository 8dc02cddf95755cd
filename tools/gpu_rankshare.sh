set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
for rs in 8 4; do for st in 1 3; do
timeout -k 10 200 python bench.py --rank-share $rs --streams $st --cpu-rays 0 --ref-gpu-rays 0 --steps 40 > $OUT/rs_${rs}_${st}.log 2>&1 || exit $?
python -c "import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('share', sys.argv[3], 'streams', sys.argv[2], round(r['ms_per_step'],3), round(r['value']/1e6,2), 'Mrays/s', {k: round(v,3) for k,v in r['stage_ms'].items()})" $OUT/rs_${rs}_${st}.log $st $rs
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_rs8" -o trace -- python "$GRAFT_REPO_ROOT/bench.py" --rank-share 8 --streams 1 --steps 20 --warmup 3 --cpu-rays 0 --ref-gpu-rays 0 > "$GRAFT_REPO_ROOT/$OUT/prof_rs8.log" 2>&1
