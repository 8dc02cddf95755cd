set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6k; mkdir -p $OUT
for r in 1 2 3; do
  for s in 2 3 4; do
    timeout -k 10 120 python bench.py --steps 30 --no-alt --cpu-rays 0 --ref-gpu-rays 0 --streams $s > $OUT/s${s}_$r.log 2>&1 || { tail -5 $OUT/s${s}_$r.log; exit 1; }
    tail -1 $OUT/s${s}_$r.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); c=r['config']; print('streams $s round $r', round(r['ms_per_step'],4), 'clock', c['timed_clock_ghz'])"
  done
done
