set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6u; mkdir -p $OUT
DIAG=segment-anything-nerf_amd/samnerf_amd/libsamnerf_hip_diag.so
for r in 1 2 3; do
  for S in 1 2; do
    SAMNERF_LIB=$GRAFT_REPO_ROOT/$DIAG SAMNERF_FINAL_S=$S timeout -k 10 120 python bench.py --steps 30 --no-alt --cpu-rays 0 --ref-gpu-rays 0 > $OUT/s${S}_$r.log 2>&1 || { tail -5 $OUT/s${S}_$r.log; exit 1; }
    tail -1 $OUT/s${S}_$r.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('S=$S round $r', round(r['ms_per_step'],4), {k: round(v,4) for k,v in r['stage_ms'].items()}, r['config']['timed_clock_ghz'])"
  done
done
