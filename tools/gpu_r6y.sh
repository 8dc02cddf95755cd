set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6y; mkdir -p $OUT
TAG=r6y STEPS="smoke tests bench surface prof pmc" BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_run.sh || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench2.log 2>&1 || { tail -5 $OUT/bench2.log; exit 1; }
tail -1 $OUT/bench2.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); c=r['config']; print('bench2', round(r['ms_per_step'],4), c['views_in_flight'], c['views_in_flight_tuned_ms'], c['views_in_flight_tuned_clock_ghz'], c['timed_clock_ghz'], r['mask_default_head']['ms_per_step'])"
