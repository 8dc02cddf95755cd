set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6d; mkdir -p $OUT
TAG=r6d STEPS="tests" PYTEST_FILES="tests/test_gpu_n1.py tests/test_gpu_rgb_train.py tests/test_gpu_render.py" bash tools/gpu_run.sh || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.log 2>&1 || { echo "bench $i failed"; tail -5 $OUT/bench_$i.log; exit 1; }
  tail -1 $OUT/bench_$i.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('bench', $i, round(r['ms_per_step'],4), r['config']['views_in_flight'], r['config']['views_in_flight_tuned_ms'], r['config']['timed_clock_ghz'], {k: round(v,4) for k,v in r['stage_ms'].items()})"
done
AB_DIR=$OUT/ab bash tools/ab_libs.sh 3 product tools/bin/lib_w8a.so tools/bin/lib_w8b.so > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; [ $rc -ge 124 ] && exit $rc
bash tools/pmc_cfg5.sh r6d_cfg5 || exit $?
TAG=r6d STEPS="share" SHARE_STREAMS="1 2 3" bash tools/gpu_run.sh
