set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6f; mkdir -p $OUT
timeout -k 10 200 python -u tools/host_overhead.py > $OUT/host.log 2>&1; rc=$?; grep '^{' $OUT/host.log; [ $rc -ne 0 ] && { tail -20 $OUT/host.log; exit $rc; }
timeout -k 10 300 python -u tools/graph_view.py > $OUT/graph.log 2>&1; rc=$?; grep '^{' $OUT/graph.log; [ $rc -ne 0 ] && { tail -30 $OUT/graph.log; exit $rc; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); c=r['config']; print(round(r['ms_per_step'],4), c['views_in_flight'], c['views_in_flight_tuned_ms'], c['views_in_flight_tuned_clock_ghz'], c['timed_clock_ghz'])"
