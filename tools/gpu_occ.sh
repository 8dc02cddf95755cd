set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "train or variants" > $OUT/pytest_sel.log 2>&1; echo "pytest rc=$?"; tail -3 $OUT/pytest_sel.log
for o in 1 5 6; do for h in 512 64; do
SAMNERF_PROP_OCC=$o timeout -k 10 200 python bench.py --H $h --cpu-rays 0 --ref-gpu-rays 0 --steps 30 > $OUT/occ_${o}_$h.log 2>&1 || exit $?
python -c "import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], round(r['ms_per_step'],3), {k: round(v,3) for k,v in r['stage_ms'].items()})" $OUT/occ_${o}_$h.log $o $h
done; done
timeout -k 10 300 python bench.py --cpu-rays 0 > $OUT/bench_full.log 2>&1; echo "full rc=$?"; tail -1 $OUT/bench_full.log
