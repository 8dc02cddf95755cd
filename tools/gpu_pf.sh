set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "prefetch or variants or golden or segment" > $OUT/pytest_pf.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_pf.log; [ $rc -ne 0 ] && exit $rc
for h in 512 64; do for pf in 0 1; do
SAMNERF_FINAL_PF=$pf timeout -k 10 200 python bench.py --H $h --cpu-rays 0 --ref-gpu-rays 0 --steps 30 > $OUT/pf_${pf}_$h.log 2>&1 || exit $?
python -c "import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('H', sys.argv[3], 'PF', sys.argv[2], round(r['ms_per_step'],3), {k: round(v,3) for k,v in r['stage_ms'].items()})" $OUT/pf_${pf}_$h.log $pf $h
done; done
