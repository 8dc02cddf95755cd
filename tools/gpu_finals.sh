set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
for h in 64 128 512; do for sg in 1 2 4; do
SAMNERF_FINAL_S=$sg timeout -k 10 200 python bench.py --H $h --cpu-rays 0 --ref-gpu-rays 0 --steps 30 > $OUT/fs_${sg}_$h.log 2>&1 || exit $?
python -c "import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('H', sys.argv[3], 'S', sys.argv[2], round(r['ms_per_step'],3), {k: round(v,3) for k,v in r['stage_ms'].items()})" $OUT/fs_${sg}_$h.log $sg $h
done; done
