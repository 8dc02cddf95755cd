# One rank's band of the 512x512 view at N = 2 / 4 / 8 ranks, 1-3 HIP streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
for rs in 2 4 8; do for st in 1 2 3; do
timeout -k 10 200 python bench.py --rank-share $rs --streams $st --cpu-rays 0 --ref-gpu-rays 0 --steps 60 --warmup 5 > $OUT/ss_${rs}_$st.log 2>&1 || exit $?
python -c "import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('share', sys.argv[2], 'streams', sys.argv[3], round(r['ms_per_step'],4))" $OUT/ss_${rs}_$st.log $rs $st
done; done
