# One rank's share of a strong-scaled view: stream sweep + kernel trace at H=64.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
for h in ${HS:-64 128}; do for st in ${STS:-1 3 4 6}; do
timeout -k 10 200 python bench.py --H $h --streams $st --cpu-rays 0 --ref-gpu-rays 0 --steps 40 > $OUT/st_${st}_$h.log 2>&1 || exit $?
python -c "import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('H', sys.argv[3], 'streams', sys.argv[2], round(r['ms_per_step'],3), round(r['value']/1e6,2), 'Mrays/s', {k: round(v,3) for k,v in r['stage_ms'].items()})" $OUT/st_${st}_$h.log $st $h
done; done
[ "${PROF:-1}" = "1" ] && bash tools/prof_small.sh 64
exit 0
