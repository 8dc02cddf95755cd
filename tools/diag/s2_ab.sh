cd $GRAFT_REPO_ROOT
for h in 64 128; do
for cfg in "head::" "allS:0:1" "allS:1:1" "allS:0:0" "allS:1:0"; do
  IFS=: read lib pf cl <<< "$cfg"
  L=""; [ "$lib" = allS ] && L=$GRAFT_REPO_ROOT/diag/lib_allS.so
  SAMNERF_LIB="$L" SAMNERF_FINAL_PF="$pf" SAMNERF_FINAL_CLASSES="$cl" timeout -k 10 120 python bench.py --H $h --cpu-rays 0 --ref-gpu-rays 0 --steps 30 > gpurun_out/s2_$h.log 2>&1 || exit $?
  python -c "
import json,sys; r=[json.loads(l) for l in open('gpurun_out/s2_$h.log') if l.startswith('{')][-1]; print('H=$h $cfg', round(r['stage_ms']['final'],4), round(r['ms_per_step'],3))"
done; done
