#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do for v in default kpre0; do
  if [ $v = default ]; then unset SAMNERF_LIB; else export SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/diag/lib/$v.so; fi
  timeout -k 10 200 python bench.py --no-alt --cpu-rays 0 --ref-gpu-rays 0 --steps 30 --streams 1 > gpurun_out/r2g_$v.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/r2g_$v.log').read().splitlines()[-1]);print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stage_ms'].items()})"
done; done
unset SAMNERF_LIB
for n in 70000 40000; do SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/diag/lib/kpre0.so timeout -k 10 200 python tools/diag/final_determinism.py $n > gpurun_out/r2g_det_$n.log 2>&1 || exit $?; echo "kpre0 n=$n"; grep -E "repeat|rows" gpurun_out/r2g_det_$n.log; done
