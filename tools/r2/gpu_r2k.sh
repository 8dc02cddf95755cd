#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-alt --cpu-rays 0 --ref-gpu-rays 0 --steps 30 --streams 1 "$@" > gpurun_out/r2k.log 2>&1 || exit $?; python -c "import json;d=json.loads(open('gpurun_out/r2k.log').read().splitlines()[-1]);print('$tag', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(d['stage_ms']['final'],4))"; }
tag=default; unset SAMNERF_LIB SAMNERF_FINAL_PF; run
tag=default_nopf; export SAMNERF_FINAL_PF=0; run
tag=w3_nopf; export SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/diag/lib/w3.so; run
tag=w3_nopf_share8; run --rank-share 8
tag=default_share8; unset SAMNERF_LIB SAMNERF_FINAL_PF; run --rank-share 8
