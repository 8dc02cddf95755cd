#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-alt --cpu-rays 0 --ref-gpu-rays 0 --steps 30 "$@" > gpurun_out/r2l.log 2>&1 || exit $?; python -c "import json;d=json.loads(open('gpurun_out/r2l.log').read().splitlines()[-1]);print('$tag', round(d['value']/1e6,2), round(d['ms_per_step'],3), {k: round(v,4) for k,v in d['stage_ms'].items()})"; }
for rep in 1 2; do
tag=default; unset SAMNERF_LIB; run
tag=sg4; export SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/diag/lib/sg4.so; run
tag=sg4_share8; run --rank-share 8
tag=default_share8; unset SAMNERF_LIB; run --rank-share 8
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_render.py > gpurun_out/r2l_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r2l_tests.log; exit $rc
