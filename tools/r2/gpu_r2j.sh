#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for sp in 1 4 8 16; do for m in box corner; do SAMNERF_SGRID_BWD_SPLIT=$sp SAMNERF_SGRID_BWD=$m timeout -k 10 200 python bench.py --mode train --steps 30 --warmup 5 > gpurun_out/r2j_train_${m}_$sp.log 2>&1 || exit $?; python -c "import json;d=json.loads(open('gpurun_out/r2j_train_${m}_$sp.log').read().splitlines()[-1]);print('$m split $sp', round(d['ms_per_step'],3))"; done; done
