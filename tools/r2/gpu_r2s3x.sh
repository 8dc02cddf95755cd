#!/bin/bash
# N>1 rehearsal on the one-GPU box (two ranks sharing GPU 0, gloo): the launcher and the sharded path still run
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --dist-backend gloo --steps 5 --warmup 2 > gpurun_out/r2s3x_rehearse.log 2>&1 || { tail -20 gpurun_out/r2s3x_rehearse.log; exit 1; }
tail -1 gpurun_out/r2s3x_rehearse.log | cut -c1-300
