#!/bin/bash
# kernel trace of the 2-stream headline (does view i+1 overlap view i?) + the
# head without its weight DMA (diagnostic form 11)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ov -o t -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-rays 0 --ref-gpu-rays 0 --no-alt > $OUT/ov.log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/overlap.py $OUT/ov/t_kernel_trace.csv | head -20
cd $GRAFT_REPO_ROOT && HEAD_VARIANTS=${HEAD_VARIANTS:-4,11} bash tools/gpu_head.sh
