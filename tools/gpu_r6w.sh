set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6w; mkdir -p $OUT
timeout -k 10 400 python bench.py --gpus 2 --share-gpu --dist-backend gloo --steps 10 --warmup 3 > $OUT/bench_n2.log 2>&1; rc=$?
tail -3 $OUT/bench_n2.log | cut -c1-600; exit $rc
