set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6x; mkdir -p $OUT
TAG=r6x STEPS="smoke tests bench" BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_run.sh || exit $?
