cd "$GRAFT_REPO_ROOT" && MODES=default bash tools/gpu_ab.sh > gpurun_out/ab_full.txt 2>&1; rc=$?; tail -40 gpurun_out/ab_full.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_official.log 2>&1; rc=$?; tail -2 gpurun_out/bench_official.log; exit $rc
