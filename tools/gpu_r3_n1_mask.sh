timeout -k 10 300 python -u -m pytest tests/test_gpu_n1.py tests/test_gpu_mask_train.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -ge 124 ] && exit $rc
bash tools/n1_prof.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/mt -o t -- python3 $GRAFT_REPO_ROOT/tools/mask_train_prof.py > $GRAFT_REPO_ROOT/gpurun_out/mt.log 2>&1 || exit $?
tail -1 $GRAFT_REPO_ROOT/gpurun_out/mt.log; head -14 $GRAFT_REPO_ROOT/gpurun_out/mt/*kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/mtt -o t -- python3 $GRAFT_REPO_ROOT/tools/mask_train_prof.py torch > $GRAFT_REPO_ROOT/gpurun_out/mtt.log 2>&1 || exit $?
tail -1 $GRAFT_REPO_ROOT/gpurun_out/mtt.log; head -8 $GRAFT_REPO_ROOT/gpurun_out/mtt/*kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
