cd $GRAFT_REPO_ROOT
for n in 70000 40000 9000; do timeout -k 10 200 python tools/diag/final_determinism.py $n > gpurun_out/det_$n.log 2>&1 || exit $?; echo "n=$n"; grep -E "repeat|image" gpurun_out/det_$n.log; done
