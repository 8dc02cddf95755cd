cd /tmp && export TMPDIR=/tmp
for c in 1 2 4; do
SAMNERF_N1_CHUNKS=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/n1c$c -o t -- python3 $GRAFT_REPO_ROOT/tools/n1_prof.py > $GRAFT_REPO_ROOT/gpurun_out/n1c$c.log 2>&1 || exit $?
echo "chunks $c"; grep -h -E "k_final|k_n1|k_sgrid" $GRAFT_REPO_ROOT/gpurun_out/n1c$c/*kernel_stats.csv | awk -F'",' '{print $1}' | cut -c1-90 | paste - <(grep -h -E "k_final|k_n1|k_sgrid" $GRAFT_REPO_ROOT/gpurun_out/n1c$c/*kernel_stats.csv | awk -F, '{print $(NF-6), $(NF-5)}')
done
