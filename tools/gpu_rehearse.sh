# Rehearsal of the N-rank bench path on a one-GPU box: N processes share GPU 0
# over gloo (RCCL needs one GPU per rank); checks that the multi-rank code
# (row bands, streams, all-gather pipeline, max-over-ranks timing) runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
for n in 2 4; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 6 --warmup 2 --dist-backend gloo --share-gpu > $OUT/rehearse_$n.log 2>&1; rc=$?
echo "N=$n rc=$rc"; grep '^{' $OUT/rehearse_$n.log | tail -1 | cut -c1-400; [ $rc -ne 0 ] && tail -20 $OUT/rehearse_$n.log && exit $rc
done
exit 0
