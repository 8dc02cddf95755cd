# Transport codec: GPU tests, kernel timing, multi-rank rehearsal (gloo ranks sharing GPU 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_tile_codec.py tests/test_capi.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/codec_tests.log 2>&1; rc=$?; tail -8 $OUT/codec_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/codec_time.py > $OUT/codec_time.json 2> $OUT/codec_time.err || { tail -5 $OUT/codec_time.err; exit 1; }
cat $OUT/codec_time.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29508 bench.py --gpus 8 --steps 6 --warmup 2 --dist-backend gloo --share-gpu > $OUT/rehearse_q16.log 2>&1; rc=$?
echo "N=8 q16 rc=$rc"; grep '^{' $OUT/rehearse_q16.log | tail -1 | cut -c1-700; [ $rc -ne 0 ] && tail -20 $OUT/rehearse_q16.log
exit $rc
