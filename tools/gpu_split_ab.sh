set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5sp
timeout -k 10 120 tools/bin/valu_rate > gpurun_out/r5sp/valu_rate3.json &&
timeout -k 10 240 python tools/lib_bits.py > gpurun_out/r5sp/bits_new.json 2> gpurun_out/r5sp/bits_new.err &&
SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/bin/lib_mix.so timeout -k 10 240 python tools/lib_bits.py > gpurun_out/r5sp/bits_mix.json 2> gpurun_out/r5sp/bits_mix.err &&
cat gpurun_out/r5sp/bits_new.json gpurun_out/r5sp/bits_mix.json &&
AB_ROUNDS=3 bash tools/ab_scenes.sh product tools/bin/lib_mix.so > gpurun_out/r5sp/ab_scenes.txt 2>&1 &&
bash tools/ab_mask.sh 2 product tools/bin/lib_mix.so > gpurun_out/r5sp/ab_mask.txt 2>&1
