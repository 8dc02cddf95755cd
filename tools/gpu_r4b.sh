#!/bin/bash
# Round-4 batch: (1) the k_final prefetch forms' determinism with the inline-asm
# f16x3 split (in-tree diagnostic build) and with the plain-C split
# (tools/bin/lib_dnoasm.so in its place); (2) interleaved A/B timing of the
# candidate builds (mask head LDS-DMA weight ring, view weights from L2 at 3 /
# 4 waves per SIMD) and the mask head's attribution builds.  A test assertion
# does not stop the batch; a time limit or crash does.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
K="final_forms_deterministic or slot_classes"
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -k "$K" -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_pf_asm.log 2>&1
rc=$?; echo "pf asm rc=$rc"; tail -1 $OUT/pytest_pf_asm.log; [ $rc -gt 1 ] && exit $rc
cp tools/bin/lib_dnoasm.so segment-anything-nerf_amd/samnerf_amd/libsamnerf_hip_diag.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -k "$K" -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_pf_noasm.log 2>&1
rc=$?; echo "pf noasm rc=$rc"; tail -1 $OUT/pytest_pf_noasm.log; [ $rc -gt 1 ] && exit $rc
bash tools/ab_mask.sh 2 tools/bin/lib_copies.so tools/bin/lib_mr3.so tools/bin/lib_mr5.so || exit $?
bash tools/ab_mask.sh 1 tools/bin/lib_mnog.so tools/bin/lib_mnow.so tools/bin/lib_mnos.so tools/bin/lib_sgdma.so || exit $?
bash tools/ab_libs.sh 2 tools/bin/lib_sgdma.so tools/bin/lib_copies.so tools/bin/lib_vg3.so tools/bin/lib_vg4.so || exit $?
