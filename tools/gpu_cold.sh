#!/bin/bash
# the removed k_final prefetch form's first-render
# difference, reproduced under forced-cold caches (tools/cold_render_check.py)
# for the round-4 builds of that form and for the product.  Libraries (built
# from git b7fed49^, the last tree with the form, -DSAMNERF_DIAG_VARIANTS):
#   tools/bin/lib_oldpf.so        as round 4 had it
#   tools/bin/lib_oldpf_noasm.so  + -DSAMNERF_F16X3_NOASM (split8_f16 without inline asm)
#   tools/bin/lib_oldpf_wz.so     + -mllvm -amdgpu-waitcnt-forcezero
#   tools/bin/lib_oldpf_w1.so     + s_waitcnt vmcnt(0) right after the next sample's gathers are issued
#   tools/bin/lib_oldpf_w2.so     + s_waitcnt vmcnt(0) after layers 2-3 (before the composite)
# usage (GPU box): RUNS="product oldpf_pf1 ..." bash tools/gpu_cold.sh [REPS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/cold"
mkdir -p "$OUT"
REPS=${1:-12}
run() {   # tag lib args...
  local tag=$1 lib=$2; shift 2
  if [ "$lib" = product ]; then unset SAMNERF_LIB; else export SAMNERF_LIB="$GRAFT_REPO_ROOT/$lib"; fi
  timeout -k 10 200 python tools/cold_render_check.py --reps $REPS "$@" > "$OUT/$tag.log" 2>&1
  local rc=$?
  echo "$tag rc=$rc: $(grep SUMMARY "$OUT/$tag.log")"
  grep -A1 DIFFERS "$OUT/$tag.log" | head -6
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
PF1="--env SAMNERF_FINAL_PF=1 --ref-env SAMNERF_FINAL_PF=0"
for r in ${RUNS:-product product_tiled oldpf_pf1 oldpf_pf0 oldpf_pf1_noasm oldpf_pf1_warm}; do
  case $r in
    product) run $r product || exit 1 ;;
    product_tiled) run $r product --view-width 512 || exit 1 ;;
    oldpf_pf1) run $r tools/bin/lib_oldpf.so $PF1 || exit 1 ;;
    oldpf_pf1_taps) run $r tools/bin/lib_oldpf.so $PF1 --taps || exit 1 ;;
    oldpf_pf0) run $r tools/bin/lib_oldpf.so --env SAMNERF_FINAL_PF=0 || exit 1 ;;
    oldpf_pf1_noasm) run $r tools/bin/lib_oldpf_noasm.so $PF1 || exit 1 ;;
    oldpf_pf1_wz) run $r tools/bin/lib_oldpf_wz.so $PF1 || exit 1 ;;
    oldpf_pf1_w1) run $r tools/bin/lib_oldpf_w1.so $PF1 || exit 1 ;;
    oldpf_pf1_w2) run $r tools/bin/lib_oldpf_w2.so $PF1 || exit 1 ;;
    oldpf_pf1_warm) run $r tools/bin/lib_oldpf.so --no-cold $PF1 || exit 1 ;;
  esac
done
exit 0
