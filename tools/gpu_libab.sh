#!/bin/bash
# Bench two builds of libsamnerf_hip.so in one GPU session, interleaved:
# $AB_OLD (default ab_old/libsamnerf_hip.so) vs the in-tree build.
#   env: ROUNDS=2  BENCH_ARGS="--steps 20"  TEST_K=<pytest -k expr, run first>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
OLD="${AB_OLD:-$GRAFT_REPO_ROOT/ab_old/libsamnerf_hip.so}"
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
summ() {
  python -c "
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
r = json.loads(line)
print('   value %.4g rays/s  %.3f ms/step  ' % (r['value'], r['ms_per_step']),
      {k: round(v, 3) for k, v in r.get('stage_ms', {}).items()})
" "$1" || tail -3 "$1"
}
if [ -n "${TEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "$TEST_K" > "$OUT/pytest_ab.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" "$OUT/pytest_ab.log" | tail -12
  fatal $rc && exit $rc
fi
for i in $(seq ${ROUNDS:-2}); do
  for v in old new; do
    lib=""; [ $v = old ] && lib="$OLD"
    SAMNERF_LIB="$lib" timeout -k 10 300 python bench.py --cpu-rays 0 --ref-gpu-rays 0 ${BENCH_ARGS:---steps 20} > "$OUT/ab_${v}_$i.log" 2>&1
    rc=$?; echo "bench $v #$i rc=$rc"; summ "$OUT/ab_${v}_$i.log"; fatal $rc && exit $rc
  done
done
exit 0
