#!/bin/bash
# Bench several builds of libsamnerf_hip.so in one GPU session, interleaved.
#   LIBS="label=path label2=path2"  (the in-tree build is always "cur")
#   env: ROUNDS=2  BENCH_ARGS="--steps 20"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
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
for i in $(seq ${ROUNDS:-2}); do
  for e in cur ${LIBS:-}; do
    label=${e%%=*}; lib=""; [ "$e" != cur ] && lib="$GRAFT_REPO_ROOT/${e#*=}"
    SAMNERF_LIB="$lib" timeout -k 10 300 python bench.py --cpu-rays 0 --ref-gpu-rays 0 ${BENCH_ARGS:---steps 20} > "$OUT/libs_${label}_$i.log" 2>&1
    rc=$?; echo "bench $label #$i rc=$rc"; summ "$OUT/libs_${label}_$i.log"; fatal $rc && exit $rc
  done
done
exit 0
