#!/bin/bash
# One parametrised GPU-box session (replaces round 4's 24 single-use
# tools/gpu_r4*.sh scripts).  usage (under gpurun, from the repo root):
#   TAG=r5a STEPS="smoke tests ab bench prof pmc" bash tools/gpu_run.sh
# STEPS (in this order, any subset):
#   smoke   __graft_entry__.smoke()
#   tests   pytest -m gpu (PYTEST_FILES, PYTEST_K narrow it)
#   ab      tools/ab_libs.sh $AB_ROUNDS $AB_LIBS (interleaved library A/B on the headline view)
#   bench   python bench.py $BENCH_ARGS (the driver's default line unless set)
#   share   bench.py --rank-share $SHARE_N (8) at $SHARE_STREAMS (1 2 3) streams
#   surface bench.py --scene surface (the opaque-sphere headline)
#   prof    rocprofv3 --kernel-trace --stats of the headline (bench.py --no-alt --streams 1)
#   pmc     tools/pmc_passes.sh (PASSES selects counter groups)
# Logs go to gpurun_out/$TAG/.  Every GPU step runs under its own time limit;
# a fault, abort, segfault or time-out (rc 124/134/137/139) ends the session.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-run}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
has() { [[ " ${STEPS:-smoke tests bench} " == *" $1 "* ]]; }
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
step() {   # step NAME SECONDS CMD... : run, report, stop the session on a fatal rc
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; fi
  if fatal $rc; then echo "FATAL in $name"; exit $rc; fi
  return $rc
}
if has smoke; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if has tests; then
  step tests 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -q ${PYTEST_K:+-k "$PYTEST_K"} \
    -p no:cacheprovider -rfE --timeout 120 --timeout-method thread --durations=15 ${PYTEST_ARGS:-}
  rc=$?
  grep -E "passed|failed" "$OUT/tests.log" | tail -3
  [ $rc -ne 0 ] && [ "${KEEP_GOING:-0}" != "1" ] && exit $rc
fi
if has ab; then
  AB_DIR="$OUT" bash tools/ab_libs.sh ${AB_ROUNDS:-3} ${AB_LIBS:-product} > "$OUT/ab.log" 2>&1
  rc=$?; cat "$OUT/ab.log"; fatal $rc && exit $rc
fi
if has bench; then
  step bench 400 python bench.py ${BENCH_ARGS:-} || exit 1
  tail -1 "$OUT/bench.log" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], {k: round(v, 4) for k, v in r['stage_ms'].items()})"
fi
if has share; then   # one rank's band of the N = 8 split on this GPU, 1-3 streams
  for s in ${SHARE_STREAMS:-1 2 3}; do
    step share_s$s 200 python bench.py --rank-share ${SHARE_N:-8} --streams $s --no-alt --steps 60 --warmup 5 \
      --cpu-rays 0 --ref-gpu-rays 0 || exit 1
    tail -1 "$OUT/share_s$s.log" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('streams $s', r['ms_per_step'], {k: round(v, 4) for k, v in r['stage_ms'].items()})"
  done
fi
if has surface; then
  step surface 200 python bench.py --scene surface --no-alt --cpu-rays 0 --ref-gpu-rays 0 || exit 1
  tail -1 "$OUT/surface.log" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('surface', r['ms_per_step'], {k: round(v, 4) for k, v in r['stage_ms'].items()})"
fi
if has prof; then
  cd /tmp && export TMPDIR=/tmp
  step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-alt --streams 1 --steps 20 --warmup 3 --cpu-rays 0 --ref-gpu-rays 0 ${PROF_ARGS:-} || exit 1
  cd "$GRAFT_REPO_ROOT"
  python3 -c "
import csv, glob, sys
f = sorted(glob.glob('$OUT/trace/**/*kernel_stats.csv', recursive=True))
rows = list(csv.DictReader(open(f[0]))) if f else []
for r in rows[:14]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
"
fi
if has pmc; then
  bash tools/pmc_passes.sh "$TAG" ${PMC_ARGS:-} > "$OUT/pmc.log" 2>&1
  rc=$?; tail -30 "$OUT/pmc.log"; fatal $rc && exit $rc
fi
exit 0
