#!/bin/bash
# GPU-box check: build, smoke, parity tests, bench, rocprofv3 trace + PMC passes.
# Every GPU step has its own time limit; a crash/timeout stops the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
stop_if_fatal() {  # $1 = rc, $2 = step
  if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then echo "FATAL rc=$1 in $2"; exit "$1"; fi
}
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { echo BUILD FAIL; tail -30 "$OUT/build.log"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; stop_if_fatal $rc smoke
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -q ${PYTEST_K:+-k "$PYTEST_K"} -p no:cacheprovider -rA --timeout 120 --timeout-method thread --durations=25 > "$OUT/pytest_gpu.log" 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" "$OUT/pytest_gpu.log" | tail -15; stop_if_fatal $rc pytest
fi
if [ "${RUN_TA:-0}" = "1" ]; then
timeout -k 10 120 tools/bin/ta_rate > "$OUT/ta_rate.json" 2> "$OUT/ta_rate.err"; rc=$?; echo "ta_rate rc=$rc"; cat "$OUT/ta_rate.json"; stop_if_fatal $rc ta_rate
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 "$OUT/bench.log"; stop_if_fatal $rc bench
fi
# per-rank loads of an N-GPU strong-scaled 512x512 view: H = 512/N rows
for h in ${SWEEP_H:-}; do
timeout -k 10 200 python bench.py --H $h --cpu-rays 0 --steps 20 > "$OUT/bench_h$h.log" 2>&1; rc=$?; echo "bench H=$h rc=$rc"; tail -1 "$OUT/bench_h$h.log" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], {k: round(v,3) for k,v in r['stage_ms'].items()})"; stop_if_fatal $rc bench_h$h
done
if [ "${SKIP_PROF:-0}" != "1" ]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_trace" -o trace -- python "$GRAFT_REPO_ROOT/bench.py" --streams 1 --steps 5 --warmup 2 --cpu-rays 0 > "$OUT/prof_trace.log" 2>&1; rc=$?; echo "prof trace rc=$rc"; stop_if_fatal $rc prof_trace
[ "${TRACE_ONLY:-0}" = "1" ] && exit 0
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/prof_fetch" -o fetch -- python "$GRAFT_REPO_ROOT/bench.py" --streams 1 --steps 3 --warmup 1 --cpu-rays 0 > "$OUT/prof_fetch.log" 2>&1; rc=$?; echo "prof fetch rc=$rc"; stop_if_fatal $rc prof_fetch
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/prof_write" -o write -- python "$GRAFT_REPO_ROOT/bench.py" --streams 1 --steps 3 --warmup 1 --cpu-rays 0 > "$OUT/prof_write.log" 2>&1; rc=$?; echo "prof write rc=$rc"; stop_if_fatal $rc prof_write
fi
find "$OUT" -name "*.csv" | head -20
