#!/bin/bash
# GPU-box session: smoke, parity tests, bench of each gather variant
# (SAMNERF_LOOKUP = packed | ref | box), a kernel-trace profile and PMC passes.
# Every GPU step has its own time limit; a crash / timeout ends the script.
#   env: MODES="packed ref box"  SKIP_TESTS=1  SKIP_PMC=1  SWEEP_H="64 128"
#        TEST_K=<pytest -k expr>  PROF_MODE=<mode for the profiles>
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

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; fatal $rc && exit $rc

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider ${TEST_K:+-k "$TEST_K"} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" "$OUT/pytest_gpu.log" | tail -12
  fatal $rc && exit $rc
fi

lk() { [ "$1" = "default" ] && echo "" || echo "$1"; }
for m in ${MODES:-default packed ref box4}; do
  SAMNERF_LOOKUP=$(lk $m) timeout -k 10 300 python bench.py --cpu-rays 0 --ref-gpu-rays 0 --steps 20 > "$OUT/bench_$m.log" 2>&1
  rc=$?; echo "bench $m rc=$rc"; summ "$OUT/bench_$m.log"; fatal $rc && exit $rc
  for h in ${SWEEP_H:-}; do
    SAMNERF_LOOKUP=$(lk $m) timeout -k 10 200 python bench.py --H $h --cpu-rays 0 --ref-gpu-rays 0 --steps 30 > "$OUT/bench_${m}_h$h.log" 2>&1
    rc=$?; echo "bench $m H=$h rc=$rc"; summ "$OUT/bench_${m}_h$h.log"; fatal $rc && exit $rc
  done
done

[ "${SKIP_PROF:-0}" = "1" ] && exit 0
export SAMNERF_LOOKUP=$(lk ${PROF_MODE:-default})
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_trace" -o trace \
  -- python "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --cpu-rays 0 --ref-gpu-rays 0 > "$OUT/prof_trace.log" 2>&1
rc=$?; echo "prof trace rc=$rc"; fatal $rc && exit $rc
[ "${SKIP_PMC:-0}" = "1" ] && exit 0
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/pmc_avail.txt" 2>&1; echo "list-avail rc=$?"
GROUPS_=(
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
  "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for g in "${GROUPS_[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/pmc/p$i" -o p$i \
    -- python "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --cpu-rays 0 --ref-gpu-rays 0 > "$OUT/pmc_p$i.log" 2>&1
  rc=$?; echo "pmc pass $i rc=$rc ($g)"
  if fatal $rc; then break; fi
  i=$((i+1))
done
python "$GRAFT_REPO_ROOT/tools/pmc_table.py" "$OUT/pmc" > "$OUT/pmc_table.txt" 2>&1
head -40 "$OUT/pmc_table.txt"
