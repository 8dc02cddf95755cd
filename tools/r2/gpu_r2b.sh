#!/bin/bash
# round 2: full GPU suite, bench, kernel-trace stats, PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r2b_tests.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/r2b_tests.log | tail -5
[ $rc -ne 0 ] && { tail -40 gpurun_out/r2b_tests.log; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/r2b_bench.log 2>&1; rc=$?
tail -c 1500 gpurun_out/r2b_bench.log
[ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/r2_counters.txt" 2>&1); echo "list rc=$?"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2b" -o r2b -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --cpu-rays 0 --ref-gpu-rays 0 --no-alt > "$GRAFT_REPO_ROOT/gpurun_out/r2b_prof.log" 2>&1; rc=$?
echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
bash "$GRAFT_REPO_ROOT/tools/pmc_r2.sh" r2b
