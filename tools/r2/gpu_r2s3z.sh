#!/bin/bash
# Round-2 (third session) evidence for HEAD: smoke, the full -m gpu suite, the
# default bench line, its kernel-trace stats and the PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-r2s3z}
timeout -k 10 600 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed" gpurun_out/${T}_tests.log | cut -c1-300 | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log > gpurun_out/${T}_bench.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${T}" -o trace -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --cpu-rays 0 --ref-gpu-rays 0 --no-alt --streams 1 > "$GRAFT_REPO_ROOT/gpurun_out/${T}_trace.log" 2>&1 || { echo trace failed; exit 1; }
cd "$GRAFT_REPO_ROOT"
bash tools/pmc_r2.sh ${T} > gpurun_out/${T}_pmc.log 2>&1 || { tail -20 gpurun_out/${T}_pmc.log; exit 1; }
echo ok
