#!/bin/bash
# Round-6 session: fingerprints of the product against round 5's, the GPU
# tests named in PYTEST_FILES, and an interleaved A/B of the product against
# the libraries in AB_LIBS (under gpurun, from the repo root):
#   TAG=r6b PYTEST_FILES="tests/test_gpu_render.py" AB_LIBS="tools/bin/lib_r5.so" bash tools/gpu_r6.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 240 python tools/lib_bits.py > $OUT/bits_product.json 2> $OUT/bits_product.err
rc=$?; echo "bits rc=$rc"; fatal $rc && exit $rc
python - "$OUT/bits_product.json" profiles/r5f5_lib_bits.json <<'PY'
import json, sys
a, b = (json.load(open(p)) for p in sys.argv[1:3])
print("BITS vs round 5:", "IDENTICAL" if a == b else "DIFFER", {k: (a[k] == b.get(k)) for k in a})
PY
if [ -n "${PYTEST_FILES:-}" ]; then
  timeout -k 10 600 python -u -m pytest $PYTEST_FILES -m gpu -q -p no:cacheprovider -rfE --timeout 120 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $OUT/tests.log | tail -3; fatal $rc && exit $rc
fi
if [ -n "${AB_LIBS:-}" ]; then
  AB_DIR="$OUT/ab" bash tools/ab_libs.sh ${AB_ROUNDS:-3} product $AB_LIBS > $OUT/ab.log 2>&1
  rc=$?; cat $OUT/ab.log; fatal $rc && exit $rc
fi
exit 0
