#!/bin/bash
# Views in flight on 1 / 2 / 3 HIP streams (bench.py --streams), on the full
# view and on one rank's band of the N = 2 / 4 / 8 split (--rank-share),
# interleaved.  usage (GPU box): [SHARES="1 2 4 8"] [ROUNDS=2] bash tools/streams_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/streams"
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do
  for n in ${SHARES:-1 2 4 8}; do
    for s in 1 2 3; do
      share=""; [ "$n" != 1 ] && share="--rank-share $n"
      timeout -k 10 120 python bench.py --steps 60 --no-alt --cpu-rays 0 --ref-gpu-rays 0 --streams $s $share \
        > "$OUT/n${n}_s${s}_$r.log" 2>&1 || exit 1
      tail -1 "$OUT/n${n}_s${s}_$r.log" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('share $n streams $s', round(r['ms_per_step'],4))"
    done
  done
done
