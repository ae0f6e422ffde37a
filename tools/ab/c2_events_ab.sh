#!/bin/bash
# C2 wall clock with and without a HIP event pair around every K1 launch (A/B, one box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-c2ev}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for ev in 1 0; do
    timeout -k 10 300 env AVDB_BENCH_STAGE_EVENTS=$ev python bench.py --steps 20 --warmup 3 --cpu-baseline off \
        --keyed off > "$OUT/c2_ev${ev}_$rep.json" 2> "$OUT/c2_ev${ev}_$rep.err" || { tail -5 "$OUT/c2_ev${ev}_$rep.err"; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/c2_ev${ev}_$rep.json').read().strip().splitlines()[-1]); print('events=$ev rep $rep', round(d['ms_per_step'], 4), 'ms/step', d['config']['stage_ms'])"
  done
done
