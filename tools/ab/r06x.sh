#!/bin/bash
# Round 6: C1 graph with the keyed K2's grid at 4 (default) / 5 / 8 workgroups per CU
# (AVDB_K2_BLOCKS_PER_CU): 1.1 M records are 1,074 workgroup-trips, one more than 4 x 256.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06x; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for k in 4 5 8; do
  timeout -k 10 300 env AVDB_K2_BLOCKS_PER_CU=$k python bench.py --steps 200 --warmup 20 --cpu-baseline off --workload c1 > "$OUT/bench_c1_k$k.log" 2>&1 || exit $?
  python - "$OUT/bench_c1_k$k.log" "c1 k2/cu=$k" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,4) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
done; done
