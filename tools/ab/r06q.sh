#!/bin/bash
# Round 6: C1 graph with K7's write-pass grid capped (AVDB_BENCH_K7_GRID -> AVDB_OPT_K7_GRID):
# 17 K one-tile groups at the default grid, several tiles per wave when capped.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06q; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for g in 0 8192 4096 2048; do
  timeout -k 10 300 env AVDB_BENCH_K7_GRID=$g python bench.py --steps 200 --warmup 20 --cpu-baseline off --workload c1 > "$OUT/bench_c1_g$g.log" 2>&1 || exit $?
  python - "$OUT/bench_c1_g$g.log" "c1 k7grid=$g" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,4) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
done; done
