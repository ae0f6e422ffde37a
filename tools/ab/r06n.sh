#!/bin/bash
# Round 6: C1 (one HIP graph) in the serial and the one-pass layout, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06n; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2 3; do
for lay in serial onepass; do
  timeout -k 10 300 env AVDB_BENCH_LAYOUT=$lay python bench.py --steps 200 --warmup 20 --cpu-baseline off --workload c1 > "$OUT/bench_c1_$lay.log" 2>&1 || exit $?
  python - "$OUT/bench_c1_$lay.log" "c1 $lay" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,4) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
done; done
