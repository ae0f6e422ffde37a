#!/bin/bash
# C1 step forms on one box: the graph (fork / serial layout) and plain launches,
# 10 and 50 timed steps.  tools/ab/c1_ab.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-c1ab}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for rep in 1 2; do
  for cfg in "fork:auto:10" "fork:auto:50" "serial:auto:50" "fork:off:50"; do
    IFS=: read lay gr st <<< "$cfg"
    AVDB_BENCH_LAYOUT=$lay timeout -k 10 200 python bench.py --workload c1 --steps $st --warmup 3 --graph $gr \
      --cpu-baseline off > "$OUT/c1_${lay}_${gr}_${st}_$rep.json" 2>&1 || { tail -5 "$OUT/c1_${lay}_${gr}_${st}_$rep.json"; exit 1; }
    python3 - "$OUT/c1_${lay}_${gr}_${st}_$rep.json" "$cfg" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
sm = d["config"]["stage_ms"]
print(sys.argv[2], "wall %.4f" % d["ms_per_step"], "events %.4f" % sm["timed_step_events"], {k: round(v, 4) for k, v in sm.items() if isinstance(v, float)})
PY
  done
done
echo DONE
