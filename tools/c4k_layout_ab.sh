#!/bin/bash
# C4k step layouts A/B on one box (pipeline.KeyedStep: serial | fork | overlap, and
# the overlap layout with K4's persistent grid capped, AVDB_BENCH_K4_GRID workgroups).
#   tools/c4k_layout_ab.sh TAG [layout:grid ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-c4k_ab}; shift
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
CASES=${@:-serial:0 overlap:0 fork:0 overlap:512 overlap:256 overlap:128 serial:0}
for c in $CASES; do
  L=${c%%:*}; G=${c##*:}
  timeout -k 10 300 env AVDB_BENCH_LAYOUT=$L AVDB_BENCH_K4_GRID=$G python bench.py --workload c4k --steps 10 \
      --warmup 3 --cpu-baseline off > "$OUT/c4k_${L}_${G}.json" 2> "$OUT/c4k_${L}_${G}.err"
  rc=$?
  [ $rc -ne 0 ] && { echo "FAIL $c rc=$rc"; tail -5 "$OUT/c4k_${L}_${G}.err"; exit $rc; }
  python - "$OUT/c4k_${L}_${G}.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sm = d["config"]["stage_ms"]
print(sys.argv[2], "step %.3f ms" % d["ms_per_step"], "span %.3f" % sm["step_span"],
      " ".join("%s=%.3f" % (k, v) for k, v in sm.items() if k != "step_span"), "frac %.3f" % d["roofline"]["frac"])
PY
done
echo DONE
