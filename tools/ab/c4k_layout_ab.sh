#!/bin/bash
# C4k step layouts A/B on one box (pipeline.KeyedStep: serial | fork | overlap, and
# the overlap layout with K4's persistent grid capped, AVDB_BENCH_K4_GRID workgroups,
# and K7's write pass capped, AVDB_BENCH_K7_GRID one-wave workgroups).
#   tools/ab/c4k_layout_ab.sh TAG [layout:k4grid:k7grid ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-c4k_ab}; shift
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
CASES=${@:-serial:0:0 overlap:0:0 fork:0:0 overlap:512:0 overlap:256:0 overlap:128:0 serial:0:0}
for c in $CASES; do
  IFS=: read -r L G K <<< "$c"
  K=${K:-0}
  tag="${L}_${G}_${K}"
  timeout -k 10 300 env AVDB_BENCH_LAYOUT=$L AVDB_BENCH_K4_GRID=$G AVDB_BENCH_K7_GRID=$K python bench.py \
      --workload c4k --steps 10 --warmup 3 --cpu-baseline off > "$OUT/c4k_$tag.json" 2> "$OUT/c4k_$tag.err"
  rc=$?
  [ $rc -ne 0 ] && { echo "FAIL $c rc=$rc"; tail -5 "$OUT/c4k_$tag.err"; exit $rc; }
  python - "$OUT/c4k_$tag.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sm = d["config"]["stage_ms"]
print(sys.argv[2], "step %.3f ms" % d["ms_per_step"], "span %.3f" % sm["step_span"],
      " ".join("%s=%.3f" % (k, v) for k, v in sm.items() if k != "step_span"), "frac %.3f" % d["roofline"]["frac"])
PY
done
echo DONE
