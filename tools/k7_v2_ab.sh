#!/bin/bash
# K7 write pass A/B: round-3 (AVDB_K7_V2=0) vs the split-range renderer (=1) on the
# keyed C4 batch (tools/k7_probe.py) and the C4k bench step, plus its GPU tests.
#   tools/k7_v2_ab.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-k7v2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_c1.py tests/test_gpu_c4k.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
for v in 0 1 0 1; do
  AVDB_K7_V2=$v timeout -k 10 240 python tools/k7_probe.py 125000000 4 > "$OUT/probe_v$v.json" 2>&1 || exit 1
  echo "v$v $(cat $OUT/probe_v$v.json | tail -1)"
done
for v in 0 1; do
  AVDB_K7_V2=$v timeout -k 10 300 python bench.py --workload c4k --steps 10 --warmup 3 --cpu-baseline off \
    > "$OUT/bench_c4k_v$v.log" 2>&1 || exit 1
  python - "$OUT/bench_c4k_v$v.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], "ms", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 4), d["config"]["stage_ms"])
PY
done
