#!/bin/bash
# K7 change check: its GPU tests (C1 + the 1e9 keyed C4k check), then the C4k bench
# step twice and the keys + paths probe.   tools/k7_check.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-k7c}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_c1.py tests/test_gpu_c4k.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for k in 1 2; do
  timeout -k 10 300 python bench.py --workload c4k --steps 10 --warmup 3 --cpu-baseline off > "$OUT/bench_c4k_$k.log" 2>&1 || exit 1
  python - "$OUT/bench_c4k_$k.log" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[1], "ms", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 4),
      {k: round(v, 3) for k, v in d["config"]["stage_ms"].items()})
PY
done
AVDB_K7_PROBE_MODE=both timeout -k 10 240 python tools/k7_probe.py 125000000 4 > "$OUT/probe.json" 2>&1 && tail -1 "$OUT/probe.json"
