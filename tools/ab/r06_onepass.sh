#!/bin/bash
# Round 6: the one-pass keyed prep — its parity tests, then the C4k line in both layouts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06b}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_onepass.py "tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle" "tests/test_gpu_c1.py::test_c1_graph_replay_vs_c_oracle" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_onepass.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_onepass.log"; [ $rc -ne 0 ] && exit $rc
for L in onepass serial onepass; do
  timeout -k 10 300 env AVDB_BENCH_LAYOUT=$L python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload c4k > "$OUT/bench_c4k_$L.log" 2>&1 || exit $?
  python - "$OUT/bench_c4k_$L.log" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(d["config"]["layout"], round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["config"]["stage_ms"].items() if isinstance(v,float)})
PY
done
