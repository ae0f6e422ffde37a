#!/bin/bash
# Round 6: K7 small-batch grid = one resident generation: K7 / C1 / grid tests, then the C1 line x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06r; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_c1.py "tests/test_gpu_parity.py::test_grid_knobs_parity" "tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle" tests/test_gpu_onepass.py tests/test_gpu_adsp.py tests/test_gpu_existing.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-baseline off --workload c1 > "$OUT/bench_c1.log" 2>&1 || exit $?
  python - "$OUT/bench_c1.log" "c1" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,4) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
done
