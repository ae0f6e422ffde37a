#!/bin/bash
# Round 6: narrow key / path offsets (AVDB_KEYS_OFF32) in the serial keyed step — parity tests, then
# the C4k line with and without (AVDB_BENCH_NARROW=0), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06j; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_c1.py tests/test_gpu_onepass.py "tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle" "tests/test_gpu_c4k.py::test_c4k_shard_vs_c_oracle[0]" -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  timeout -k 10 300 env AVDB_BENCH_NARROW=$v python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload c4k > "$OUT/bench_narrow$v.log" 2>&1 || exit $?
  python - "$OUT/bench_narrow$v.log" "narrow=$v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["config"]["stage_ms"].items() if isinstance(v,float)})
PY
done
