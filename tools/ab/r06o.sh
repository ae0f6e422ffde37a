#!/bin/bash
# Round 6: C5 through pipeline.PrepStep (keyed K2 without K7 totals: K4 codes + K3 marks) vs
# the plain K2 -> K3 -> K4 chain; parity tests first.
# (AVDB_BENCH_C5_PLAIN was a temporary bench switch for this A/B, removed after it: the plain arm no longer exists)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06o; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest "tests/test_gpu_parity.py::test_c5_all_shards_vs_c_oracle" "tests/test_gpu_parity.py::test_c5_full_size_vs_c_oracle" "tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle" tests/test_gpu_c1.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in 1 0; do
  timeout -k 10 300 env AVDB_BENCH_C5_PLAIN=$v python bench.py --steps 20 --warmup 3 --cpu-baseline off --workload c5 > "$OUT/bench_c5_plain$v.log" 2>&1 || exit $?
  python - "$OUT/bench_c5_plain$v.log" "c5 plain=$v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,4) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
done; done
