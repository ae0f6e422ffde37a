#!/bin/bash
# Round 6: layout "early" (K4 from the SoA on a second stream beside K2 + K3) against the
# serial step, with K4's persistent grid at the default / 512 / 256 workgroups.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06k; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for arm in serial:0 early:0 early:512 early:256; do
  lay=${arm%%:*}; g=${arm##*:}
  timeout -k 10 300 env AVDB_BENCH_LAYOUT=$lay AVDB_BENCH_K4_GRID=$g python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload c4k > "$OUT/bench_${lay}_$g.log" 2>&1 || exit $?
  python - "$OUT/bench_${lay}_$g.log" "$arm" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["config"]["stage_ms"].items() if isinstance(v,float)})
PY
done; done
