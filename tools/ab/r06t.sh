#!/bin/bash
# Round 6: K7 flush with plain stores in each span's first and last 128-byte line (variant
# -DAVDB_K7_EDGE_PLAIN=1) vs the same-flags base: C4k small + C1 parity on the variant, then the C4k line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06t; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_edge.so python -u -m pytest "tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle" "tests/test_gpu_c4k.py::test_c4k_shard_vs_c_oracle[3]" tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
for v in base edge; do
  timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload c4k > "$OUT/bench_c4k_$v.log" 2>&1 || exit $?
  python - "$OUT/bench_c4k_$v.log" "c4k $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,3) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
done; done
