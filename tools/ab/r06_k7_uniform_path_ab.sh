#!/bin/bash
# Round 6: K7 write pass rendering a tile's ltree paths from scalar registers when all its records share one bin
# ('upath', AVDB_K7_UNIFORM_PATH=1 on a patched copy) vs a same-flags base build (tools/build_variant.sh):
# K7 tests on the variant, then the C4k and C1 lines alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06_k7upath; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in upath; do
  timeout -k 10 600 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python -u -m pytest tests/test_gpu_c1.py "tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle" tests/test_gpu_onepass.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.log" 2>&1
  rc=$?; echo "$v: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
for v in base upath; do
  for wl in c4k c1; do
    timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload $wl > "$OUT/bench_${wl}_$v.log" 2>&1 || exit $?
    python - "$OUT/bench_${wl}_$v.log" "$wl $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,3) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
  done
done; done
