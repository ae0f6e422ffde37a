#!/bin/bash
# K7 A/B: the K7 GPU parity tests on the in-tree library, then the keyed C4 probe
# (tools/k7_probe.py, keys + paths) alternating the in-tree library with every
# variant under annotatedvdb_amd/_lib/var/, then the C4k bench step for each.
#   tools/ab/k7_lib_ab.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-k7ab}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
export AVDB_K7_PROBE_MODE=both
timeout -k 10 900 python -u -m pytest tests/test_gpu_c1.py tests/test_gpu_parity.py tests/test_gpu_adsp.py \
  tests/test_gpu_c4k.py ${AVDB_AB_TESTS:-} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
LIBS="annotatedvdb_amd/_lib/libavdb_hip.so $(ls annotatedvdb_amd/_lib/var/libavdb_*.so 2>/dev/null)"
for rep in 1 2; do
  for lib in $LIBS; do
    v=$(basename "$lib" .so)
    AVDB_LIB=$lib timeout -k 10 240 python tools/k7_probe.py 125000000 4 > "$OUT/probe_${v}_$rep.json" 2>&1 || exit 1
    echo "$v $(tail -1 $OUT/probe_${v}_$rep.json | cut -c1-160)"
  done
done
for lib in $LIBS; do
  v=$(basename "$lib" .so)
  AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload c4k --steps 10 --warmup 3 --cpu-baseline off \
    > "$OUT/bench_c4k_$v.log" 2>&1 || exit 1
  python - "$OUT/bench_c4k_$v.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], "ms", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 4), d["config"]["stage_ms"])
PY
done
