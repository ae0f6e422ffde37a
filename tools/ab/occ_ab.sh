#!/bin/bash
# Occupancy A/B for the C4k step's kernels (variant libraries under _lib/var built by
# tools/build_variant.sh with -DAVDB_K2_KEYED_WAVES / -DAVDB_DIGEST_WAVES): each
# variant's keyed parity tests, then the C4k bench line per library, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-occab}
OUT=gpurun_out/$T
mkdir -p "$OUT"
LIBS="annotatedvdb_amd/_lib/libavdb_hip.so $(ls annotatedvdb_amd/_lib/var/libavdb_*.so 2>/dev/null)"
for lib in $LIBS; do
  v=$(basename "$lib" .so)
  AVDB_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle \
    "tests/test_gpu_c1.py::test_keyed_record_prep_feeds_k7" tests/test_gpu_parity.py::test_c5_all_shards_vs_c_oracle \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.log" 2>&1 \
    || { tail -30 "$OUT/pytest_$v.log"; exit 1; }
  echo "$v $(tail -1 $OUT/pytest_$v.log)"
done
for rep in 1 2; do
  for lib in $LIBS; do
    v=$(basename "$lib" .so)
    AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload c4k --steps 10 --warmup 3 --cpu-baseline off \
      > "$OUT/c4k_${v}_$rep.json" 2> "$OUT/c4k_${v}_$rep.err" || { tail -5 "$OUT/c4k_${v}_$rep.err"; exit 1; }
    python - "$OUT/c4k_${v}_$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sm = d["config"]["stage_ms"]
print(sys.argv[2], "step %.3f" % d["ms_per_step"], " ".join("%s=%.3f" % (k, v) for k, v in sm.items() if isinstance(v, float)))
PY
  done
done
echo DONE
