#!/bin/bash
# K3 marks filtered in the keyed K2: the keyed / dedup GPU tests, then the C4k and C1
# lines for the new library and the round's baseline (_lib/var/libavdb_r05base.so), alternating.
#   tools/ab/r05k3.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05k3}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_c1.py tests/test_gpu_c4k.py -m gpu -x -q --timeout 600 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
  for lib in ${LIBS:-annotatedvdb_amd/_lib/libavdb_hip.so annotatedvdb_amd/_lib/var/libavdb_r05base.so}; do
    v=$(basename "$lib" .so)
    for w in c4k c1; do
      AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --cpu-baseline off \
        > "$OUT/${w}_${v}_$rep.json" 2> "$OUT/${w}_${v}_$rep.err" || { tail -5 "$OUT/${w}_${v}_$rep.err"; exit 1; }
      python - "$OUT/${w}_${v}_$rep.json" "$w $v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sm = d["config"]["stage_ms"]
print(sys.argv[2], "step %.4f" % d["ms_per_step"], " ".join("%s=%.4f" % (k, v) for k, v in sm.items() if isinstance(v, float)))
PY
    done
  done
done
echo DONE
