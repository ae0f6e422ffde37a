#!/bin/bash
# K0 / K5 A/B: the vcf (or WORKLOAD) bench line for the in-tree library and every
# variant under annotatedvdb_amd/_lib/var/ (two passes), after the tokenizer GPU tests.
#   tools/ab/vcf_ab.sh TAG [WORKLOAD]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-vcfab}
W=${2:-vcf}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tokenize.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
LIBS="annotatedvdb_amd/_lib/libavdb_hip.so $(ls annotatedvdb_amd/_lib/var/libavdb_*.so 2>/dev/null)"
for rep in 1 2; do
  for lib in $LIBS; do
    v=$(basename "$lib" .so)
    AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload "$W" --steps 10 --warmup 3 --cpu-baseline off \
      > "$OUT/${W}_${v}_$rep.log" 2>&1 || exit 1
    python3 - "$OUT/${W}_${v}_$rep.log" "$v" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], round(d["ms_per_step"], 4), d["config"]["stage_ms"])
PY
  done
done
