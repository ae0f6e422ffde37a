#!/bin/bash
# Round 5: LDS stages filled with every load in flight (stage_copy) — tokenizer /
# format tests, K0 kernel times, then the load line (K5 staging batched vs the
# one-load-per-trip loop, variant libavdb_k5loop) twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05o}
OUT=gpurun_out/$T
mkdir -p "$OUT"
bash tools/ab/r05j.sh "$T" || exit 1
for rep in 1 2; do
  for lib in annotatedvdb_amd/_lib/libavdb_hip.so $(ls annotatedvdb_amd/_lib/var/libavdb_*.so 2>/dev/null); do
    v=$(basename "$lib" .so)
    AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload load --steps 10 --warmup 3 --cpu-baseline off \
      > "$OUT/load_${v}_$rep.log" 2>&1 || { tail -5 "$OUT/load_${v}_$rep.log"; exit 1; }
    python3 - "$OUT/load_${v}_$rep.log" "$v" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], round(d["ms_per_step"], 4), {k: round(v, 3) for k, v in d["config"]["stage_ms"].items() if isinstance(v, float)})
PY
  done
done
echo DONE
