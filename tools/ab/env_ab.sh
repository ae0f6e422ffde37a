#!/bin/bash
# Environment-knob A/B on the in-tree library: the WORKLOAD bench line with no
# knob set and with each VAR=VALUE given, two passes, interleaved.
#   tools/ab/env_ab.sh TAG WORKLOAD VAR=VALUE [VAR=VALUE ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; W=$2; shift 2
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for kv in base "$@"; do
    if [ "$kv" = base ]; then
      timeout -k 10 300 python bench.py --workload "$W" --steps 10 --warmup 3 --cpu-baseline off \
        > "$OUT/${W}_${kv}_$rep.log" 2>&1 || { tail -20 "$OUT/${W}_${kv}_$rep.log"; exit 1; }
    else
      env "$kv" timeout -k 10 300 python bench.py --workload "$W" --steps 10 --warmup 3 --cpu-baseline off \
        > "$OUT/${W}_${kv}_$rep.log" 2>&1 || { tail -20 "$OUT/${W}_${kv}_$rep.log"; exit 1; }
    fi
    python3 - "$OUT/${W}_${kv}_$rep.log" "$kv" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], round(d["ms_per_step"], 4), d["config"].get("stage_ms"))
PY
  done
done
