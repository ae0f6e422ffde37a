#!/bin/bash
# Round 6 probe: the text sink's 8-byte stores all folded into the first 64 KB of the output
# (variant -DAVDB_PROBE_L2SINK=1: wrong text, same store instructions, no HBM write stream)
# vs base: how much of K5's write pass is its write traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06u; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for v in base l2sink; do
  timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload load > "$OUT/bench_load_$v.log" 2>&1 || exit $?
  python - "$OUT/bench_load_$v.log" "load $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,3) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
done; done
