#!/bin/bash
# Round 6 probe: K7 flush stores folded into the first 64 KB of each output (variant -DAVDB_PROBE_FLUSH_L2=1,
# a patch not kept: wrong text, the same instructions, no HBM write stream for the text) vs base:
# what the text store stream costs K7 on the C4k line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06z; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for v in base flushl2; do
  timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload c4k > "$OUT/bench_c4k_$v.log" 2>&1 || exit $?
  python - "$OUT/bench_c4k_$v.log" "c4k $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,3) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
done; done
