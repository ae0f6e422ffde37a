#!/bin/bash
# Round 6 K7 attribution (patched copies, not kept; wrong text): no key rendering / no path rendering /
# no flush, against the same-flags base, C4k line stage times, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06ab; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for v in base nokeys nopaths noflush; do
  timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload c4k > "$OUT/bench_c4k_$v.log" 2>&1 || exit $?
  python - "$OUT/bench_c4k_$v.log" "c4k $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), "K7", round(d["config"]["stage_ms"]["primary_keys"],3))
PY
done; done
