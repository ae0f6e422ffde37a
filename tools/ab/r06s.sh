#!/bin/bash
# Round 6: the text sink's 8-byte global stores as nontemporal (variant build -DAVDB_OUT_NT=1, not
# kept in the sources) vs the same-flags base: load and vcf lines, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06s; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for v in base nt; do
  for wl in load vcf; do
    timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload $wl > "$OUT/bench_${wl}_$v.log" 2>&1 || exit $?
    python - "$OUT/bench_${wl}_$v.log" "$wl $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,3) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
  done
done; done
