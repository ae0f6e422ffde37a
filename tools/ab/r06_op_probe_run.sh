#!/bin/bash
# k_keyed_onepass attribution: the C4k onepass line with each probe library (tools/ab/r06_op_probes.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06f}; shift; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in base "$@" base; do
  lib=annotatedvdb_amd/_lib/libavdb_hip.so; [ "$v" != base ] && lib=annotatedvdb_amd/_lib/var/libavdb_$v.so
  timeout -k 10 300 env AVDB_LIB=$lib AVDB_BENCH_LAYOUT=onepass python bench.py --steps 8 --warmup 2 --cpu-baseline off --workload c4k > "$OUT/bench_$v.log" 2>&1 || exit $?
  python - "$OUT/bench_$v.log" "$v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["config"]["stage_ms"].items() if isinstance(v,float)})
PY
done
