#!/bin/bash
# Round 6: K0 window-parse variants (launch bound 4 waves; 20 / 28 KB windows) on the vcf line
# against the same-flags base build, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06p; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for v in base pw4 w20 w28; do
  timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 20 --warmup 5 --cpu-baseline off --workload vcf > "$OUT/bench_vcf_$v.log" 2>&1 || exit $?
  python - "$OUT/bench_vcf_$v.log" "vcf $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), d["config"].get("path"))
PY
done; done
