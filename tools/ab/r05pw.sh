#!/bin/bash
# Window-parse launch bound A/B: AVDB_VCF_PARSE_WAVES=5 (_lib/var/libavdb_pw5.so) against the
# shipped 6 (which the compiler misses: 95 VGPRs, five waves), on the counted vcf path and the
# load line, alternating.   tools/ab/r05pw.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05pw}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in annotatedvdb_amd/_lib/libavdb_hip.so annotatedvdb_amd/_lib/var/libavdb_pw5.so; do
    v=$(basename "$lib" .so)
    for w in vcf load; do
      AVDB_BENCH_VCF_COUNTED=1 AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 \
        --cpu-baseline off > "$OUT/${w}_${v}_$rep.json" 2> "$OUT/${w}_${v}_$rep.err" || { tail -5 "$OUT/${w}_${v}_$rep.err"; exit 1; }
      python - "$OUT/${w}_${v}_$rep.json" "$w $v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "step %.4f" % d["ms_per_step"], {k: round(v, 4) for k, v in d["config"]["stage_ms"].items() if isinstance(v, float)})
PY
    done
  done
done
echo DONE
