#!/bin/bash
# The count-free records path (avdb_vcf_parse_local / avdb_vcf_emit_local): tokenizer
# and format tests, then the vcf line with it and with the counted path
# (AVDB_BENCH_VCF_COUNTED=1), alternating, and a kernel summary of each.
#   tools/ab/r05lc.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05lc}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
[ -n "$PROF_ONLY" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_format.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
[ -n "$PROF_ONLY" ] || tail -1 "$OUT/pytest.log"
for rep in $([ -n "$PROF_ONLY" ] || echo 1 2); do
  for counted in 0 1; do
    AVDB_BENCH_VCF_COUNTED=$counted timeout -k 10 300 python bench.py --workload vcf --steps 20 --warmup 3 \
      --cpu-baseline off > "$OUT/vcf_c${counted}_$rep.json" 2> "$OUT/vcf_c${counted}_$rep.err" \
      || { tail -5 "$OUT/vcf_c${counted}_$rep.err"; exit 1; }
    python - "$OUT/vcf_c${counted}_$rep.json" "counted=$counted" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "step %.4f" % d["ms_per_step"], "value %.4g" % d["value"], d["config"]["stage_ms"])
PY
  done
done
for counted in 0 1; do
  AVDB_BENCH_VCF_COUNTED=$counted timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$counted" \
    -o run --output-format csv -- python bench.py --workload vcf --steps 20 --warmup 3 --cpu-baseline off > "$OUT/rocprof_c$counted.log" 2>&1 \
    || { tail -5 "$OUT/rocprof_c$counted.log"; exit 1; }
  python - "$OUT/prof_c$counted" "counted=$counted" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
print(sys.argv[2], " ".join("%s=%.1f" % (r["Name"].split("(")[0].replace("void ", "").replace("avdb::", "")[:40],
      float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(f)) if "vcf" in r["Name"] or "scan" in r["Name"]))
PY
done
echo DONE
