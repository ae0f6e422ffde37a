#!/bin/bash
# K0 count-free emit A/B: this library against _lib/var/libavdb_emitold.so (the committed
# emit), tokenizer tests first, then the vcf line twice each, alternating, and a kernel
# summary of each (round 5: the window stage from the block index; then per-lane span slots).   tools/ab/r05em.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05em}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
LIBS="annotatedvdb_amd/_lib/libavdb_hip.so annotatedvdb_amd/_lib/var/libavdb_emitold.so"
timeout -k 10 600 python -u -m pytest tests/test_gpu_tokenize.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
  for lib in $LIBS; do
    v=$(basename "$lib" .so)
    AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload vcf --steps 20 --warmup 3 --cpu-baseline off \
      > "$OUT/vcf_${v}_$rep.json" 2> "$OUT/vcf_${v}_$rep.err" || { tail -5 "$OUT/vcf_${v}_$rep.err"; exit 1; }
    python - "$OUT/vcf_${v}_$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "step %.4f" % d["ms_per_step"], d["config"]["stage_ms"], d["config"].get("path"))
PY
  done
done
for lib in $LIBS; do
  v=$(basename "$lib" .so)
  AVDB_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$v" -o run --output-format csv \
    -- python bench.py --workload vcf --steps 20 --warmup 3 --cpu-baseline off > "$OUT/rocprof_$v.log" 2>&1 \
    || { tail -5 "$OUT/rocprof_$v.log"; exit 1; }
  python - "$OUT/prof_$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
print(sys.argv[2], " ".join("%s=%.1f" % (r["Name"].split("(")[0].replace("void ", "").replace("avdb::", "")[:40],
      float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(f)) if "local" in r["Name"] or "<true>" in r["Name"]))
PY
done
echo DONE
