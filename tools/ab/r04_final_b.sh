#!/bin/bash
# Round-end measurement (part B): bench lines, kernel stats and traffic / SQ counters
# from one box.  tools/ab/r04_final_b.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04fin}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_run.sh "$T" c1 c3 c4 c5 c4k load vcf prof:c2 prof:c4k prof:c1 prof:c5 prof:load prof:vcf || exit 1
for w in c4k load vcf; do
  bash tools/traffic_counters.sh "$w" "$T/traffic_$w" > "$OUT/traffic_$w.log" 2>&1 || { tail -5 "$OUT/traffic_$w.log"; exit 1; }
  echo "traffic $w done"
done
bash tools/k7_counters.sh "$T/k7" > "$OUT/k7_counters.log" 2>&1 || { tail -5 "$OUT/k7_counters.log"; exit 1; }
echo DONE-B
