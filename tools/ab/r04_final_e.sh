#!/bin/bash
# Round-end measurement after the grid changes (part 2: kernel stats, traffic, K7 counters).
#   tools/ab/r04_final_e.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04fe}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_run.sh "$T" prof:c2 prof:c4k prof:c1 prof:c5 prof:load prof:vcf || exit 1
for w in c4k load vcf; do
  bash tools/traffic_counters.sh "$w" "$T/traffic_$w" > "$OUT/traffic_$w.log" 2>&1 || { tail -5 "$OUT/traffic_$w.log"; exit 1; }
  echo "traffic $w done"
done
bash tools/k7_counters.sh "$T/k7" > "$OUT/k7_counters.log" 2>&1 || { tail -5 "$OUT/k7_counters.log"; exit 1; }
echo DONE-E
