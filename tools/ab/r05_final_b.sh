#!/bin/bash
# Round-5 measurement (part B): rocprofv3 kernel stats per workload, request-size
# traffic (c4k, load, vcf), K7 counters, and the C2 FETCH_SIZE / WRITE_SIZE passes.
#   tools/ab/r05_final_b.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05fb}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_run.sh "$T" prof:c2 prof:c4k prof:c1 prof:c5 prof:load prof:vcf || exit 1
for w in c4k load vcf; do
  bash tools/traffic_counters.sh "$w" "$T/traffic_$w" > "$OUT/traffic_$w.log" 2>&1 || { tail -5 "$OUT/traffic_$w.log"; exit 1; }
  echo "traffic $w done"
done
bash tools/k7_counters.sh "$T/k7" > "$OUT/k7_counters.log" 2>&1 || { tail -5 "$OUT/k7_counters.log"; exit 1; }
echo "k7 counters done"
echo DONE-B
