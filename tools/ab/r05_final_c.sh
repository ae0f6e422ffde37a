#!/bin/bash
# Round-5 re-measurement after the K0 candidate pass and the one-stream C1 graph:
# GPU suite, smoke, the default / C1 / C4k / vcf / load lines, their kernel stats and
# the vcf / load traffic.   tools/ab/r05_final_c.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05fc}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_run.sh "$T" test smoke c2 c1 c4k vcf load prof:vcf prof:load prof:c1 || exit 1
for w in vcf load; do
  bash tools/traffic_counters.sh "$w" "$T/traffic_$w" > "$OUT/traffic_$w.log" 2>&1 || { tail -5 "$OUT/traffic_$w.log"; exit 1; }
  echo "traffic $w done"
done
echo DONE-C
