#!/bin/bash
# Round-end re-measurement after the K0 window parse: GPU suite, smoke, the default
# line, C1, vcf, load, their kernel stats and the vcf / load traffic.
#   tools/ab/r04_final_c.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04fd}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_run.sh "$T" test smoke c2 c1 vcf load prof:vcf prof:load || exit 1
for w in vcf load; do
  bash tools/traffic_counters.sh "$w" "$T/traffic_$w" > "$OUT/traffic_$w.log" 2>&1 || { tail -5 "$OUT/traffic_$w.log"; exit 1; }
  echo "traffic $w done"
done
echo DONE-C
