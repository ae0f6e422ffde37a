#!/bin/bash
# Round-5 last measurement (after the K3 marks filter and the count-free K0 records path):
#   part a: GPU suite, smoke, the default / C1 / C4k / vcf lines, C4k and vcf kernel summaries and traffic
#   part b: vcf, load, C3, C4, C5, drop-in lines, vcf / C1 / load kernel summaries, vcf and load traffic
#   tools/ab/r05_final_d.sh TAG a|b
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05fd}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$2" = a ]; then
  bash tools/gpu_run.sh "$T" test smoke c2 c1 c4k vcf prof:vcf prof:c4k || exit 1
  TW="vcf c4k"
else
  bash tools/gpu_run.sh "$T" vcf load c3 c4 c5 dropin prof:vcf prof:c1 prof:load || exit 1
  TW="vcf load"
fi
for w in $TW; do
  bash tools/traffic_counters.sh "$w" "$T/traffic_$w" > "$OUT/traffic_$w.log" 2>&1 || { tail -5 "$OUT/traffic_$w.log"; exit 1; }
  echo "traffic $w done"
done
echo DONE-D
