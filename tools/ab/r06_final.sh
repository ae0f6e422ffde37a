#!/bin/bash
# Round-6 measurement (one GPU-box call per part):
#   t: GPU suite + smoke
#   a: default / C1 / C4k / vcf lines, C4k / vcf / C1 kernel summaries, C4k + vcf traffic
#   b: load, C3, C4, C5, drop-in lines, load / C2 kernel summaries, load traffic, K7 counters
#   tools/ab/r06_final.sh TAG t|a|b
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${1:-r06f}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
TW=""
case "$2" in
  t) bash tools/gpu_run.sh "$T" test smoke || exit 1 ;;
  a) bash tools/gpu_run.sh "$T" c2 c1 c4k vcf prof:c4k prof:vcf prof:c1 || exit 1; TW="c4k vcf" ;;
  b) bash tools/gpu_run.sh "$T" load c3 c4 c5 dropin prof:load prof:c2 || exit 1; TW="load"
     bash tools/k7_counters.sh "$T/k7" > "$OUT/k7_counters.log" 2>&1 || { tail -5 "$OUT/k7_counters.log"; exit 1; } ;;
esac
for w in $TW; do
  bash tools/traffic_counters.sh "$w" "$T/traffic_$w" > "$OUT/traffic_$w.log" 2>&1 || { tail -5 "$OUT/traffic_$w.log"; exit 1; }
  echo "traffic $w done"
done
echo DONE-$2
