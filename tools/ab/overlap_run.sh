#!/bin/bash
# tools/overlap_probe.py at K4 grids of 1, 2, 3 workgroups per CU (one process each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-overlap}
mkdir -p "$OUT"
for g in 3 2 1; do
  AVDB_K4_BLOCKS_PER_CU=$g timeout -k 10 240 python tools/overlap_probe.py 125000000 4 > "$OUT/k4g$g.json" 2> "$OUT/k4g$g.err" || exit $?
  cat "$OUT/k4g$g.json"
done
