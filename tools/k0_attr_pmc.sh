#!/bin/bash
# K0 instruction counts per library (in-tree + annotatedvdb_amd/_lib/var/*): one SQ
# counter pass each over tools/k0_attr.py (VALU / SALU / LDS / branch / waves).
#   tools/k0_attr_pmc.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-k0pmc}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in annotatedvdb_amd/_lib/libavdb_hip.so $(ls annotatedvdb_amd/_lib/var/libavdb_*.so 2>/dev/null); do
  v=$(basename "$lib" .so)
  AVDB_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH SQ_WAVE_CYCLES \
    -d "$OUT/pmc_$v" -o run --output-format csv -- python3 tools/k0_attr.py 3 > "$OUT/pmc_$v.log" 2>&1 || { tail -5 "$OUT/pmc_$v.log"; exit 1; }
  python3 - "$OUT/pmc_$v" "$v" <<'PY'
import sys
sys.path.insert(0, "tools")
from prof_summary import per_kernel
for k, c in per_kernel(sys.argv[1]).items():
    if "parse" in k:
        w = c["SQ_WAVES"]
        print(sys.argv[2], k, "per wave: VALU %.0f SALU %.0f LDS %.0f BR %.0f cyc %.0f" % (
            c["SQ_INSTS_VALU"] / w, c["SQ_INSTS_SALU"] / w, c["SQ_INSTS_LDS"] / w, c["SQ_INSTS_BRANCH"] / w,
            c["SQ_WAVE_CYCLES"] / w))
PY
done
echo DONE
