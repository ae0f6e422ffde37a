#!/bin/bash
# K0 kernel times per library: the in-tree one and every variant under
# annotatedvdb_amd/_lib/var/ (rocprofv3 --kernel-trace --stats over tools/k0_attr.py).
#   tools/k0_attr.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-k0attr}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
LIBS="annotatedvdb_amd/_lib/libavdb_hip.so $(ls annotatedvdb_amd/_lib/var/libavdb_*.so 2>/dev/null)"
for rep in 1 2; do
  for lib in $LIBS; do
    v=$(basename "$lib" .so)
    AVDB_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${v}_$rep" -o run --output-format csv \
      -- python3 tools/k0_attr.py 6 > "$OUT/prof_${v}_$rep.log" 2>&1 || { tail -5 "$OUT/prof_${v}_$rep.log"; exit 1; }
    python3 - "$OUT/prof_${v}_$rep" "$v" <<'PY'
import glob, os, sys
sys.path.insert(0, "tools")
from prof_summary import stats
d = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_stats.csv"), recursive=True)
rows = stats(os.path.dirname(d[0]))
print(sys.argv[2], " ".join("%s=%.1f" % (r["kernel"].replace("avdb::", ""), r["avg_us"]) for r in rows if "vcf" in r["kernel"]))
PY
  done
done
echo DONE
