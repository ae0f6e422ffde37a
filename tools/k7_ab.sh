#!/bin/bash
# K7 write-pass A/B over library variants (tools/build_variant.sh NAME -DAVDB_K7_EXP=..):
#   tools/k7_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in annotatedvdb_amd/_lib/var/libavdb_*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 200 python tools/k7_probe.py 125000000 3 || exit 1
done
