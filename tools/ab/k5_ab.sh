#!/bin/bash
# A/B of K5 sink variants built as annotatedvdb_amd/_lib/var/libavdb_*.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in annotatedvdb_amd/_lib/var/libavdb_*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 120 python tools/k5_probe.py ${1:-8388608} || exit 1
done
