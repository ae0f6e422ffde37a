#!/bin/bash
# A/B of library variants built as annotatedvdb_amd/_lib/var/libavdb_*.so on one
# bench workload: tools/ab/lib_ab.sh WORKLOAD [STEPS]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in annotatedvdb_amd/_lib/var/libavdb_*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload "$1" --steps "${2:-5}" --warmup 2 --cpu-baseline off || exit 1
done
