#!/bin/bash
# K7 write-pass attribution: for each library variant built with
#   tools/build_variant.sh xN -DAVDB_K7V2_EXP=N
# (each knob drops one part of k_record_keys_v2, see avdb_keys.hip), the C4k
# keys + paths time (tools/k7_probe.py) and one SQ counter pass.
#   tools/k7_attr.sh TAG         summary: python tools/k7_attr_report.py gpurun_out/TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-k7attr}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
export AVDB_K7_PROBE_MODE=both
P="tools/k7_probe.py 125000000 3"
for lib in annotatedvdb_amd/_lib/var/libavdb_x*.so; do
  v=$(basename "$lib" .so); v=${v#libavdb_}
  echo "== $v $(date +%T)"
  AVDB_LIB=$lib timeout -k 10 200 python $P > "$OUT/probe_$v.json" 2> "$OUT/probe_$v.err" || exit 1
  tail -1 "$OUT/probe_$v.json"
  AVDB_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH \
    -d "$OUT/pmc_$v" -o run --output-format csv -- python3 $P > "$OUT/pmc_$v.log" 2>&1 || exit 1
done
echo DONE
