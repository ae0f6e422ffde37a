#!/bin/bash
# K4 (VRS digest) on the C5 batch: event timing, kernel stats and two SQ counter
# passes (each its own rocprofv3 run; MI355X_MICROARCH.md PMC slot limits).
#   tools/k4_counters.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-k4}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 python tools/k4_probe.py 25000000 5 > "$OUT/probe.json" 2> "$OUT/probe.err" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 tools/k4_probe.py 25000000 3 > "$OUT/prof.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU GRBM_GUI_ACTIVE -d "$OUT/pmc1" -o run --output-format csv -- python3 tools/k4_probe.py 25000000 2 > "$OUT/pmc1.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH -d "$OUT/pmc2" -o run --output-format csv -- python3 tools/k4_probe.py 25000000 2 > "$OUT/pmc2.log" 2>&1
rc=$?
cat "$OUT/probe.json"
exit $rc
