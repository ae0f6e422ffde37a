#!/bin/bash
# K7 (primary keys + ltree paths) on the keyed C4 batch: probe timing, kernel
# stats, two SQ counter passes and the request-size traffic passes.
#   tools/k7_counters.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-k7}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
P="tools/k7_probe.py 125000000 3"
export AVDB_K7_PROBE_MODE=both
timeout -k 10 240 python $P > "$OUT/probe.json" 2> "$OUT/probe.err" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 $P > "$OUT/prof.log" 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD -d "$OUT/pmc1" -o run --output-format csv -- python3 $P > "$OUT/pmc1.log" 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS -d "$OUT/pmc2" -o run --output-format csv -- python3 $P > "$OUT/pmc2.log" 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_32B_sum -d "$OUT/rd" -o run --output-format csv -- python3 $P > "$OUT/rd.log" 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum -d "$OUT/wr" -o run --output-format csv -- python3 $P > "$OUT/wr.log" 2>&1
rc=$?
cat "$OUT/probe.json"
exit $rc
