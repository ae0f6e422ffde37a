#!/bin/bash
# K0 (VCF tokenizer) on the bench's 8.4 M-line text: kernel stats and two SQ
# counter passes (each its own rocprofv3 run; MI355X_MICROARCH.md PMC slot limits).
#   tools/k0_counters.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-k0}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --workload vcf --steps 3 --warmup 1 --cpu-baseline off"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 $B > "$OUT/prof.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD -d "$OUT/pmc1" -o run --output-format csv -- python3 $B > "$OUT/pmc1.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS -d "$OUT/pmc2" -o run --output-format csv -- python3 $B > "$OUT/pmc2.log" 2>&1
