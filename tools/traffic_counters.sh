#!/bin/bash
# Exact L2->fabric bytes per kernel from request-size counters (two rocprofv3
# --pmc passes, 4 TCC counters each):
#   read  = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B,  DRAM_32B = read requests to DRAM in 32-B units
#   write = 32*(WRREQ - WRREQ_64B) + 64*WRREQ_64B,          WRITE_DRAM_32B likewise for writes
#   tools/traffic_counters.sh WORKLOAD [OUT]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
W=$1; O=gpurun_out/${2:-traffic_$W}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_32B_sum -d "$O/rd" -o run --output-format csv -- python3 bench.py --workload "$W" --steps 2 --warmup 1 --cpu-baseline off > "$O/rd.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum -d "$O/wr" -o run --output-format csv -- python3 bench.py --workload "$W" --steps 2 --warmup 1 --cpu-baseline off > "$O/wr.log" 2>&1 &&
python3 tools/prof_summary.py traffic "$O/rd" "$O/wr" > "$O/traffic.json" && cat "$O/traffic.json"
