#!/bin/bash
# One workload on the GPU box: bench line, rocprofv3 kernel stats, and separate
# FETCH_SIZE / WRITE_SIZE passes.  Usage: tools/gpu_prof_workload.sh WORKLOAD [STEPS]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
W=$1; S=${2:-5}
OUT=gpurun_out/$W
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --workload "$W" --steps "$S" --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --workload "$W" --steps 3 --warmup 1 --cpu-baseline off > "$OUT/prof.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --workload "$W" --steps 2 --warmup 1 --cpu-baseline off > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --workload "$W" --steps 2 --warmup 1 --cpu-baseline off > "$OUT/pmc_write.log" 2>&1
rc=$?
tail -c 3000 "$OUT/bench.json"
exit $rc
