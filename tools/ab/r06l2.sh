#!/bin/bash
# Round 6: kernel summary of the vcf line (count-free K0, slot path)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06l2; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --workload vcf > "$OUT/prof.log" 2>&1 || exit $?
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1); cp "$f" "$OUT/vcf_kernel_stats.csv"; cut -d, -f1-4 "$OUT/vcf_kernel_stats.csv" | cut -c1-60,200-400 | head -12
