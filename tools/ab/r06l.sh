#!/bin/bash
# Round 6: count-free K0 with the parse writing records + allele bytes to window slots
# (emit = coalesced slot moves, no second read of the text): tokenizer tests, the vcf
# line twice, the kernel summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06l; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tokenize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --workload vcf > "$OUT/bench_vcf$k.log" 2>&1 || exit $?
  python - "$OUT/bench_vcf$k.log" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print("vcf", round(d["ms_per_step"],4), d["roofline"]["frac"], d["config"].get("stage_ms"))
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python bench.py --steps 20 --warmup 5 --cpu-baseline off --workload vcf > "$OUT/prof.log" 2>&1 || exit $?
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1); cp "$f" "$OUT/vcf_kernel_stats.csv"; cut -d, -f1-4 "$OUT/vcf_kernel_stats.csv" | cut -c1-150 | head -12
