#!/bin/bash
# C2 step launched per step vs replayed as a captured HIP graph (ms_per_step only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c2graph; mkdir -p $OUT
for rep in 1 2; do for g in off on; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline off --keyed off --graph $g > $OUT/c2_${g}_$rep.log 2>&1 || { tail -20 $OUT/c2_${g}_$rep.log; exit 1; }
  python3 -c "
import json; l=[x for x in open('$OUT/c2_${g}_$rep.log') if x.startswith('{')][-1]; d=json.loads(l)
print('graph=$g', round(d['ms_per_step'],4), d['config']['stage_ms'], d['roofline'].get('kernel_ms'))"
done; done
