#!/bin/bash
# Round 5: K0 parse + emit in one launch (avdb_vcf_parse_emit) — tokenizer tests,
# then K0 kernel times (tools/k0_attr.sh) and the vcf line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05p}
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 240 python -u -m pytest tests/test_gpu_tokenize.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest_tok.log" 2>&1 || { tail -40 "$OUT/pytest_tok.log"; exit 1; }
tail -1 "$OUT/pytest_tok.log"
bash tools/k0_attr.sh "$T/attr" || exit 1
timeout -k 10 300 python bench.py --workload vcf --steps 10 --warmup 3 --cpu-baseline off > "$OUT/vcf.json" 2>&1 || { tail -5 "$OUT/vcf.json"; exit 1; }
tail -c 900 "$OUT/vcf.json"
