#!/bin/bash
# Round 6: count-free K0 slot writes with an SNV fast path (one record slot + one 2-byte heap
# store) vs the base build: tokenizer tests on the variant, then the vcf line alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06v; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_snv.so python -u -m pytest tests/test_gpu_tokenize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
for v in base snv; do
  timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 20 --warmup 5 --cpu-baseline off --workload vcf > "$OUT/bench_vcf_$v.log" 2>&1 || exit $?
  python - "$OUT/bench_vcf_$v.log" "vcf $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4))
PY
done; done
