#!/bin/bash
# Round 6: the count-free emit's workgroup size (AVDB_VCF_SLOT_BLOCK 256 / 128 / 64; one workgroup per
# window of ~200 records): tokenizer tests on the 64 variant, then the vcf line alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06aa; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_s64.so python -u -m pytest tests/test_gpu_tokenize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in base s128 s64; do
  timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 20 --warmup 5 --cpu-baseline off --workload vcf > "$OUT/bench_vcf_$v.log" 2>&1 || exit $?
  python - "$OUT/bench_vcf_$v.log" "vcf $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4))
PY
done; done
