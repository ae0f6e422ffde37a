#!/bin/bash
# K0 A/B: tokenizer GPU tests on each variant library, then tools/ab/vcf_ab.sh (in-tree vs variants)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04_k0occ
for v in xold xpw5 xe32; do
  AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_tokenize.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_k0occ/pytest_$v.log 2>&1 || { tail -20 gpurun_out/r04_k0occ/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r04_k0occ/pytest_$v.log)"
done
bash tools/ab/vcf_ab.sh r04_k0occ vcf
