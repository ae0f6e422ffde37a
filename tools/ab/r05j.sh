#!/bin/bash
# Round 5: K0 tab bitmap + SWAR INFO/ID scans — the tokenizer / format tests on the
# in-tree and each variant library, then K0 kernel times per library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05j}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for lib in annotatedvdb_amd/_lib/libavdb_hip.so $(ls annotatedvdb_amd/_lib/var/libavdb_*.so 2>/dev/null); do
  v=$(basename "$lib" .so)
  AVDB_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_format.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.log" 2>&1 || { tail -30 "$OUT/pytest_$v.log"; exit 1; }
  echo "$v $(tail -1 $OUT/pytest_$v.log)"
done
bash tools/k0_attr.sh "$T/attr" || exit 1
