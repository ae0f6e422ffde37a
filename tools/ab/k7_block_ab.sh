#!/bin/bash
# K7 write-pass workgroup size A/B: the C1 / keyed GPU tests on each variant library,
# then tools/ab/k7_lib_ab.sh (in-tree 256 threads vs _lib/var variants).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_k7block
for v in $(ls annotatedvdb_amd/_lib/var/ | sed -n 's/^libavdb_\(.*\)\.so$/\1/p'); do
  AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_c1.py tests/test_gpu_c4k.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_k7block/pytest_$v.log 2>&1 || { tail -20 gpurun_out/r04_k7block/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r04_k7block/pytest_$v.log)"
done
bash tools/ab/k7_lib_ab.sh r04_k7block
