#!/bin/bash
# Round 5: K4 beside a grid-capped K7 (overlap layout) and the split K5 write pass, A/B on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05c
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py::test_grid_knobs_parity tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle tests/test_gpu_format.py tests/test_gpu_tokenize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05c/pytest.log 2>&1 || { tail -30 gpurun_out/r05c/pytest.log; exit 1; }
tail -2 gpurun_out/r05c/pytest.log
AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_k5split.so timeout -k 10 600 python -u -m pytest tests/test_gpu_format.py tests/test_integration_recipe.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05c/pytest_k5split.log 2>&1 || { tail -30 gpurun_out/r05c/pytest_k5split.log; exit 1; }
tail -2 gpurun_out/r05c/pytest_k5split.log
bash tools/ab/c4k_layout_ab.sh r05c_ab serial:0:0 overlap:256:2048 overlap:512:1024 overlap:256:3072 serial:0:2048 serial:0:3072 serial:0:0 || exit 1
for lib in annotatedvdb_amd/_lib/libavdb_hip.so annotatedvdb_amd/_lib/var/libavdb_k5split.so annotatedvdb_amd/_lib/libavdb_hip.so annotatedvdb_amd/_lib/var/libavdb_k5split.so; do
  AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload load --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/r05c/load_$(basename $lib .so).json 2>gpurun_out/r05c/load.err || { tail -5 gpurun_out/r05c/load.err; exit 1; }
  python -c "
import json,sys; d=json.loads(open('gpurun_out/r05c/load_$(basename $lib .so).json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], d['config']['stage_ms'])"
done
echo DONE
