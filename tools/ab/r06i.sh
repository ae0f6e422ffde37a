#!/bin/bash
# Round 6: the pipelined one-pass keyed prep — its parity tests, then the C4k onepass line per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06i; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_onepass.py "tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle" "tests/test_gpu_c1.py::test_c1_graph_replay_vs_c_oracle" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_onepass.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_onepass.log"; [ $rc -ne 0 ] && exit $rc
bash tools/ab/r06_op_probe_run.sh r06i t1np t2np t2p t4np
