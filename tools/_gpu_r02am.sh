# Final check of the exact committed library: full GPU suite, smoke, default bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/am
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/am/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/am/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/am/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/am/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/am/bench_c2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --workload c4k --cpu-baseline off > gpurun_out/am/bench_c4k.log 2>&1
