cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_c4k.py -k "small or 0" > gpurun_out/c4k_test.log 2>&1 || { tail -30 gpurun_out/c4k_test.log; exit 1; }
tail -5 gpurun_out/c4k_test.log
timeout -k 10 300 python bench.py --workload c4k --steps 5 --warmup 2 > gpurun_out/bench_c4k.log 2>&1 || { tail -20 gpurun_out/bench_c4k.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4k -o run --output-format csv -- python3 bench.py --workload c4k --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/prof_c4k.log 2>&1
