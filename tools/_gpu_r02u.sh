cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "not c4k_shard and not one_billion" -p no:cacheprovider > gpurun_out/pytest_u.log 2>&1 || { tail -40 gpurun_out/pytest_u.log; exit 1; }
tail -3 gpurun_out/pytest_u.log
timeout -k 10 200 python tools/k7_probe.py 125000000 3 > gpurun_out/k7_probe_u.json 2>&1; cat gpurun_out/k7_probe_u.json
timeout -k 10 300 python bench.py --workload c4k --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/bench_c4k_u.log 2>&1
timeout -k 10 300 python bench.py --workload load --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/bench_load_u.log 2>&1
timeout -k 10 300 python bench.py --workload c1 --steps 20 --warmup 3 --cpu-baseline off > gpurun_out/bench_c1_u.log 2>&1
grep -h '^{' gpurun_out/bench_*_u.log | python3 -c "import sys,json; [print(d['config']['workload'][:20], d['value'], d['ms_per_step'], d['config']['stage_ms']) for d in map(json.loads, sys.stdin)]"
