cd $GRAFT_REPO_ROOT
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c1 --steps 20 --warmup 3 > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
cat $O/bench_c1.json
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --cpu-baseline off > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
cat $O/bench_c5.json
AVDB_K2_VECTOR=0 timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --cpu-baseline off > $O/bench_c5_k2scalar.json 2>&1 || exit 1
bash tools/k4_counters.sh r02c/k4 > /dev/null 2>&1 || exit 1
cat $O/k4/probe.json
