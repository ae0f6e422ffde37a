cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r02b/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in w3 w4; do AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so timeout -k 10 120 python tools/k4_probe.py 25000000 6 > gpurun_out/r02b/k4_$v.json 2>&1 || exit 1; cat gpurun_out/r02b/k4_$v.json; done
timeout -k 10 300 python bench.py --workload c1 --steps 20 --warmup 3 > gpurun_out/r02b/bench_c1.json 2> gpurun_out/r02b/bench_c1.err; cat gpurun_out/r02b/bench_c1.json; tail -3 gpurun_out/r02b/bench_c1.err
