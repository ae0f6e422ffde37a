cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload dropin > $O/dropin.json 2> $O/dropin.err || { tail -20 $O/dropin.err; exit 1; }
cat $O/dropin.json
timeout -k 10 300 python bench.py --workload c1 --steps 20 --warmup 3 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
cat $O/c1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c1prof -o run --output-format csv -- python3 bench.py --workload c1 --steps 10 --warmup 2 --cpu-baseline off > $O/c1prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/loadprof -o run --output-format csv -- python3 bench.py --workload load --steps 3 --warmup 1 --cpu-baseline off > $O/loadprof.log 2>&1 || exit 1
grep -h avdb $O/c1prof/run_kernel_stats.csv $O/loadprof/run_kernel_stats.csv | cut -c1-160
