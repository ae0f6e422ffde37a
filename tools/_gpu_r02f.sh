cd $GRAFT_REPO_ROOT
O=gpurun_out/r02f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload dropin > $O/dropin.json 2> $O/dropin.err || { tail -20 $O/dropin.err; exit 1; }
cat $O/dropin.json
bash tools/k4_counters.sh r02f/k4 > /dev/null 2>&1 || exit 1
cat $O/k4/probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5prof -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --warmup 2 --cpu-baseline off > $O/c5prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c1prof -o run --output-format csv -- python3 bench.py --workload c1 --steps 10 --warmup 2 --cpu-baseline off > $O/c1prof.log 2>&1 || exit 1
grep -h avdb $O/c5prof/run_kernel_stats.csv $O/c1prof/run_kernel_stats.csv | cut -c1-160
