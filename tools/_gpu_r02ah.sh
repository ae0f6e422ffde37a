# Final round-2 check of the committed tree: GPU suite, smoke, every bench line, kernel stats, load/vcf traffic.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ah; mkdir -p $O
step() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -2 $O/$n.log; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
step pytest 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider
step smoke 200 python __graft_entry__.py smoke
step bench_c2 300 python bench.py --steps 20 --warmup 5
step bench_c3 300 python bench.py --steps 20 --warmup 3 --workload c3 --cpu-baseline off
step bench_c1 300 python bench.py --steps 20 --warmup 3 --workload c1
step bench_c5 300 python bench.py --steps 5 --warmup 2 --workload c5 --cpu-baseline off
step bench_c4k 300 python bench.py --steps 5 --warmup 2 --workload c4k --cpu-baseline off
step bench_load 300 python bench.py --steps 5 --warmup 2 --workload load
step bench_vcf 300 python bench.py --steps 5 --warmup 2 --workload vcf --cpu-baseline off
step bench_dropin 300 python bench.py --workload dropin
step prof_load 300 rocprofv3 --kernel-trace --stats -d $O/prof_load -o run --output-format csv -- python3 bench.py --workload load --steps 3 --warmup 1 --cpu-baseline off
step prof_c4k 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4k -o run --output-format csv -- python3 bench.py --workload c4k --steps 3 --warmup 1 --cpu-baseline off
step prof_c2 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off


step traffic_load 400 bash tools/traffic_counters.sh load ah/traffic_load
step traffic_vcf 400 bash tools/traffic_counters.sh vcf ah/traffic_vcf
echo DONE
