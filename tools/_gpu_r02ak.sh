# bench lines with their CPU baselines (C3, C5, C4k) on the final code
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ak
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --workload c3 > gpurun_out/ak/bench_c3.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --workload c5 > gpurun_out/ak/bench_c5.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --workload c4k > gpurun_out/ak/bench_c4k.log 2>&1
