cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dropin.py tests/test_gpu_format.py tests/test_gpu_shard.py tests/test_gpu_adsp.py tests/test_gpu_existing.py tests/test_gpu_c4k.py -k "not c4k_shard" -m gpu -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 1; }
tail -2 gpurun_out/pytest_ab.log
for w in vcf load; do
timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --cpu-baseline off | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$w', d['value'], d['config']['stage_ms'])" || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_vcf -o run --output-format csv -- python3 bench.py --workload vcf --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/ab_vcf.log 2>&1
python3 tools/prof_summary.py stats gpurun_out/ab_vcf
