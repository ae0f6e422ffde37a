cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_c4k.py tests/test_gpu_adsp.py tests/test_gpu_dropin.py tests/test_gpu_format.py -m gpu -k "not c4k_shard or c4k_shard and 2" -p no:cacheprovider > gpurun_out/pytest_an.log 2>&1 || { tail -40 gpurun_out/pytest_an.log; exit 1; }
tail -1 gpurun_out/pytest_an.log
for rep in 1 2; do
for lib in annotatedvdb_amd/_lib/var/libavdb_*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload c4k --steps 5 --warmup 2 --cpu-baseline off | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['stage_ms'])" || exit 1
done
done
