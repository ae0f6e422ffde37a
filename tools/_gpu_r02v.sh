cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_c4k.py tests/test_gpu_format.py tests/test_gpu_dropin.py tests/test_gpu_adsp.py -m gpu -k "not c4k_shard or c4k_shard and 3" -p no:cacheprovider > gpurun_out/pytest_v.log 2>&1 || { tail -40 gpurun_out/pytest_v.log; exit 1; }
tail -3 gpurun_out/pytest_v.log
for lib in annotatedvdb_amd/_lib/var/libavdb_*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 200 python tools/k7_probe.py 125000000 3 || exit 1
  AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload load --steps 5 --warmup 2 --cpu-baseline off | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['stage_ms'])" || exit 1
done
