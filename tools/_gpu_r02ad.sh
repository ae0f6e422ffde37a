cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_b_swar2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_format.py tests/test_gpu_dropin.py tests/test_gpu_adsp.py tests/test_gpu_existing.py -m gpu -p no:cacheprovider > gpurun_out/pytest_ad.log 2>&1 || { tail -40 gpurun_out/pytest_ad.log; exit 1; }
AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_c_swar1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_format.py -m gpu -p no:cacheprovider >> gpurun_out/pytest_ad.log 2>&1 || { tail -40 gpurun_out/pytest_ad.log; exit 1; }
tail -2 gpurun_out/pytest_ad.log
for rep in 1 2; do
for lib in annotatedvdb_amd/_lib/var/libavdb_*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload load --steps 5 --warmup 2 --cpu-baseline off | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['stage_ms'])" || exit 1
done
done
