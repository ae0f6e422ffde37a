cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_c4k.py -m gpu -k "not c4k_shard or c4k_shard and 6" -p no:cacheprovider > gpurun_out/pytest_w.log 2>&1 || { tail -40 gpurun_out/pytest_w.log; exit 1; }
tail -3 gpurun_out/pytest_w.log
for lib in annotatedvdb_amd/_lib/var/libavdb_*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 200 python tools/k7_probe.py 125000000 3 || exit 1
done
