cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_b_pf2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_c4k.py -m gpu -k "not c4k_shard or c4k_shard and 6" -p no:cacheprovider > gpurun_out/pytest_aj.log 2>&1 || { tail -40 gpurun_out/pytest_aj.log; exit 1; }
tail -1 gpurun_out/pytest_aj.log
for rep in 1 2; do
for lib in annotatedvdb_amd/_lib/var/libavdb_*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 200 python tools/k7_probe.py 125000000 3 || exit 1
done
done
