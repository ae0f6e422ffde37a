cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c1.py tests/test_gpu_c4k.py -k "k4 or c5 or k7 or c4k_small or c4k_shard and 4" -m gpu -p no:cacheprovider > gpurun_out/pytest_ag.log 2>&1 || { tail -40 gpurun_out/pytest_ag.log; exit 1; }
tail -2 gpurun_out/pytest_ag.log
for rep in 1 2; do
for lib in annotatedvdb_amd/_lib/var/libavdb_[ab]_*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload load --steps 5 --warmup 2 --cpu-baseline off | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['stage_ms'])" || exit 1
done
for lib in annotatedvdb_amd/_lib/var/libavdb_[wx]_*.so; do
  for w in c5 c4k; do
  echo "== $lib $w"
  AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --cpu-baseline off | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['stage_ms'])" || exit 1
  done
done
done
