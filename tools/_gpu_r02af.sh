cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
for lib in annotatedvdb_amd/_lib/var/libavdb_*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 300 python bench.py --workload load --steps 5 --warmup 2 --cpu-baseline off | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['stage_ms'])" || exit 1
done
done
