cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/fork
mkdir -p $OUT
for rep in 1 2; do for f in 1 0; do for w in c1 c4k; do
  AVDB_BENCH_FORK=$f timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-baseline off > $OUT/${w}_f${f}_$rep.log 2>&1 || { tail -20 $OUT/${w}_f${f}_$rep.log; exit 1; }
  python3 -c "
import json,sys
l=[x for x in open('$OUT/${w}_f${f}_$rep.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$w fork=$f rep=$rep', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), d['config'].get('stage_ms'))"
done; done; done
bash tools/k7_counters.sh r04k7b > $OUT/k7c.log 2>&1 && echo k7counters ok
