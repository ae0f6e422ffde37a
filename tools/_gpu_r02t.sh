cd $GRAFT_REPO_ROOT
O=gpurun_out/r02t; mkdir -p $O
for ov in 0 1; do
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --cpu-baseline off --c5-overlap $ov > $O/c5_$ov.json 2> $O/c5_$ov.err || { tail -20 $O/c5_$ov.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5_$ov.json')); print($ov, d['value'], d['ms_per_step'], d['config']['stage_ms'], d['pipeline_roofline']['frac'])"
done
