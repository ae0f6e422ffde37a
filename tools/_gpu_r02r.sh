cd $GRAFT_REPO_ROOT
O=gpurun_out/r02r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 > $O/torchrun_c2.json 2> $O/torchrun_c2.err || { tail -20 $O/torchrun_c2.err; exit 1; }
cat $O/torchrun_c2.json
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline']), d['config']['stage_ms'])"
python3 - <<'PY' > $O/mkvcf.log 2>&1 || exit 1
import sys; sys.path.insert(0, '.')
from annotatedvdb_amd import synth
open('/tmp/x.vcf', 'wb').write(synth.vcf_text(200000, seed=3))
PY
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 -m annotatedvdb_amd.load_vcf_file --fileName /tmp/x.vcf --outDir $O/loadout > $O/driver.log 2>&1 || { tail -20 $O/driver.log; exit 1; }
tail -3 $O/driver.log; ls -la $O/loadout
