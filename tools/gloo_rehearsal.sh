#!/bin/bash
# N>1 bench path rehearsed on a 1-GPU box: 2 ranks over gloo sharing the card
# (RCCL refuses two ranks on one device).  tools/gloo_rehearsal.sh TAG WORKLOAD...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
OUT=gpurun_out/$T
mkdir -p "$OUT"
for w in "$@"; do
  AVDB_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --workload "$w" \
    > "$OUT/n2_$w.log" 2>&1 || { echo "FAILED $w"; tail -20 "$OUT/n2_$w.log"; exit 1; }
  grep '^{' "$OUT/n2_$w.log" | cut -c1-400
done
