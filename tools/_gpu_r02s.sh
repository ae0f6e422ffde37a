cd $GRAFT_REPO_ROOT
for u in 1 2 4; do for b in 2 4 8; do
  AVDB_K2_UNROLL=$u AVDB_K2_BLOCKS_PER_CU=$b timeout -k 10 120 python tools/k2_probe.py 25000000 10 2>&1 | tail -1 || exit 1
done; done
