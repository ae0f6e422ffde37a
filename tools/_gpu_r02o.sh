cd $GRAFT_REPO_ROOT
O=gpurun_out/r02o; mkdir -p $O
export TMPDIR=/tmp
true

for v in y_nofast; do
  echo "== $v"
  AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so timeout -k 10 150 python tools/k5_probe.py 8388608 2>&1 | tail -3 || exit 1
done
echo "== default"
timeout -k 10 150 python tools/k5_probe.py 8388608 2>&1 | tail -3 || exit 1
