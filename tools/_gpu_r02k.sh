cd $GRAFT_REPO_ROOT
O=gpurun_out/r02k; mkdir -p $O
export TMPDIR=/tmp
for v in s0 s1_disp s2_freq s4_bin s8_pk s15_all; do
  echo "== $v"
  AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so timeout -k 10 150 python tools/k5_probe.py 8388608 2>&1 | grep -v checksum | tail -2 || exit 1
done
