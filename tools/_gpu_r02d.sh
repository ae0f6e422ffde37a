cd $GRAFT_REPO_ROOT
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "k4 or c5_full" > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in u0 u1; do AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so timeout -k 10 120 python tools/k4_probe.py 25000000 6 > $O/k4_$v.json 2>&1 || exit 1; cat $O/k4_$v.json; done
AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_u1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "k4 or c5_full" > $O/pytest_u1.log 2>&1; tail -2 $O/pytest_u1.log
