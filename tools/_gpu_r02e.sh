cd $GRAFT_REPO_ROOT
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/pytest.log | grep -v PASSED | head -20; tail -3 $O/pytest.log; exit $rc
