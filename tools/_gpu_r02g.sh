cd $GRAFT_REPO_ROOT
O=gpurun_out/r02g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload dropin > $O/dropin.json 2> $O/dropin.err || { tail -20 $O/dropin.err; exit 1; }
cat $O/dropin.json
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --cpu-baseline off > $O/c5.json 2> $O/c5.err || exit 1
cat $O/c5.json
