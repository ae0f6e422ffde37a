cd $GRAFT_REPO_ROOT
O=gpurun_out/r02p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
cat $O/smoke.log
bash tools/gpu_prof_workload.sh load 5 || exit 1
mkdir -p $O/load && cp -r gpurun_out/load/* $O/load/
python3 tools/prof_summary.py stats $O/load/prof | head -30
