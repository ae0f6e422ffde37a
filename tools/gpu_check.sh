#!/bin/bash
# GPU-box driver for one measurement round.  Every GPU step has its own time
# limit; a crash/abort/timeout (124,134,137,139) stops the script, a plain test
# failure (1) does not stop the measurement steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -ge 128 ] && return 0; return 1; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
  step smoke 300 python __graft_entry__.py smoke
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench_c2 600 python bench.py --steps 20 --warmup 3
  step bench_c3 600 python bench.py --steps 20 --warmup 3 --workload c3 --cpu-baseline off
  step bench_c5 600 python bench.py --steps 5 --warmup 2 --workload c5
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  step rocprof_c2 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-baseline off
  step pmc_fetch_c2 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-baseline off
  step pmc_write_c2 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-baseline off
fi
echo DONE
