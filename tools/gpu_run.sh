#!/bin/bash
# One GPU-box call: named steps, each under its own time limit; a crash, abort or
# timeout (124, 134, 137, 139, >= 128) stops the script.  Logs in gpurun_out/<tag>/.
#   tools/gpu_run.sh <tag> <step>...      steps: test smoke dropin c2 c3 c4k c5 c1 load vcf prof:<workload>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ]; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    test) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    test:*) step "pytest_${s#test:}" 600 python -u -m pytest "tests/${s#test:}" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    smoke) step smoke 300 python __graft_entry__.py smoke ;;
    dropin) step bench_dropin 600 python bench.py --workload dropin ;;
    c2) step bench_c2 600 python bench.py --steps 20 --warmup 3 ;;
    gloo2) step bench_gloo2 600 env AVDB_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 10 --warmup 3 ;;
    c1|c3|c4|c4k|c5|load|vcf) step "bench_$s" 600 python bench.py --steps 10 --warmup 3 --workload "$s" ;;
    ab:*) # ab:NAME=VALUE:workload  — one bench line with an env knob set (A/B)
      kv=${s#ab:}; w=${kv##*:}; kv=${kv%:*}
      step "bench_${w}_${kv//=/_}" 600 env "$kv" python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload "$w" ;;
    prof:*) w=${s#prof:}
      step "rocprof_$w" 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$w" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-baseline off --workload "$w" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo DONE
