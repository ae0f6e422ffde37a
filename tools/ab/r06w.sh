#!/bin/bash
# Round 6: K4 with the chaining value and the location characters parked in the lane's LDS slot
# across the rounds (152 VGPRs at 3 waves/SIMD; 128 with 84 B of spills at 4) vs base (166 VGPRs):
# digest tests on each variant, then the C5 and C4k lines alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06w; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in parked parked4; do
  timeout -k 10 600 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python -u -m pytest "tests/test_gpu_parity.py::test_c5_full_size_vs_c_oracle" "tests/test_gpu_parity.py::test_prep_step_equals_plain_chain" "tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.log" 2>&1
  rc=$?; echo "$v: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
for v in base parked parked4; do
  for wl in c5 c4k; do
    timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload $wl > "$OUT/bench_${wl}_$v.log" 2>&1 || exit $?
    python - "$OUT/bench_${wl}_$v.log" "$wl $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,3) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
  done
done; done
