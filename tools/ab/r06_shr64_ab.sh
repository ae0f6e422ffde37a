#!/bin/bash
# Round 6: K4 with the message schedule's 64-bit shifts (sigma0 >> 7, sigma1 >> 6) as one v_lshrrev_b64
# instead of a funnel shift + a 32-bit shift, vs base (same flags): digest tests on the variant, then the C5 and C4k lines alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06_shr64; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in shr64; do
  timeout -k 10 600 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python -u -m pytest "tests/test_gpu_parity.py::test_c5_full_size_vs_c_oracle" "tests/test_gpu_parity.py::test_prep_step_equals_plain_chain" "tests/test_gpu_c4k.py::test_c4k_small_vs_c_oracle" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.log" 2>&1
  rc=$?; echo "$v: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
for v in base shr64; do
  for wl in c5 c4k; do
    timeout -k 10 300 env AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload $wl > "$OUT/bench_${wl}_$v.log" 2>&1 || exit $?
    python - "$OUT/bench_${wl}_$v.log" "$wl $v" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,3) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
  done
done; done
