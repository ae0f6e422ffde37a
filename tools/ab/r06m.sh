#!/bin/bash
# Round 6: Out::finish tail as <= 3 stores (4/2/1 bytes) instead of a byte loop: K5 / K0 / K8
# tests, then load + vcf lines with the HEAD library (AVDB_LIB=_lib/var/libavdb_base.so) and the new one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06m; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_format.py tests/test_gpu_tokenize.py tests/test_gpu_dropin.py tests/test_gpu_adsp.py tests/test_gpu_existing.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for lib in base new; do
  if [ $lib = base ]; then L=annotatedvdb_amd/_lib/var/libavdb_base.so; else L=annotatedvdb_amd/_lib/libavdb_hip.so; fi
  for wl in load vcf; do
    timeout -k 10 300 env AVDB_LIB=$L python bench.py --steps 10 --warmup 3 --cpu-baseline off --workload $wl > "$OUT/bench_${wl}_$lib.log" 2>&1 || exit $?
    python - "$OUT/bench_${wl}_$lib.log" "$wl $lib" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],4), {k: round(v,3) for k,v in d["config"].get("stage_ms",{}).items() if isinstance(v,float)})
PY
  done
done; done
