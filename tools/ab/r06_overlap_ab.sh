#!/bin/bash
# Round 6: K4 beside K7 when they can share a SIMD's registers — K7 capped to 3 waves
# per SIMD (3,072 one-wave workgroups) and K4 at 128 VGPRs (AVDB_DIGEST_WAVES=4 build,
# _lib/var/libavdb_dw4.so) with one workgroup per CU.  Each arm one C4k line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r06h}; mkdir -p "$OUT"; export TMPDIR=/tmp
run() {  # name lib layout k4grid k7grid
  timeout -k 10 300 env AVDB_LIB=$2 AVDB_BENCH_LAYOUT=$3 AVDB_BENCH_K4_GRID=$4 AVDB_BENCH_K7_GRID=$5 python bench.py --steps 8 --warmup 2 --cpu-baseline off --workload c4k > "$OUT/bench_$1.log" 2>&1 || exit $?
  python - "$OUT/bench_$1.log" "$1" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["config"]["stage_ms"].items() if isinstance(v,float)})
PY
}
B=annotatedvdb_amd/_lib/libavdb_hip.so; V=annotatedvdb_amd/_lib/var/libavdb_dw4.so
run serial $B serial 0 0
run serial_k7g3072 $B serial 0 3072
run serial_dw4 $V serial 0 0
run overlap_dw4_256_3072 $V overlap 256 3072
run overlap_dw4_512_3072 $V overlap 512 3072
run overlap_dw4_256_2048 $V overlap 256 2048
run overlap_base $B overlap 0 0
run serial_end $B serial 0 0
