#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer run of libavdb_hip.so
# (SURVEY.md §5 "Race detection / sanitizers: ASan on the C++ host lib").
# Build container only: the host half of every translation unit is instrumented
# (each -fsanitize= sits after -Xarch_host; device code is untouched), then the CPU
# test suite runs against that library with the ASan runtime preloaded.  It covers
# context creation and argument checks, host formatting, the RCCL argument checks,
# and the per-call host entries (K1h / K8h / K5h) on the golden fixtures.
#   tools/host_sanitizers.sh [pytest args]      log: profiles/r03_host_sanitizers.log
set -o pipefail
cd "$(dirname "$0")/.."
LIB=annotatedvdb_amd/_lib/libavdb_hip_san.so
python3 - <<'PY' || exit 1
from annotatedvdb_amd import build_native as b
san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer", "-g"]
b.build(force=False, out=b.os.path.join(b.OUT_DIR, "libavdb_hip_san.so"), flags=san, objdir="obj_san",
        link_flags=["-fsanitize=address,undefined", "-shared-libsan"])
PY
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
export AVDB_LIB=$PWD/$LIB
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
{ echo "# $(date -u +%FT%TZ) $LIB: $(nm -D "$LIB" | grep -c '__asan_report\|__ubsan_handle') ASan/UBSan hooks; runtime $RT"
  LD_PRELOAD=$RT python3 -c "import ctypes,os; ctypes.CDLL(os.environ['AVDB_LIB']); print('# loaded', os.environ['AVDB_LIB'])"
} > profiles/r03_host_sanitizers.log
LD_PRELOAD=$RT python3 -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@" 2>&1 | tee -a profiles/r03_host_sanitizers.log
