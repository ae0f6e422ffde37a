#!/bin/bash
# Register / scratch / LDS use of the K5 kernels for given sink options.
# Usage: tools/k5_regs.sh "-DAVDB_K5_SINK=1 -DAVDB_K5_WAVES=3" ...
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cd "$T" || exit 1
for opts in "$@"; do
  echo "== $opts"
  # shellcheck disable=SC2086
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -I "$ROOT/include" $opts -c "$ROOT/annotatedvdb_amd/csrc/avdb_format_write.hip" \
    --save-temps -o f.o 2>&1 | grep -A3 error
  python3 - <<'EOF'
import re
s = open("avdb_format_write-hip-amdgcn-amd-amdhsa-gfx950.s").read()
for b in re.split(r"\n  - ", s):
    n = re.search(r"\.name:\s+(\S+)", b)
    if n and ("format" in n.group(1) or "display" in n.group(1)):
        g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", b) or [None, None])[1]
        print("  %-45s vgpr %s lds %s scratch %s" % (n.group(1)[:45], g("vgpr_count"),
              g("group_segment_fixed_size"), g("private_segment_fixed_size")))
EOF
done
rm -rf "$T"
