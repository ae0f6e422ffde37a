#!/bin/bash
# K0 one-pass A/B: tools/k0_onepass_probe.py with the in-tree library and each variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
echo "== in-tree"; timeout -k 10 200 python tools/k0_onepass_probe.py || exit 1
for lib in annotatedvdb_amd/_lib/var/libavdb_tok*.so; do
  echo "== $lib"
  AVDB_LIB=$lib timeout -k 10 200 python tools/k0_onepass_probe.py || exit 1
done
