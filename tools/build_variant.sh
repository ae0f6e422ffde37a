#!/bin/bash
# Build a variant of libavdb_hip.so with extra compile flags for on-device A/B:
#   tools/build_variant.sh NAME [-DFOO=1 ...]  ->  annotatedvdb_amd/_lib/var/libavdb_NAME.so
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p annotatedvdb_amd/_lib/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -I include "$@" \
  -o annotatedvdb_amd/_lib/var/libavdb_$name.so annotatedvdb_amd/csrc/*.hip
